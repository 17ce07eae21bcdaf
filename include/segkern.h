/*
 * segkern.h -- C-ABI of the MI355X (gfx950) segmentation training path.
 *
 * This library replaces the TensorFlow 1.x kernels that the reference's hot
 * path executes inside `sess.run(train_step)`.  Each entry
 * point names the TF op / reference call site it stands in for.  The Python
 * host layer (`semanticsegmentation_tensorflow_amd/layers.py`) mirrors the
 * reference's layer builders on top of these calls.
 *
 * Conventions
 *  - Plain C types only: device pointers as `void*`/`float*`, sizes as int /
 *    size_t, the HIP stream as `void*` (a `hipStream_t`; NULL = null stream).
 *  - The caller owns every buffer, including workspaces; the library never
 *    allocates on the hot path.  `seg_*_workspace` reports the bytes needed.
 *  - Activations are NHWC; the channel dimension is padded to a multiple of
 *    8 (`C`, `K` in the descriptors) and the padding channels hold zeros.
 *    `ldx`/`ldy` (elements between consecutive pixels) allow channel-slice
 *    views, e.g. a layer writing into a concat buffer.
 *  - Every function returns 0 on success or a SEG_E* code; shapes are
 *    validated with TF's rules (incl. the conv2d_transpose shape rule).
 *    `seg_status_string()` turns a code into text.
 */
#ifndef SEGKERN_H
#define SEGKERN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SEG_F16: IEEE half storage with fp32 accumulation (v_mfma_f32_16x16x32_f16),
 * config C5's "fp16 with fp32 accum" (BASELINE.json configs[4]); runs on the
 * generic implicit-GEMM kernels (the bf16-specialised halo / 256x256 paths are
 * bf16 only). */
enum seg_dtype { SEG_F32 = 0, SEG_BF16 = 1, SEG_F16 = 2 };

enum seg_status {
    SEG_OK = 0,
    SEG_EINVAL = 1,      /* bad argument (null pointer, bad dtype, ...)        */
    SEG_ESHAPE = 2,      /* TF shape rule violated (InvalidArgumentError)      */
    SEG_EALIGN = 3,      /* channel count / stride not a multiple of 8         */
    SEG_EWORKSPACE = 4,  /* workspace too small                                */
    SEG_ELAUNCH = 5      /* HIP launch failure                                 */
};

/* Convolution descriptor.  For Conv2D: input [N,H,W,C], filter [R,S,C,K]
 * (HWIO), output [N,OH,OW,K].  For conv2d_transpose: input [N,H,W,C],
 * filter [R,S,K,C] (TF's [kh,kw,out,in]), output [N,OH,OW,K].
 * C and K are padded channel counts (multiples of 8); c_valid/k_valid are
 * the real counts used to address the fp32 master filter. */
typedef struct seg_conv_desc {
    int N, H, W, C;
    int OH, OW, K;
    int R, S;
    int stride_h, stride_w;
    int dil_h, dil_w;
    int pad_top, pad_bottom, pad_left, pad_right;
    int ldx, ldy;          /* pixel strides (elements) of input / output   */
    int c_valid, k_valid;  /* unpadded channel counts                      */
    int dtype;             /* enum seg_dtype of activations and packed W   */
} seg_conv_desc;

/* Epilogue fused into a convolution's output write:
 *   v = acc * scale[k] + shift[k] (+ bias[k]);  v = relu(v) if relu;
 *   v = v / keep_prob * floor(keep_prob + U) if keep_prob < 1 (TF1 dropout);
 *   v += residual[pixel, k]  (tf.add skip fusion);
 *   v = relu_mask[pixel, k] > 0 ? v * mask_scale : 0   (if relu_mask)
 * The last step is ReluGrad (x dropout's 1/keep_prob) of the layer that
 * produced this op's input, fused into Conv2DBackpropInput / the tconv input
 * gradient: relu_mask is that layer's (post-ReLU/dropout) output, laid out
 * like the gradient being written (ld_relu_mask 0 = same stride).           */
typedef struct seg_epilogue {
    const float* bias;
    const float* scale;
    const float* shift;
    const void* residual;
    int ld_residual;
    int relu;
    float keep_prob;
    uint64_t seed;
    const void* relu_mask;
    int ld_relu_mask;
    float mask_scale;
} seg_epilogue;

/* ---- descriptor helpers ------------------------------------------------ */
/* Fill a Conv2D descriptor with TF SAME/VALID padding (padding: 0=SAME,
 * 1=VALID).  Mirrors tf.nn.conv2d's shape function (Network/model/FCN.py:130). */
int seg_conv_desc_init(seg_conv_desc* d, int N, int H, int W, int C, int K, int R, int S,
                       int stride, int dilation, int padding, int dtype);
/* Fill a conv2d_transpose descriptor from the requested output shape; fails
 * with SEG_ESHAPE unless ceil(out/stride) == in (SAME) -- TF's rule
 * (Network/model/FCN.py:155, :106). */
int seg_tconv_desc_init(seg_conv_desc* d, int N, int H, int W, int C, int OH, int OW, int K,
                        int R, int S, int stride, int padding, int dtype);

/* ---- Conv2D (Network/model/FCN.py:130-134, Network/utils/utils.py:182) --- */
/* w_krsc: packed filter [K][R][S][C] in `dtype` (seg_pack_filter mode 0). */
int seg_conv2d_fwd(const seg_conv_desc* d, const void* x, const void* w_krsc,
                   const seg_epilogue* epi, void* y, void* ws, size_t ws_bytes, void* stream);
/* Conv2D from the HWIO filter copy w_hwio [R][S][C][K] (seg_pack_filter mode
 * 1, the copy seg_conv2d_bwd_data reads): same results as seg_conv2d_fwd on
 * the KRSC copy, so a weight needs one packed copy (FCN conv6 / conv7,
 * Network/model/FCN.py:78-83: the fused filter-gradient + Adam launch then
 * writes no KRSC copy).  16-bit dtypes, C a multiple of 64, and a conv
 * whose launch runs igemm_nt3 whole: seg_conv2d_fwd_hwio_ok(d) == 1,
 * SEG_EINVAL otherwise. */
int seg_conv2d_fwd_hwio_ok(const seg_conv_desc* d);
int seg_conv2d_fwd_hwio(const seg_conv_desc* d, const void* x, const void* w_hwio,
                        const seg_epilogue* epi, void* y, void* ws, size_t ws_bytes, void* stream);
/* Conv2D + bias + ReLU + MaxPool(2x2, stride 2) in one launch: conv_layer
 * followed by max_pool (Network/model/FCN.py:56-57, :63, :69, :75, :81 with
 * :158-160).  The conv output is never written: y_pool gets the pooled map
 * [N][OH/2][OW/2] (row stride ld_pool), idx (may be NULL) the MaxPool
 * switches in seg_maxpool2x2_fwd_argmax's encoding (row stride ld_idx bytes),
 * both equal bit for bit to seg_conv2d_fwd + seg_maxpool2x2_fwd_argmax.
 * 16-bit dtypes, even OH / OW, epilogue bias + ReLU only (no scale / shift /
 * residual / mask / dropout), and a launch whose kernel has the pooled
 * epilogue: seg_conv2d_fwd_pool_ok(d) == 1, SEG_EINVAL otherwise. */
int seg_conv2d_fwd_pool_ok(const seg_conv_desc* d);
int seg_conv2d_fwd_pool(const seg_conv_desc* d, const void* x, const void* w_krsc,
                        const seg_epilogue* epi, void* y_pool, int ld_pool, void* idx, int ld_idx,
                        void* ws, size_t ws_bytes, void* stream);
/* Conv2DBackpropInput.  w_hwio: packed filter [R][S][C][K] in `dtype`
 * (seg_pack_filter mode 1).  dx may be a channel-slice view (ldx). */
/* Conv2DBackpropInput + MaxPoolGrad in one launch, for the conv that
 * consumes a 2x2 / 2 MaxPool's output (Network/model/FCN.py:63-69 conv2_1 /
 * conv3_1 after pool1 / pool2, with :158-160): the pooled input gradient is
 * never written; dx_full [N][2H][2W] (row stride ld_full, H x W = d's input)
 * gets it routed by idx (seg_maxpool2x2_fwd_argmax switches, row stride
 * ld_idx bytes; zero where relu != 0 and the switch's bit 2 is clear: the
 * ReluGrad of the post-ReLU pool input) and zeros at the other three window
 * elements -- bit for bit seg_conv2d_bwd_data + seg_maxpool2x2_bwd_argmax.
 * epi: NULL, or a residual only (the pooled gradient of the pool's other
 * consumers, added before routing).  16-bit dtypes, stride 1, a launch whose
 * kernel has the epilogue: seg_conv2d_bwd_data_unpool_ok(d) == 1, SEG_EINVAL
 * otherwise.  Replaces the pair nn_ops MaxPoolGrad + Conv2DBackpropInput of
 * tf.train.AdamOptimizer.minimize (Network/model/FCN.py:338-340). */
int seg_conv2d_bwd_data_unpool_ok(const seg_conv_desc* d);
int seg_conv2d_bwd_data_unpool(const seg_conv_desc* d, const void* dy, const void* w_hwio,
                               const seg_epilogue* epi, const void* idx, int ld_idx, int relu,
                               void* dx_full, int ld_full, void* ws, size_t ws_bytes, void* stream);
/* A-operand prologue: the conv reads relu(x * gamma / sqrt(1 + eps) + beta)
 * in place of x (frozen-statistics tf.layers.batch_normalization + ReLU
 * feeding the conv, Network/model/FCDenseNet.py:25-28 and :39-41,
 * Network/utils/utils.py:300-303) without the BN output ever being written:
 * zero-padded taps stay zero, as TF pads the BN output.  gamma / beta: fp32
 * [c_valid]; relu 0/1. */
typedef struct seg_prologue {
    const float* gamma;
    const float* beta;
    float eps;
    int relu;
} seg_prologue;
/* Conv2D of relu(BN(x)) (tf.nn.conv2d on the Batch_Normalization + ReLU
 * output, utils.py:182 / :300-303) with the epilogue of seg_conv2d_fwd. */
int seg_conv2d_fwd_pro(const seg_conv_desc* d, const void* x, const seg_prologue* pro, const void* w,
                       const seg_epilogue* epi, void* y, void* ws, size_t ws_bytes, void* stream);
/* Conv2D (pro optional: NULL = seg_conv2d_fwd) whose output y also feeds a
 * frozen Batch_Normalization (+ReLU) -- FC-DenseNet's bottleneck conv1 ->
 * dropout -> BN -> ReLU (Network/model/FCDenseNet.py:28-31, utils.py:300-303):
 * writes y as seg_conv2d_fwd[_pro] and y2 = relu(y * gamma2 / sqrt(1 + eps2)
 * + beta2) from the stored y, bit-identical to seg_bn_relu_fwd(y, y2, ...),
 * so the BN forward pass never re-reads y.  Also DeepLab's ASPP conv -> BN
 * -> ReLU (Network/utils/utils.py:186-229), where the split-K reducer after
 * igemm_nt3 writes y2.  ld_y2: y2's pixel stride (elements, multiple of 8).
 * SEG_EINVAL when the kernel the conv runs on has no second output (query:
 * seg_conv2d_fwd_bn2_ok). */
int seg_conv2d_fwd_bn2(const seg_conv_desc* d, const void* x, const seg_prologue* pro, const void* w,
                       const seg_epilogue* epi, void* y, void* y2, int ld_y2, const float* gamma2,
                       const float* beta2, float eps2, int relu2, void* ws, size_t ws_bytes, void* stream);
int seg_conv2d_fwd_bn2_ok(const seg_conv_desc* d, int with_prologue);
/* Conv2DBackpropFilter with input relu(BN(x)) recomputed from x. */
int seg_conv2d_bwd_filter_pro(const seg_conv_desc* d, const void* x, const seg_prologue* pro,
                              const void* dy, float* dw, float* dbias, void* ws, size_t ws_bytes,
                              void* stream);
/* Conv2DBackpropInput of a stride-1 conv over relu(BN(x)), carried through
 * the BatchNorm(+ReLU) backward in the same launch (FCDenseNet.py:25-33
 * backward): the ReLU mask is re-derived from x, dx = dL/dx of the BN input,
 * dgamma / dbeta (fp32, overwritten) from per-tile column sums.  Applies to
 * 1x1 convs (the BN folded into the forward's operand prologue; accumulate
 * != 0 adds into dx, e.g. a slice of a shared concat gradient) and to 3x3
 * convs with 16 output channels (FC-DenseNet's growth convs; keep_prob < 1
 * then also applies the gradient of the TF1 dropout fused into the epilogue
 * of the conv that produced x, counter pixel * C + c; no accumulate).
 * bf16 / fp16 only; workspace from seg_conv_bwd_data_bn_workspace, which
 * returns 0 when the fused path does not apply (then seg_conv2d_bwd_data +
 * seg_bn_relu_bwd / seg_bn_relu_dropout_bwd). */
typedef struct seg_bn_bwd {
    const void* x;          /* BN input, pixel stride ldx */
    int ldx;
    const float* gamma;
    const float* beta;
    float eps;
    int relu;
    int accumulate;
    float* dgamma;
    float* dbeta;
    float keep_prob;        /* 3x3 form: dropout before the BN (>= 1 or 0: none) */
    uint64_t seed;
} seg_bn_bwd;
size_t seg_conv_bwd_data_bn_workspace(const seg_conv_desc* d);
/* The same launch with the dgamma / dbeta reduction left to the caller:
 * the per-tile partial column sums go to `part` ([seg_conv_bwd_data_bn_part_rows(d)]
 * rows of 2*C fp32: C dgamma partials (unscaled) then C dbeta partials); bn->dgamma /
 * dbeta are not written.  part_rows must equal seg_conv_bwd_data_bn_part_rows(d)
 * (the row count a finish plan was made for; SEG_EWORKSPACE otherwise).  Finish
 * many of them at once with seg_bn_grad_finish_batch (a step's BN backward sums
 * in two launches). */
long seg_conv_bwd_data_bn_part_rows(const seg_conv_desc* d);
int seg_conv2d_bwd_data_bn_part(const seg_conv_desc* d, const void* dy, const void* w_hwio, const seg_bn_bwd* bn,
                                void* dx, float* part, long part_rows, void* stream);
typedef struct seg_bn_finish_segment {
    const float* part;      /* [nrows][2*C] partial rows */
    int nrows, C, cv;
    float inv;              /* 1 / sqrt(1 + eps): dgamma = inv * sum */
    float* dgamma;
    float* dbeta;
    /* filled by seg_bn_finish_batch_plan */
    float* scratch;
    int a_blk0, a_nblk, b_blk0, b_nblk;
} seg_bn_finish_segment;
/* Host-side plan: fills the launch offsets and scratch pointers of segs[]
 * (scratch carved from `scratch`, may be NULL to size it) and returns the
 * scratch bytes; *a_blocks / *b_blocks: the two launches' grids. */
size_t seg_bn_finish_batch_plan(seg_bn_finish_segment* segs, int nsegs, float* scratch, int* a_blocks,
                                int* b_blocks);
/* dgamma / dbeta of every segment (dev_segs: the planned array in device
 * memory), bit-identical to seg_conv2d_bwd_data_bn's own finish. */
int seg_bn_grad_finish_batch(const seg_bn_finish_segment* dev_segs, int nsegs, int a_blocks, int b_blocks,
                             void* stream);
int seg_conv2d_bwd_data_bn(const seg_conv_desc* d, const void* dy, const void* w_hwio, const seg_bn_bwd* bn,
                           void* dx, void* ws, size_t ws_bytes, void* stream);
int seg_conv2d_bwd_data(const seg_conv_desc* d, const void* dy, const void* w_hwio,
                        const seg_epilogue* epi, void* dx, void* ws, size_t ws_bytes, void* stream);
/* The ReluGrad mask as bits (round 6).  seg_conv2d_fwd_relu_bits = seg_conv2d_fwd
 * that also writes the ReLU mask of the stored y: bit k & 7 of
 * bits[pixel * ld_bits + k / 8] = (y[pixel][k] > 0), pixels dense over the
 * batch, ld_bits >= K / 8 bytes (K = 64: a multiple of 8, bits 8-byte
 * aligned -- one 8-byte store per pixel).  seg_conv2d_bwd_data_bits = seg_conv2d_bwd_data
 * whose ReluGrad mask (epi->relu_mask, which must be NULL here; epi->mask_scale
 * applies) is read from such bits, 8-byte aligned: dx bit for bit the same as
 * with the 16-bit map.  FCN / VGG conv1_1 -> conv1_2 (Network/model/FCN.py:55-56):
 * conv1_2's input gradient reads 8 bytes per pixel instead of conv1_1's
 * 128-byte output row.  Only the kernels with these epilogues take them (the
 * first-layer C <= 8 forward; the 64 -> 64 3x3 input gradient): the _ok
 * queries, SEG_EINVAL otherwise. */
int seg_conv2d_fwd_relu_bits_ok(const seg_conv_desc* d);
int seg_conv2d_fwd_relu_bits(const seg_conv_desc* d, const void* x, const void* w_krsc, const seg_epilogue* epi,
                             void* y, void* bits, int ld_bits, void* stream);
int seg_conv2d_bwd_data_bits_ok(const seg_conv_desc* d);
int seg_conv2d_bwd_data_bits(const seg_conv_desc* d, const void* dy, const void* w_hwio, const seg_epilogue* epi,
                             const void* bits, int ld_bits, void* dx, void* ws, size_t ws_bytes, void* stream);
/* Conv2DBackpropFilter: dw_f32 is the fp32 master-gradient layout
 * [R][S][c_valid][k_valid]; written (not accumulated).  dbias (optional):
 * BiasAddGrad of the same dy, dbias[k] = sum over pixels of dy[p][k]
 * (k < k_valid) -- summed inside the filter-gradient kernel when it can. */
int seg_conv2d_bwd_filter(const seg_conv_desc* d, const void* x, const void* dy,
                          float* dw_f32, float* dbias, void* ws, size_t ws_bytes, void* stream);

/* The same in two halves: _begin runs the filter-gradient kernel (and any
 * BiasAddGrad it cannot fuse) and leaves its split-K reduction pending in ws,
 * reporting pending[2] = {splits, slab rows}; _end (same d, dw, dbias, ws)
 * performs that reduction -- on another stream if the caller orders it after
 * _begin's (an event), so it overlaps the next layer's input gradient.
 * pending[0] <= 1: nothing left to do. */
int seg_conv2d_bwd_filter_begin(const seg_conv_desc* d, const void* x, const void* dy, float* dw_f32,
                                float* dbias, void* ws, size_t ws_bytes, int* pending, void* stream);
int seg_conv2d_bwd_filter_end(const seg_conv_desc* d, float* dw_f32, float* dbias, void* ws,
                              const int* pending, void* stream);

/* ---- conv2d_transpose (Network/model/FCN.py:155, :106; utils.py:272) ---- */
/* w_rskc: packed filter [R][S][K][C] in `dtype` (TF layout, seg_pack_filter mode 2). */
int seg_tconv2d_fwd(const seg_conv_desc* d, const void* x, const void* w_rskc,
                    const seg_epilogue* epi, void* y, void* ws, size_t ws_bytes, void* stream);
/* Gradient w.r.t. the tconv input = strided Conv2D of dy.  w_crsk: packed
 * [C][R][S][K] (seg_pack_filter mode 3). */
int seg_tconv2d_bwd_data(const seg_conv_desc* d, const void* dy, const void* w_crsk,
                         const seg_epilogue* epi, void* dx, void* ws, size_t ws_bytes, void* stream);
/* Filter gradient in TF layout [R][S][k_valid][c_valid], fp32; dbias as above. */
int seg_tconv2d_bwd_filter(const seg_conv_desc* d, const void* x, const void* dy,
                           float* dw_f32, float* dbias, void* ws, size_t ws_bytes, void* stream);
/* Output-channel extent `a_pad` of the packed tconv filters (modes 2 and 3)
 * that the three tconv entry points expect for this descriptor: d->K (the
 * channel count padded to 8) in general; the true even channel count for a
 * "tap-dense" tconv (few output channels, stride >= 4, square kernel -- FCN
 * conv_t3, Network/model/FCN.py:101-107), whose GEMMs skip padding channels.
 * Negative status on an invalid descriptor. */
int seg_tconv_filter_apad(const seg_conv_desc* d);

/* Workspace bytes for op: 0 fwd, 1 bwd_data, 2 bwd_filter, 3 tconv fwd,
 * 4 tconv bwd_data, 5 tconv bwd_filter. */
size_t seg_conv_workspace(const seg_conv_desc* d, int op);

/* Which kernel instantiation an op (numbering as seg_conv_workspace) will
 * launch ("igemm_nt<bf16,128,128>"), its split-K factor (>1 adds a reduce
 * kernel) and its algorithmic FLOPs (2 * MACs over unpadded channels).
 * Host-only; used by bench.py to attribute HIP-event timings. */
int seg_conv_kernel_info(const seg_conv_desc* d, int op, char* name, int len, int* splits,
                         double* flops);

/* Kernel-selection knobs (host-only): the library's only mutable state, one
 * set per HIP device (the tuned defaults until changed; SURVEY.md 8b:
 * "stateless apart from a mutex-guarded, per-device tuned-config cache").
 * seg_set_option validates the value, then writes the calling thread's current
 * device's set under a mutex; every later launch on that device reads it.
 * No reference interface: TensorFlow's kernels pick their algorithms
 * internally (Network/ never selects one).  Returns SEG_EINVAL for an unknown
 * name or a value outside the knob's parity-tested set. */
int seg_set_option(const char* name, int value);
int seg_get_option(const char* name, int* value);

/* ---- filter packing: fp32 master -> compute copy ----------------------- */
/* src: fp32 master [R][S][A][B] with A=a_valid, B=b_valid; dst (dtype,
 * channel dims padded to a_pad/b_pad with zeros):
 *   mode 0: [B][R][S][A]   (conv fwd, K-major "KRSC")
 *   mode 1: [R][S][A][B]   (conv bwd_data, HWIO)
 *   mode 2: [R][S][A][B]   (tconv fwd; same as 1, TF [kh,kw,out,in])
 *   mode 3: [B][R][S][A]   (tconv bwd_data)                             */
int seg_pack_filter(const float* src, void* dst, int R, int S, int a_valid, int b_valid,
                    int a_pad, int b_pad, int mode, int dtype, void* stream);

/* ---- ReluGrad + BiasAddGrad (implicit in minimize, FCN.py:340) --------- */
/* dz = scale * dy * (y > 0) if relu else scale * dy; dbias[k] = sum over
 * pixels of dz (k < k_valid; dbias may be NULL).  dz may alias dy.  scale is
 * 1/keep_prob when TF1 dropout followed the ReLU (y is then the dropped
 * output, so y > 0 also encodes the dropout mask).
 * ws >= seg_bias_grad_workspace() (always required). */
int seg_bias_relu_bwd(const void* dy, int ld_dy, const void* y, int ld_y, void* dz, int ld_dz,
                      float* dbias, long P, int K, int k_valid, int relu, float scale, int dtype,
                      void* ws, size_t ws_bytes, void* stream);
size_t seg_bias_grad_workspace(long P, int K);

/* ---- MaxPool / AvgPool 2x2 stride 2 VALID (FCN.py:161-163; utils.py:309) */
int seg_maxpool2x2_fwd(const void* x, void* y, int N, int H, int W, int C, int ldx, int ldy,
                       int dtype, void* stream);
/* dx (dense [N,H,W,C], ldx) is fully written; routes dy to the first max
 * in row-major window order (TF CPU MaxPoolGrad tie rule).  relu_mask != 0
 * also applies ReluGrad of the (post-ReLU) pool input x: the routed value is
 * kept only where that max is > 0. */
int seg_maxpool2x2_bwd(const void* x, const void* y, const void* dy, void* dx, int N, int H,
                       int W, int C, int ldx, int ldy, int relu_mask, int dtype, void* stream);
/* Training form (same ops, replaces the pair above inside a train step): the
 * forward also records, per pooled element, one byte of idx (row stride C,
 * 8-byte aligned): bits 0-1 the first-max window position (row-major), bit 2
 * set where that max is > 0.  The gradient then reads dy and idx only (not x).
 * Requires N*ceil(H/2)*ceil(W/2)*C/epc < 2^31 (SEG_EINVAL otherwise: use the
 * x-reading pair). */
int seg_maxpool2x2_fwd_argmax(const void* x, void* y, void* idx, int N, int H, int W, int C,
                              int ldx, int ldy, int dtype, void* stream);
int seg_maxpool2x2_bwd_argmax(const void* idx, const void* dy, void* dx, int N, int H, int W,
                              int C, int ldx, int ldy, int relu_mask, int dtype, void* stream);
int seg_avgpool2x2_fwd(const void* x, void* y, int N, int H, int W, int C, int ldx, int ldy,
                       int dtype, void* stream);
int seg_avgpool2x2_bwd(const void* dy, void* dx, int N, int H, int W, int C, int ldx, int ldy,
                       int dtype, void* stream);

/* ---- elementwise -------------------------------------------------------- */
/* y = a + b  (tf.add, FCN.py:171), dense, n elements. */
int seg_add(const void* a, const void* b, void* y, long n, int dtype, void* stream);
/* y = x / kp * floor(kp + U[0,1)), U from a counter hash of (seed, index)
 * (tf.nn.dropout, FCN.py:167). */
int seg_dropout_fwd(const void* x, void* y, long n, float keep_prob, uint64_t seed, int dtype,
                    void* stream);
int seg_dropout_bwd(const void* dy, void* dx, long n, float keep_prob, uint64_t seed, int dtype,
                    void* stream);
/* Gradient of a dropout fused into a conv epilogue without ReLU (the
 * epilogue draws element (pixel p, channel c) with counter p * c_valid + c):
 * dz = dy / keep_prob * floor(keep_prob + U), padding channels zeroed.
 * NHWC with pixel strides ldy / ldz, C % 8 == 0. */
int seg_dropout_bwd_ch(const void* dy, int ldy, void* dz, int ldz, long P, int C, int c_valid,
                       float keep_prob, uint64_t seed, int dtype, void* stream);
/* Frozen-stat BatchNorm (+ReLU): y = relu?(x*scale[c] + shift[c])
 * (Network/utils/utils.py:300-301).  scale = gamma/sqrt(1+eps). */
int seg_bn_relu_fwd(const void* x, int ldx, void* y, int ldy, const float* gamma,
                    const float* beta, float eps, long P, int C, int c_valid, int relu,
                    int dtype, void* stream);
/* dx = dy*(y>0)*scale; dgamma = sum(dy*(y>0)*x)/sqrt(1+eps); dbeta = sum(dy*(y>0)).
   flags: bit 0 = the forward had the ReLU (mask by y > 0), bit 1 = accumulate
   (dx += ..., for gradients landing in a shared concat buffer).  y may be
   NULL when beta is given: the mask is then re-derived from x with the
   forward's arithmetic (x*gamma/sqrt(1+eps) + beta > 0) and y is not read. */
int seg_bn_relu_bwd(const void* x, int ldx, const void* y, int ldy, const void* dy, int lddy,
                    void* dx, int lddx, const float* gamma, const float* beta, float eps, float* dgamma,
                    float* dbeta, long P, int C, int c_valid, int flags, int dtype, void* ws,
                    size_t ws_bytes, void* stream);
/* seg_bn_relu_bwd whose x is the output of a conv epilogue with a fused TF1
 * dropout and no ReLU (Conv2D_Block -> Dropout -> Batch_Normalization,
 * Network/model/FCDenseNet.py:28-30): dx is additionally multiplied by that
 * dropout's mask / keep_prob (counter pixel * drop_c_valid + c, as
 * seg_dropout_bwd_ch), so the conv's separate dropout-gradient pass goes
 * away.  No accumulation (flags bit 1 must be 0). */
int seg_bn_relu_dropout_bwd(const void* x, int ldx, const void* y, int ldy, const void* dy, int lddy,
                            void* dx, int lddx, const float* gamma, const float* beta, float eps, float* dgamma,
                            float* dbeta, long P, int C, int c_valid, int flags, float keep_prob, uint64_t seed,
                            int drop_c_valid, int dtype, void* ws, size_t ws_bytes, void* stream);
/* resize_bilinear(align_corners=True) (Network/utils/utils.py:329-330). */
int seg_resize_bilinear_fwd(const void* x, void* y, int N, int H, int W, int C, int OH, int OW,
                            int dtype, void* stream);
/* dx is zeroed then scatter-added (fp32 dx only). */
int seg_resize_bilinear_bwd(const void* dy, float* dx, int N, int H, int W, int C, int OH,
                            int OW, int dtype, void* stream);
/* Global average pooling (tflearn global_avg_pool = tf.reduce_mean(x, [1, 2]),
 * Network/utils/utils.py:312; DeepLab's image-pooling branch,
 * Network/model/DeepLabv3Plus.py:215-225): y[n, c] = scale * sum_hw x[n, h, w, c]
 * (scale = 1/(H*W); scale = 1 is the gradient of a 1x1 -> HxW align_corners
 * resize).  y is [N, C] in the compute dtype; ws: N*C fp32 scratch.
 * C <= 256 chunks of 16 bytes. */
int seg_spatial_reduce(const void* x, int ldx, void* y, int N, int H, int W, int C, float scale,
                       float* ws, int dtype, void* stream);
/* y[n, h, w, c] = scale * x[n, c]: the gradient of global average pooling
 * (scale = 1/(H*W)) and the forward of a 1x1 -> HxW align_corners resize
 * (scale = 1, Network/model/DeepLabv3Plus.py:222-223). */
int seg_spatial_broadcast(const void* x, void* y, int ldy, int N, int H, int W, int C, float scale,
                          int dtype, void* stream);
/* tf.concat(axis=-1) (Network/utils/utils.py:332-333; DenseBlock
 * FCDenseNet.py:48-61): parts at arbitrary (unaligned) channel offsets.
 * fwd: y[p, off_i + c] = part_i[p, c]; channels >= sum are written 0.
 * bwd: part_i[p, c] (+)= dy[p, off_i + c]  (accumulate != 0 adds), padding
 * channels of each part are left 0 (or unchanged when accumulating).     */
#define SEG_CONCAT_MAX 64
typedef struct seg_concat_part {
    const void* ptr;     /* fwd: source; bwd: destination (cast away const) */
    int ld;              /* pixel stride (elements) */
    int channels;        /* valid channels of this part */
    int accumulate;      /* bwd only */
} seg_concat_part;
int seg_concat_fwd(const seg_concat_part* parts, int nparts, void* y, int ldy, int ychannels, long P, int dtype,
                   void* stream);
int seg_concat_bwd(const void* dy, int ldy, const seg_concat_part* parts, int nparts, long P, int dtype,
                   void* stream);
/* Channel-slice copy: y[p, 0:C] = x[p, 0:C] (tf.concat building block). */
int seg_copy_channels(const void* x, int ldx, void* y, int ldy, long P, int C, int dtype,
                      void* stream);
/* fp32 NHWC image (values 0..255, c_in channels, H x W) -> dtype NHWC padded
 * to [N, HP, WP, CP] with zeros (SURVEY.md 0-3 pad policy). */
int seg_prepare_input(const float* img, void* x, int N, int H, int W, int c_in, int HP, int WP,
                      int CP, int dtype, void* stream);
/* Same from uint8 images (the decoded / augmented batch as the reference
 * feeds it: feed_dict uint8 arrays into the float32 placeholder). */
int seg_prepare_input_u8(const uint8_t* img, void* x, int N, int H, int W, int c_in, int HP, int WP,
                         int CP, int dtype, void* stream);

/* ---- host PNG decode (scipy.misc.imread of merge/ and gt_image_2/ PNGs,
 * FCN.py:267-268).  8-bit grey / grey+alpha / RGB / RGBA, non-interlaced;
 * other PNGs return SEG_EINVAL (decode those another way).  Host memory
 * only; thread-safe, no GPU work. */
int seg_png_info(const void* png, size_t n, int* h, int* w, int* channels);
/* out = uint8 [h][w][channels] (out_bytes >= h * w * channels). */
int seg_png_decode(const void* png, size_t n, void* out, size_t out_bytes);

/* ---- training-data augmentation (gen_batch_function, FCN.py:235-307) ----
 * One view = one training sample cut from a decoded uint8 image in device
 * memory: the window [y0, y0+h) x [x0, x0+w) of src [H0][W0][C]
 * (crop_image, FCN.py:176-182; the whole image otherwise), optionally
 * mirrored along x (flip_image, :184-185), resized to OH x OW exactly as
 * scipy.misc.imresize(..., 'bilinear') = PIL Image.resize(BILINEAR) does
 * (antialiased two-pass 8-bit resample; RGBA premultiplied), then, if bc,
 * bc_img(img, contrast, bright) (:187-193). */
typedef struct seg_aug_view {
    const void* src;
    int H0, W0;
    int x0, y0, w, h;
    int flip;
    int bc;
    int bright;
    double contrast;
} seg_aug_view;
/* labels = 0: out = uint8 [nviews][OH][OW][C] images (C = 3 RGB or 4 RGBA).
 * labels = 1: src are ground-truth colour images (C = 3); out = uint8
 * [nviews][OH][OW] class index of process_gt_image (:195-201): 0 where the
 * resized pixel is exactly (255, 0, 0) (background), else 1.
 * Downscale factors up to 8 per axis; a window outside its source or a larger
 * downscale returns SEG_ESHAPE. */
int seg_augment(const seg_aug_view* views, int nviews, int C, int OH, int OW, int labels, void* out,
                void* stream);

/* ---- loss / prediction (FCN.py:334, :111) ------------------------------- */
/* Per pixel over the valid region (h < valid_h, w < valid_w) of
 * logits [N,H,W,ld] (classes 0..C-1), labels uint8 class index:
 *   loss_sum += logsumexp(z) - z[label];
 *   dlogits = (softmax(z) - onehot) * grad_scale   (0 outside valid region
 *   and in padding channels).  loss_sum is written (fp32, 1 element). */
int seg_softmax_xent_fwd_bwd(const void* logits, int ld, const uint8_t* labels, int N, int H,
                             int W, int C, int valid_h, int valid_w, float grad_scale,
                             float* loss_sum, void* dlogits, int ld_d, int dtype, void* ws,
                             size_t ws_bytes, void* stream);
size_t seg_xent_workspace(int N, int H, int W);
/* Soft-label variant (labels [N,H,W,C] fp32, e.g. one-hot from process_gt_image). */
int seg_softmax_xent_soft_fwd_bwd(const void* logits, int ld, const float* labels, int N, int H,
                                  int W, int C, int valid_h, int valid_w, float grad_scale,
                                  float* loss_sum, void* dlogits, int ld_d, int dtype, void* ws,
                                  size_t ws_bytes, void* stream);
/* tf.nn.softmax over channels (eval path, Network/utils/utils.py:54 and
 * Network/model/FCN.py gen_test_output): y[p, c] for c < C, 0 for padding. */
int seg_softmax(const void* x, int ldx, int C, long P, void* y, int ldy, int dtype, void* stream);
/* pred[p] = argmax_c logits[p, c] (ties -> lowest index). */
int seg_argmax(const void* logits, int ld, int C, long P, int64_t* pred, int dtype, void* stream);
/* Confusion matrix counts conf[t*C+p] += 1 over the valid region (mIoU). */
int seg_confusion(const int64_t* pred, const uint8_t* labels, int N, int H, int W, int valid_h,
                  int valid_w, int C, unsigned long long* conf, void* stream);

/* ---- AdamOptimizer (FCN.py:338-340), TF1 epsilon placement -------------- */
/* In place over a flat fp32 parameter buffer:
 *   g' = g*grad_scale; m = b1 m + (1-b1) g'; v = b2 v + (1-b2) g'^2;
 *   p -= lr*sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps).                    */
int seg_adam_tf1_step(float* p, const float* g, float* m, float* v, long n, float lr,
                      float beta1, float beta2, float eps, int t, float grad_scale, void* stream);

/* Multi-tensor Adam fused with the packed compute copies (one launch per step).
 * Each segment is one variable of the flat buffers viewed as [rs][a][b]
 * (conv HWIO: rs=R*S, a=C, b=K; tconv [kh,kw,out,in]: a=out, b=in; biases:
 * rs=a=1).  After the update the new values are also written to the optional
 * copies (element type = dtype; padding entries are left untouched):
 *   rows_dst[(rs*rows_ap + a)*rows_bp + b]   (seg_pack_filter modes 1, 2)
 *   tr_dst  [(b*RS + rs)*tr_ap + a]          (seg_pack_filter modes 0, 3)
 * replaces seg_adam_tf1_step + seg_pack_filter per step.                     */
typedef struct seg_adam_segment {
    long long offset;       /* element offset into p / g / m / v */
    int rs, a, b;
    int tile_begin;         /* filled by seg_adam_segments_plan */
    void* rows_dst;
    int rows_ap, rows_bp;
    void* tr_dst;
    int tr_ap, tr_bp;
} seg_adam_segment;
/* Host-side: fills tile_begin.  The one entry point that returns a count:
 * the total tile count (>= 0), or -SEG_EINVAL (the negated status code) when a
 * segment is malformed. */
int seg_adam_segments_plan(seg_adam_segment* segs, int nsegs);
/* dev_segs: the planned table copied to device memory. */
int seg_adam_tf1_pack(float* p, const float* g, float* m, float* v, const seg_adam_segment* dev_segs,
                      int nsegs, int total_tiles, float lr, float beta1, float beta2, float eps, int t,
                      float grad_scale, int dtype, void* stream);

/* The packed compute copies of seg_adam_tf1_pack's segments rewritten from p
 * alone (no update): the repack after a data-parallel step whose Adam ran on
 * each rank's shard and whose parameters were then all-gathered (ZeRO-1).
 * Replaces a seg_pack_filter per variable and layout. */
int seg_pack_segments(const float* p, const seg_adam_segment* dev_segs, int nsegs, int total_tiles, int dtype,
                      void* stream);

/* Conv2DBackpropFilter fused with TF1 Adam (AdamOptimizer.minimize,
 * Network/model/FCN.py:338-340) on that filter, for single-process training
 * where nothing (no all-reduce) sits between the gradient and the update:
 * the filter-gradient epilogue reads p/m/v, applies the update of
 * seg_adam_tf1_pack element-for-element and rewrites the packed bf16 copies,
 * so the fp32 gradient never round-trips through HBM.  p/m/v are the flat
 * fp32 [R][S][c_valid][k_valid] slices of the variable; rows_dst = the HWIO
 * copy (mode 1, [RS][rows_ap][rows_bp]) and tr_dst = the KRSC copy (mode 0,
 * [K][RS][tr_ap]), either may be NULL.  dw_f32 may be NULL; if given, the
 * gradient is stored too.  dbias as seg_conv2d_bwd_filter (not fused into
 * Adam).  Returns SEG_EINVAL when seg_conv_wgrad_adam_fusable(d) is 0. */
typedef struct seg_adam_fused {
    float* p;
    float* m;
    float* v;
    void* rows_dst;
    int rows_ap, rows_bp;
    void* tr_dst;
    int tr_ap;
    float lr, beta1, beta2, eps;
    int t;
    float grad_scale;
} seg_adam_fused;
int seg_conv_wgrad_adam_fusable(const seg_conv_desc* d);
int seg_conv2d_bwd_filter_adam(const seg_conv_desc* d, const void* x, const void* dy, float* dw_f32,
                               float* dbias, const seg_adam_fused* adam, void* ws, size_t ws_bytes,
                               void* stream);

/* ---- misc ---------------------------------------------------------------- */
int seg_fill(void* y, long n, float value, int dtype, void* stream);
/* y += alpha * x over n fp32 elements: the accumulate-then-apply template's
 * `accum.assign_add(tf.scalar_mul(const, grad))` (Network/main.py:92-95,
 * Network/model/FCDenseNet.py:213). */
int seg_axpy(float* y, const float* x, float alpha, long n, void* stream);
/* *flag = 1 if any of the n fp32 values is Inf / NaN, else 0 (dynamic loss
 * scaling for the fp16 path: a step with overflowed scaled gradients is
 * skipped and the scale halved, as TF's DynamicLossScale). g 16-byte aligned. */
int seg_check_finite(const float* g, long n, int* flag, void* stream);
int seg_cast(const void* x, int xdtype, void* y, int ydtype, long n, void* stream);
/* CRC-32C (Castagnoli) of n bytes continuing from crc (0 to start): host
 * code for tf.train.Saver's tensor-bundle checkpoints (per-tensor checksums
 * in the .index file, SSTable block trailers). */
uint32_t seg_crc32c(const void* data, size_t n, uint32_t crc);
/* Timing events (Session.timer / bench.py per-launch roofline timing): HIP
 * events created with hipEventDisableSystemFence, so recording one does not
 * write back and invalidate the caches.  A plain timing event adds that
 * system-scope release to the interval it closes: +23 us (+15 %) per
 * conv_halo2 launch in the C2 step against a kernel trace of the same steps.
 * elapsed waits for `end`.  Not a TF interface: measurement support. */
int seg_timing_event_create(void** ev);
int seg_timing_event_record(void* ev, void* stream);
int seg_timing_event_elapsed_ms(float* ms, void* start, void* end);
int seg_timing_event_destroy(void* ev);
const char* seg_status_string(int status);
int seg_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SEGKERN_H */
