"""Typed wrappers over the C-ABI (`include/segkern.h`) on torch device tensors.

Every function here launches hand-written gfx950 kernels from libsegkern.so on
the caller's current HIP stream; torch provides only memory and the stream.
Activation tensors are NHWC with the channel dim padded to a multiple of 8
(`round8`); a channel-slice view is allowed (its pixel stride is read from the
tensor's stride).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import SegBnBwd, SegBnFinishSegment, SegConvDesc, SegEpilogue, SegKernelError, SegPrologue, check

F32, BF16, F16 = 0, 1, 2
_TORCH_DT = {F32: torch.float32, BF16: torch.bfloat16, F16: torch.float16}
SAME, VALID = 0, 1


def round8(c: int) -> int:
    return (c + 7) // 8 * 8


def seg_dtype(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float32:
        return F32
    if t.dtype == torch.float16:
        return F16
    raise TypeError(f"unsupported activation dtype {t.dtype}")


def torch_dtype(d: int):
    return _TORCH_DT[d]


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def pixel_stride(t: torch.Tensor) -> int:
    """Elements between consecutive pixels of an NHWC(-view) tensor."""
    if t.stride(-1) != 1:
        raise ValueError("channel dim must be unit-stride")
    return t.stride(-2) if t.dim() >= 2 else t.shape[-1]


class Workspace:
    """Grow-only device scratch buffer (allocated outside hot loops)."""

    def __init__(self, device=None):
        self.device = device
        self.buf = None

    def get(self, nbytes: int):
        nbytes = max(int(nbytes), 256)
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return self.buf

    def ptr_size(self, nbytes):
        b = self.get(nbytes)
        return ctypes.c_void_p(b.data_ptr()), ctypes.c_size_t(b.numel())


# ---------------------------------------------------------------------------
# descriptors
# ---------------------------------------------------------------------------
class TimingEvent:
    """A HIP event for kernel timing without the system-scope cache flush
    (seg_timing_event_*); torch.cuda.Event's record / elapsed_time API."""

    def __init__(self):
        h = ctypes.c_void_p()
        check(_lib.lib().seg_timing_event_create(ctypes.byref(h)), "timing_event")
        self._h = h

    def record(self, stream=None):
        check(_lib.lib().seg_timing_event_record(self._h, stream_ptr(stream)), "timing_event")

    def elapsed_time(self, end):
        ms = ctypes.c_float()
        check(_lib.lib().seg_timing_event_elapsed_ms(ctypes.byref(ms), self._h, end._h), "timing_event")
        return ms.value

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.lib().seg_timing_event_destroy(self._h)
            self._h = None


def conv_desc(N, H, W, C, K, R, S, stride=1, dilation=1, padding="SAME", dtype=BF16):
    d = SegConvDesc()
    check(_lib.lib().seg_conv_desc_init(ctypes.byref(d), N, H, W, C, K, R, S, stride, dilation,
                                        SAME if padding == "SAME" else VALID, dtype), "conv2d")
    return d


def tconv_desc(N, H, W, C, OH, OW, K, R, S, stride, padding="SAME", dtype=BF16):
    d = SegConvDesc()
    check(_lib.lib().seg_tconv_desc_init(ctypes.byref(d), N, H, W, C, OH, OW, K, R, S, stride,
                                         SAME if padding == "SAME" else VALID, dtype),
          "conv2d_transpose")
    return d


def epilogue(bias=None, scale=None, shift=None, residual=None, relu=False, keep_prob=1.0, seed=0,
             relu_mask=None, mask_scale=1.0):
    """seg_epilogue.  relu_mask (gradient kernels): the post-ReLU output of the
    layer whose input gradient is being written; v = mask > 0 ? v*mask_scale : 0."""
    e = SegEpilogue()
    e.bias = None if bias is None else bias.data_ptr()
    e.scale = None if scale is None else scale.data_ptr()
    e.shift = None if shift is None else shift.data_ptr()
    e.residual = None if residual is None else residual.data_ptr()
    e.ld_residual = 0 if residual is None else pixel_stride(residual)
    e.relu = 1 if relu else 0
    e.keep_prob = float(keep_prob)
    e.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    e.relu_mask = None if relu_mask is None else relu_mask.data_ptr()
    e.ld_relu_mask = 0 if relu_mask is None else pixel_stride(relu_mask)
    e.mask_scale = float(mask_scale)
    # the struct holds raw device pointers: keep the tensors alive with it, or a
    # temporary (epilogue(bias=b.to(dev))) is freed and its memory reused by the
    # next allocation before the kernel reads it
    e._keep = (bias, scale, shift, residual, relu_mask)
    return e


OP_FWD, OP_BWD_DATA, OP_BWD_FILTER, OP_TFWD, OP_TBWD_DATA, OP_TBWD_FILTER = range(6)
# kernel-table only (seg_conv_kernel_info): the folded-BatchNorm forms
OP_BWD_DATA_BN, OP_FWD_PRO, OP_BWD_FILTER_PRO = 6, 7, 8


def conv_kernel_info(desc, op):
    """(kernel name, split-K factor, algorithmic FLOPs) of a conv op launch."""
    buf = ctypes.create_string_buffer(64)
    sp = ctypes.c_int(0)
    fl = ctypes.c_double(0)
    check(_lib.lib().seg_conv_kernel_info(ctypes.byref(desc), op, buf, 64, ctypes.byref(sp),
                                          ctypes.byref(fl)), "conv_kernel_info")
    return buf.value.decode(), sp.value, fl.value


def set_option(name: str, value: int):
    """Set a kernel-selection knob for the current HIP device (include/segkern.h)."""
    check(_lib.lib().seg_set_option(name.encode(), int(value)), f"set_option({name})")


def get_option(name: str) -> int:
    """The current HIP device's value of a kernel-selection knob."""
    v = ctypes.c_int(0)
    check(_lib.lib().seg_get_option(name.encode(), ctypes.byref(v)), f"get_option({name})")
    return v.value


def conv_workspace(desc, op):
    return int(_lib.lib().seg_conv_workspace(ctypes.byref(desc), op))


# ---------------------------------------------------------------------------
# convolutions
# ---------------------------------------------------------------------------
def _with_ld(desc, x=None, y=None):
    d = SegConvDesc.from_buffer_copy(desc)
    if x is not None:
        d.ldx = pixel_stride(x)
    if y is not None:
        d.ldy = pixel_stride(y)
    return d


def conv2d_fwd(desc, x, w_krsc, y, epi=None, ws=None, stream=None):
    d = _with_ld(desc, x, y)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_FWD))
    check(_lib.lib().seg_conv2d_fwd(ctypes.byref(d), ptr(x), ptr(w_krsc),
                                    None if epi is None else ctypes.byref(epi), ptr(y), wsp, wss,
                                    stream_ptr(stream)), "conv2d")
    return y


def conv2d_fwd_hwio_ok(desc):
    """Whether seg_conv2d_fwd_hwio (the forward from the HWIO copy) takes this conv."""
    return bool(_lib.lib().seg_conv2d_fwd_hwio_ok(ctypes.byref(desc)))


def conv2d_fwd_hwio(desc, x, w_hwio, y, epi=None, ws=None, stream=None):
    """Conv2D (+ epilogue) reading the HWIO filter copy (the input gradient's)."""
    d = _with_ld(desc, x, y)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_FWD))
    check(_lib.lib().seg_conv2d_fwd_hwio(ctypes.byref(d), ptr(x), ptr(w_hwio),
                                         None if epi is None else ctypes.byref(epi), ptr(y), wsp, wss,
                                         stream_ptr(stream)), "conv2d_hwio")
    return y


def conv2d_fwd_pool_ok(desc):
    """Whether seg_conv2d_fwd_pool (Conv2D + bias + ReLU + MaxPool 2x2/2 in one
    launch) takes this convolution."""
    return bool(_lib.lib().seg_conv2d_fwd_pool_ok(ctypes.byref(desc)))


def conv2d_fwd_pool(desc, x, w_krsc, y_pool, idx=None, epi=None, ws=None, stream=None):
    """Conv2D + epilogue (bias, ReLU) + MaxPool 2x2 / 2: writes the pooled map
    y_pool [N, OH/2, OW/2, K] and, when idx is given, the switches
    (maxpool2x2_fwd_argmax's encoding, row stride = y_pool's channel count);
    the conv output itself is never materialised."""
    d = _with_ld(desc, x, None)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_FWD))
    check(_lib.lib().seg_conv2d_fwd_pool(ctypes.byref(d), ptr(x), ptr(w_krsc),
                                         None if epi is None else ctypes.byref(epi), ptr(y_pool),
                                         pixel_stride(y_pool), None if idx is None else ptr(idx),
                                         y_pool.shape[3] if idx is not None else 0, wsp, wss,
                                         stream_ptr(stream)), "conv2d_pool")
    return y_pool


def prologue(gamma, beta, eps=1e-3, relu=True):
    """The conv input is relu(x * gamma / sqrt(1 + eps) + beta) (frozen BN + ReLU).
    The struct keeps gamma / beta alive (it holds raw device pointers)."""
    pro = SegPrologue(gamma.data_ptr(), beta.data_ptr(), float(eps), 1 if relu else 0)
    pro._keep = (gamma, beta)
    return pro


def conv2d_fwd_pro(desc, x, pro, w_krsc, y, epi=None, ws=None, stream=None):
    """Conv2D of relu(BN(x)) with the BN + ReLU applied while staging x."""
    d = _with_ld(desc, x, y)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_FWD))
    check(_lib.lib().seg_conv2d_fwd_pro(ctypes.byref(d), ptr(x), ctypes.byref(pro), ptr(w_krsc),
                                        None if epi is None else ctypes.byref(epi), ptr(y), wsp, wss,
                                        stream_ptr(stream)), "conv2d")
    return y


def conv2d_fwd_bn2_ok(desc, with_prologue=False):
    """Whether conv2d_fwd_bn2 runs this conv (the kernel it plans for has the
    second, BatchNorm(+ReLU), output)."""
    return bool(_lib.lib().seg_conv2d_fwd_bn2_ok(ctypes.byref(desc), 1 if with_prologue else 0))


def conv2d_fwd_bn2(desc, x, pro, w_krsc, y, y2, gamma2, beta2, relu2=True, eps2=1e-3, epi=None, ws=None,
                   stream=None):
    """Conv2D (pro: operand prologue or None) writing y and y2 = relu(BN(y))
    (seg_conv2d_fwd_bn2; y2 bit-identical to bn_relu_fwd(y, y2, ...))."""
    d = _with_ld(desc, x, y)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_FWD))
    check(_lib.lib().seg_conv2d_fwd_bn2(ctypes.byref(d), ptr(x), None if pro is None else ctypes.byref(pro),
                                        ptr(w_krsc), None if epi is None else ctypes.byref(epi), ptr(y), ptr(y2),
                                        pixel_stride(y2), ptr(gamma2), ptr(beta2), float(eps2),
                                        1 if relu2 else 0, wsp, wss, stream_ptr(stream)), "conv2d_fwd_bn2")
    return y


def conv_bwd_data_bn_workspace(desc):
    """Bytes for conv2d_bwd_data_bn, 0 where the fused path does not apply."""
    return int(_lib.lib().seg_conv_bwd_data_bn_workspace(ctypes.byref(desc)))


def conv2d_bwd_data_bn(desc, dy, w_hwio, x, gamma, beta, dx, dgamma, dbeta, eps=1e-3, relu=True,
                       accumulate=False, ws=None, stream=None, dropout=None):
    """Conv2DBackpropInput of a conv over relu(BN(x)) continued through the
    BatchNorm(+ReLU) backward: dx = dL/dx of the BN input (+= with
    accumulate), dgamma / dbeta overwritten (seg_conv2d_bwd_data_bn).
    dropout = (keep_prob, seed): the 3x3 form also applies the gradient of
    the dropout fused into the conv that produced x."""
    d = _with_ld(desc, dx, dy)
    need = conv_bwd_data_bn_workspace(d)
    if need == 0:
        raise SegKernelError("conv2d_bwd_data_bn: fused BatchNorm backward does not apply to this conv")
    wsp, wss = (ws or Workspace(dy.device)).ptr_size(need)
    kp, seed = dropout if dropout is not None else (1.0, 0)
    bn = SegBnBwd(x.data_ptr(), pixel_stride(x), gamma.data_ptr(), beta.data_ptr(), float(eps), 1 if relu else 0,
                  1 if accumulate else 0, dgamma.data_ptr(), dbeta.data_ptr(), float(kp), int(seed) & (2 ** 64 - 1))
    check(_lib.lib().seg_conv2d_bwd_data_bn(ctypes.byref(d), ptr(dy), ptr(w_hwio), ctypes.byref(bn), ptr(dx),
                                            wsp, wss, stream_ptr(stream)), "conv2d_backprop_input_bn")
    return dx


def conv_bwd_data_bn_part_rows(desc):
    """Partial rows conv2d_bwd_data_bn_part writes (0: the fused form does not apply)."""
    return int(_lib.lib().seg_conv_bwd_data_bn_part_rows(ctypes.byref(desc)))


def conv2d_bwd_data_bn_part(desc, dy, w_hwio, x, gamma, beta, dx, part, eps=1e-3, relu=True, accumulate=False,
                            stream=None, dropout=None):
    """conv2d_bwd_data_bn with the dgamma / dbeta sums left as partial rows in
    `part` (fp32, conv_bwd_data_bn_part_rows(desc) x 2 C): finish them with
    BnFinishBatch (seg_conv2d_bwd_data_bn_part)."""
    d = _with_ld(desc, dx, dy)
    kp, seed = dropout if dropout is not None else (1.0, 0)
    bn = SegBnBwd(x.data_ptr(), pixel_stride(x), gamma.data_ptr(), beta.data_ptr(), float(eps), 1 if relu else 0,
                  1 if accumulate else 0, None, None, float(kp), int(seed) & (2 ** 64 - 1))
    rows = part.numel() // (2 * desc.C)
    check(_lib.lib().seg_conv2d_bwd_data_bn_part(ctypes.byref(d), ptr(dy), ptr(w_hwio), ctypes.byref(bn), ptr(dx),
                                                 ptr(part), rows, stream_ptr(stream)), "conv2d_backprop_input_bn")
    return dx


class BnFinishBatch:
    """dgamma / dbeta of many BatchNorm backward launches (partial rows left
    by conv2d_bwd_data_bn_part) in two kernel launches (seg_bn_grad_finish_batch).
    segments: [(part, nrows, C, c_valid, eps, dgamma, dbeta)] with fp32 tensors;
    the segment table and the fold scratch live on the device for reuse."""

    def __init__(self, segments, device):
        n = len(segments)
        arr = (SegBnFinishSegment * n)()
        self._keep = [(s[0], s[5], s[6]) for s in segments]
        for i, (part, nrows, C, cv, eps, dg, db) in enumerate(segments):
            arr[i].part, arr[i].nrows, arr[i].C, arr[i].cv = part.data_ptr(), int(nrows), int(C), int(cv)
            # 1.0f / sqrtf(1.0f + eps) in fp32, as the C-ABI's own finish
            arr[i].inv = float(np.float32(1.0) / np.sqrt(np.float32(1.0) + np.float32(eps)))
            arr[i].dgamma, arr[i].dbeta = dg.data_ptr(), db.data_ptr()
        a, b = ctypes.c_int(0), ctypes.c_int(0)
        lib = _lib.lib()
        need = lib.seg_bn_finish_batch_plan(ctypes.cast(arr, ctypes.c_void_p), n, None, ctypes.byref(a), ctypes.byref(b))
        self.scratch = torch.empty(max(1, need // 4), dtype=torch.float32, device=device)
        lib.seg_bn_finish_batch_plan(ctypes.cast(arr, ctypes.c_void_p), n, ctypes.c_void_p(self.scratch.data_ptr()),
                                     ctypes.byref(a), ctypes.byref(b))
        raw = bytes(arr)
        self.table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        self.n, self.a_blocks, self.b_blocks = n, a.value, b.value
        self.key = tuple((s[0].data_ptr(), int(s[1]), s[5].data_ptr()) for s in segments)

    def run(self, stream=None):
        check(_lib.lib().seg_bn_grad_finish_batch(ptr(self.table), self.n, self.a_blocks, self.b_blocks,
                                                  stream_ptr(stream)), "bn_grad_finish_batch")


def conv2d_bwd_filter_pro(desc, x, pro, dy, dw, ws=None, stream=None, dbias=None):
    """Conv2DBackpropFilter with input relu(BN(x)) recomputed from x."""
    d = _with_ld(desc, x, dy)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_BWD_FILTER))
    check(_lib.lib().seg_conv2d_bwd_filter_pro(ctypes.byref(d), ptr(x), ctypes.byref(pro), ptr(dy), ptr(dw),
                                               None if dbias is None else ptr(dbias), wsp, wss,
                                               stream_ptr(stream)), "conv2d_backprop_filter")
    return dw


def conv2d_bwd_data(desc, dy, w_hwio, dx, ws=None, stream=None, epi=None):
    """Conv2DBackpropInput; epi (e.g. epilogue(relu_mask=y_prev)) fuses the
    ReluGrad of the layer that produced this conv's input."""
    d = _with_ld(desc, dx, dy)
    wsp, wss = (ws or Workspace(dy.device)).ptr_size(conv_workspace(d, OP_BWD_DATA))
    check(_lib.lib().seg_conv2d_bwd_data(ctypes.byref(d), ptr(dy), ptr(w_hwio),
                                         None if epi is None else ctypes.byref(epi), ptr(dx), wsp, wss,
                                         stream_ptr(stream)), "conv2d_backprop_input")
    return dx


def conv2d_fwd_relu_bits_ok(desc):
    """Whether seg_conv2d_fwd_relu_bits (the forward that also writes its ReLU
    mask as bits) takes this conv."""
    return bool(_lib.lib().seg_conv2d_fwd_relu_bits_ok(ctypes.byref(desc)))


def relu_bits_buffer(n, h, w, k, device):
    """The bit-packed ReLU mask of an [n, h, w, k] map: k / 8 bytes per pixel."""
    return torch.empty((n, h, w, (k + 7) // 8), dtype=torch.uint8, device=device)


def conv2d_fwd_relu_bits(desc, x, w_krsc, y, bits, epi=None, stream=None):
    """Conv2D + epilogue that also writes bits[..., k // 8] bit k % 8 = y[..., k] > 0
    (seg_conv2d_fwd_relu_bits), for conv2d_bwd_data_bits of the next conv."""
    d = _with_ld(desc, x, y)
    if not bits.is_contiguous() or bits.dtype != torch.uint8:
        raise ValueError("relu bits: a contiguous uint8 [N, OH, OW, K/8] buffer")
    check(_lib.lib().seg_conv2d_fwd_relu_bits(ctypes.byref(d), ptr(x), ptr(w_krsc),
                                              None if epi is None else ctypes.byref(epi), ptr(y), ptr(bits),
                                              bits.shape[-1], stream_ptr(stream)), "conv2d_relu_bits")
    return y


def conv2d_bwd_data_bits_ok(desc):
    """Whether seg_conv2d_bwd_data_bits (the ReluGrad mask read as bits) takes this conv."""
    return bool(_lib.lib().seg_conv2d_bwd_data_bits_ok(ctypes.byref(desc)))


def conv2d_bwd_data_bits(desc, dy, w_hwio, bits, dx, mask_scale=1.0, ws=None, stream=None):
    """Conv2DBackpropInput with the ReluGrad (x mask_scale) of the layer that
    produced this conv's input, its mask given as conv2d_fwd_relu_bits' bits."""
    d = _with_ld(desc, dx, dy)
    if not bits.is_contiguous() or bits.dtype != torch.uint8:
        raise ValueError("relu bits: a contiguous uint8 [N, H, W, C/8] buffer")
    wsp, wss = (ws or Workspace(dy.device)).ptr_size(conv_workspace(d, OP_BWD_DATA))
    epi = epilogue(mask_scale=mask_scale)
    check(_lib.lib().seg_conv2d_bwd_data_bits(ctypes.byref(d), ptr(dy), ptr(w_hwio), ctypes.byref(epi), ptr(bits),
                                              bits.shape[-1], ptr(dx), wsp, wss, stream_ptr(stream)),
          "conv2d_backprop_input_bits")
    return dx


def conv2d_bwd_data_unpool_ok(desc):
    """Whether seg_conv2d_bwd_data_unpool (Conv2DBackpropInput + MaxPoolGrad in
    one launch) takes this convolution."""
    return bool(_lib.lib().seg_conv2d_bwd_data_unpool_ok(ctypes.byref(desc)))


def conv2d_bwd_data_unpool(desc, dy, w_hwio, idx, dx_full, relu_mask=False, residual=None, ws=None, stream=None):
    """Conv2DBackpropInput of the conv after a 2x2 / 2 MaxPool, continued
    through the MaxPoolGrad: dx_full [N, 2H, 2W, C] gets the input gradient
    routed by the pool's switches idx (row stride = dx_full's channel count;
    with relu_mask, ReluGrad of the post-ReLU pool input), the pooled gradient
    is never written.  residual: the pooled gradient of the pool's other
    consumers [N, H, W, C], added before routing."""
    d = _with_ld(desc, residual, dy)
    epi = None if residual is None else epilogue(residual=residual)
    wsp, wss = (ws or Workspace(dy.device)).ptr_size(conv_workspace(d, OP_BWD_DATA))
    check(_lib.lib().seg_conv2d_bwd_data_unpool(ctypes.byref(d), ptr(dy), ptr(w_hwio),
                                                None if epi is None else ctypes.byref(epi), ptr(idx),
                                                dx_full.shape[3], 1 if relu_mask else 0, ptr(dx_full),
                                                pixel_stride(dx_full), wsp, wss, stream_ptr(stream)),
          "conv2d_backprop_input_maxpool_grad")
    return dx_full


def conv2d_bwd_filter(desc, x, dy, dw, ws=None, stream=None, dbias=None):
    """Conv2DBackpropFilter (+ BiasAddGrad of dy into dbias when given)."""
    d = _with_ld(desc, x, dy)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_BWD_FILTER))
    check(_lib.lib().seg_conv2d_bwd_filter(ctypes.byref(d), ptr(x), ptr(dy), ptr(dw),
                                           None if dbias is None else ptr(dbias), wsp, wss,
                                           stream_ptr(stream)), "conv2d_backprop_filter")
    return dw


def conv2d_bwd_filter_begin(desc, x, dy, dw, ws_buf, dbias=None, stream=None):
    """First half of conv2d_bwd_filter: the kernel runs, a split-K reduction
    is left pending in `ws_buf` (a uint8 device tensor owned by the caller).
    Returns the token for conv2d_bwd_filter_end."""
    d = _with_ld(desc, x, dy)
    pend = (ctypes.c_int * 2)()
    check(_lib.lib().seg_conv2d_bwd_filter_begin(ctypes.byref(d), ptr(x), ptr(dy), ptr(dw),
                                                 None if dbias is None else ptr(dbias), ptr(ws_buf),
                                                 ws_buf.numel(), pend, stream_ptr(stream)),
          "conv2d_backprop_filter")
    return d, pend


def conv2d_bwd_filter_end(token, dw, ws_buf, dbias=None, stream=None):
    """Second half: the pending split-K reduction (no-op when there is none)."""
    d, pend = token
    if pend[0] <= 1:
        return dw
    check(_lib.lib().seg_conv2d_bwd_filter_end(ctypes.byref(d), ptr(dw), None if dbias is None else ptr(dbias),
                                               ptr(ws_buf), pend, stream_ptr(stream)), "conv2d_backprop_filter")
    return dw


def tconv2d_fwd(desc, x, w_rskc, y, epi=None, ws=None, stream=None):
    d = _with_ld(desc, x, y)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_TFWD))
    check(_lib.lib().seg_tconv2d_fwd(ctypes.byref(d), ptr(x), ptr(w_rskc),
                                     None if epi is None else ctypes.byref(epi), ptr(y), wsp, wss,
                                     stream_ptr(stream)), "conv2d_transpose")
    return y


def tconv2d_bwd_data(desc, dy, w_crsk, dx, ws=None, stream=None, epi=None):
    d = _with_ld(desc, dx, dy)
    wsp, wss = (ws or Workspace(dy.device)).ptr_size(conv_workspace(d, OP_TBWD_DATA))
    check(_lib.lib().seg_tconv2d_bwd_data(ctypes.byref(d), ptr(dy), ptr(w_crsk),
                                          None if epi is None else ctypes.byref(epi), ptr(dx), wsp, wss,
                                          stream_ptr(stream)), "conv2d_transpose_grad_input")
    return dx


def tconv2d_bwd_filter(desc, x, dy, dw, ws=None, stream=None, dbias=None):
    d = _with_ld(desc, x, dy)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_TBWD_FILTER))
    check(_lib.lib().seg_tconv2d_bwd_filter(ctypes.byref(d), ptr(x), ptr(dy), ptr(dw),
                                            None if dbias is None else ptr(dbias), wsp, wss,
                                            stream_ptr(stream)), "conv2d_transpose_grad_filter")
    return dw


PACK_KRSC, PACK_HWIO, PACK_TCONV_FWD, PACK_TCONV_BWD = 0, 1, 2, 3


def wgrad_adam_fusable(desc):
    """Whether seg_conv2d_bwd_filter_adam applies to this conv (bf16, the
    256x256 TN kernel without split-K)."""
    return bool(_lib.lib().seg_conv_wgrad_adam_fusable(ctypes.byref(desc)))


def conv2d_bwd_filter_adam(desc, x, dy, p, m, v, lr, t, beta1=0.9, beta2=0.999, eps=1e-8, grad_scale=1.0,
                           rows=None, tr=None, dw=None, dbias=None, ws=None, stream=None):
    """Filter gradient fused with TF1 Adam on the filter (p, m, v: flat fp32
    slices; rows / tr = (tensor, a_pad, b_pad) packed HWIO / KRSC copies)."""
    d = _with_ld(desc, x, dy)
    a = _lib.SegAdamFused()
    a.p, a.m, a.v = p.data_ptr(), m.data_ptr(), v.data_ptr()
    if rows is not None:
        a.rows_dst, a.rows_ap, a.rows_bp = rows[0].data_ptr(), rows[1], rows[2]
    if tr is not None:
        a.tr_dst, a.tr_ap = tr[0].data_ptr(), tr[1]
    a.lr, a.beta1, a.beta2, a.eps = float(lr), float(beta1), float(beta2), float(eps)
    a.t, a.grad_scale = int(t), float(grad_scale)
    wsp, wss = (ws or Workspace(x.device)).ptr_size(conv_workspace(d, OP_BWD_FILTER))
    check(_lib.lib().seg_conv2d_bwd_filter_adam(ctypes.byref(d), ptr(x), ptr(dy),
                                                None if dw is None else ptr(dw),
                                                None if dbias is None else ptr(dbias), ctypes.byref(a), wsp, wss,
                                                stream_ptr(stream)), "conv2d_backprop_filter_adam")


def pack_filter(src, dst, a_pad, b_pad, mode, stream=None):
    """src fp32 [R,S,A,B] master -> dst packed compute copy (see segkern.h)."""
    R, S, A, B = src.shape
    check(_lib.lib().seg_pack_filter(ptr(src), ptr(dst), R, S, A, B, a_pad, b_pad, mode,
                                     seg_dtype(dst), stream_ptr(stream)), "pack_filter")
    return dst


def tconv_filter_apad(desc):
    """Output-channel extent of the packed tconv filters (modes 2, 3) for this
    descriptor: 8-padded in general, the true channel count on the tap-dense
    path (seg_tconv_filter_apad)."""
    r = int(_lib.lib().seg_tconv_filter_apad(ctypes.byref(desc)))
    if r <= 0:
        raise ValueError("tconv_filter_apad: invalid descriptor")
    return r


def packed_shape(R, S, A, B, mode, a_pad=None):
    a, b = (a_pad if a_pad is not None else round8(A)), round8(B)
    if mode in (PACK_KRSC, PACK_TCONV_BWD):
        return (b, R, S, a)
    return (R, S, a, b)


# ---------------------------------------------------------------------------
# HBM-bound ops
# ---------------------------------------------------------------------------
def bias_relu_bwd(dy, y, dz, dbias, k_valid, relu=True, ws=None, stream=None, scale=1.0):
    N, H, W, K = dy.shape
    P = N * H * W
    need = int(_lib.lib().seg_bias_grad_workspace(P, K))
    wsp, wss = (ws or Workspace(dy.device)).ptr_size(need)
    check(_lib.lib().seg_bias_relu_bwd(ptr(dy), pixel_stride(dy), ptr(y),
                                       pixel_stride(y) if y is not None else 0, ptr(dz),
                                       pixel_stride(dz), ptr(dbias), P, K, k_valid,
                                       1 if relu else 0, float(scale), seg_dtype(dy), wsp, wss,
                                       stream_ptr(stream)), "bias_relu_bwd")
    return dz


def maxpool2x2_fwd(x, y, stream=None):
    N, H, W, C = x.shape
    check(_lib.lib().seg_maxpool2x2_fwd(ptr(x), ptr(y), N, H, W, C, pixel_stride(x),
                                        pixel_stride(y), seg_dtype(x), stream_ptr(stream)),
          "max_pool")
    return y


def maxpool2x2_bwd(x, y, dy, dx, stream=None, relu_mask=False):
    """MaxPoolGrad; relu_mask=True also applies ReluGrad of the post-ReLU input x."""
    N, H, W, C = x.shape
    check(_lib.lib().seg_maxpool2x2_bwd(ptr(x), ptr(y), ptr(dy), ptr(dx), N, H, W, C,
                                        pixel_stride(dx), pixel_stride(dy), 1 if relu_mask else 0,
                                        seg_dtype(x), stream_ptr(stream)), "max_pool_grad")
    return dx


def maxpool_argmax_fits(x):
    N, H, W, C = x.shape
    return N * ((H + 1) // 2) * ((W + 1) // 2) * (C // (4 if x.dtype == torch.float32 else 8)) < 2 ** 31


def maxpool2x2_fwd_argmax(x, y, idx, stream=None):
    """MaxPool that also records its switches (1 byte per pooled element, row
    stride C) for maxpool2x2_bwd_argmax."""
    N, H, W, C = x.shape
    check(_lib.lib().seg_maxpool2x2_fwd_argmax(ptr(x), ptr(y), ptr(idx), N, H, W, C, pixel_stride(x),
                                               pixel_stride(y), seg_dtype(x), stream_ptr(stream)),
          "max_pool")
    return y


def maxpool2x2_bwd_argmax(idx, dy, dx, stream=None, relu_mask=False):
    """MaxPoolGrad from the forward's recorded switches (x not read)."""
    N, H, W, C = dx.shape
    check(_lib.lib().seg_maxpool2x2_bwd_argmax(ptr(idx), ptr(dy), ptr(dx), N, H, W, C, pixel_stride(dx),
                                               pixel_stride(dy), 1 if relu_mask else 0, seg_dtype(dx),
                                               stream_ptr(stream)), "max_pool_grad")
    return dx


def avgpool2x2_fwd(x, y, stream=None):
    N, H, W, C = x.shape
    check(_lib.lib().seg_avgpool2x2_fwd(ptr(x), ptr(y), N, H, W, C, pixel_stride(x),
                                        pixel_stride(y), seg_dtype(x), stream_ptr(stream)),
          "avg_pool")
    return y


def avgpool2x2_bwd(dy, dx, stream=None):
    N, H, W, C = dx.shape
    check(_lib.lib().seg_avgpool2x2_bwd(ptr(dy), ptr(dx), N, H, W, C, pixel_stride(dx),
                                        pixel_stride(dy), seg_dtype(dx), stream_ptr(stream)),
          "avg_pool_grad")
    return dx


def add(a, b, y, stream=None):
    check(_lib.lib().seg_add(ptr(a), ptr(b), ptr(y), y.numel(), seg_dtype(y), stream_ptr(stream)),
          "add")
    return y


def dropout_fwd(x, y, keep_prob, seed, stream=None):
    check(_lib.lib().seg_dropout_fwd(ptr(x), ptr(y), x.numel(), float(keep_prob), int(seed),
                                     seg_dtype(x), stream_ptr(stream)), "dropout")
    return y


def dropout_bwd_ch(dy, dz, c_valid, keep_prob, seed, stream=None):
    """Gradient of a conv-epilogue dropout (counter p * c_valid + c)."""
    C = dy.shape[-1]
    P = dy.numel() // C
    check(_lib.lib().seg_dropout_bwd_ch(ptr(dy), pixel_stride(dy), ptr(dz), pixel_stride(dz), P, C, int(c_valid),
                                        float(keep_prob), int(seed), seg_dtype(dy), stream_ptr(stream)),
          "dropout_grad")
    return dz


def bn_relu_fwd(x, y, gamma, beta, c_valid, relu=True, eps=1e-3, stream=None):
    N, H, W, C = x.shape
    check(_lib.lib().seg_bn_relu_fwd(ptr(x), pixel_stride(x), ptr(y), pixel_stride(y), ptr(gamma),
                                     ptr(beta), float(eps), N * H * W, C, c_valid,
                                     1 if relu else 0, seg_dtype(x), stream_ptr(stream)),
          "batch_norm")
    return y


def bn_relu_bwd(x, y, dy, dx, gamma, dgamma, dbeta, c_valid, relu=True, eps=1e-3, ws=None,
                stream=None, accumulate=False, beta=None, dropout=None):
    """accumulate: dx += the input gradient (dx a slice of a shared concat
    gradient buffer) instead of dx = ...; beta given: the ReLU mask comes from
    x (the forward's arithmetic) and y is not read.  dropout = (keep_prob,
    seed, c_valid) of the conv epilogue that produced x: dx also carries that
    dropout's gradient (seg_bn_relu_dropout_bwd)."""
    N, H, W, C = x.shape
    P = N * H * W
    wsp, wss = (ws or Workspace(x.device)).ptr_size(1024 * 2 * C * 4)
    yp, ldy = (None, 0) if (beta is not None or y is None) else (ptr(y), pixel_stride(y))
    if dropout is not None:
        kp, seed, dcv = dropout
        check(_lib.lib().seg_bn_relu_dropout_bwd(
            ptr(x), pixel_stride(x), yp, ldy, ptr(dy), pixel_stride(dy), ptr(dx), pixel_stride(dx), ptr(gamma),
            None if beta is None else ptr(beta), float(eps), ptr(dgamma), ptr(dbeta), P, C, c_valid,
            (1 if relu else 0) | (2 if accumulate else 0), float(kp), int(seed) & (2 ** 64 - 1), int(dcv),
            seg_dtype(x), wsp, wss, stream_ptr(stream)), "batch_norm_grad")
        return dx
    check(_lib.lib().seg_bn_relu_bwd(ptr(x), pixel_stride(x), yp, ldy, ptr(dy),
                                     pixel_stride(dy), ptr(dx), pixel_stride(dx), ptr(gamma),
                                     None if beta is None else ptr(beta), float(eps), ptr(dgamma), ptr(dbeta), P, C, c_valid,
                                     (1 if relu else 0) | (2 if accumulate else 0), seg_dtype(x), wsp, wss,
                                     stream_ptr(stream)),
          "batch_norm_grad")
    return dx


def resize_bilinear_fwd(x, y, stream=None):
    N, H, W, C = x.shape
    _, OH, OW, _ = y.shape
    check(_lib.lib().seg_resize_bilinear_fwd(ptr(x), ptr(y), N, H, W, C, OH, OW, seg_dtype(x),
                                             stream_ptr(stream)), "resize_bilinear")
    return y


def resize_bilinear_bwd(dy, dx_f32, stream=None):
    N, OH, OW, C = dy.shape
    _, H, W, _ = dx_f32.shape
    check(_lib.lib().seg_resize_bilinear_bwd(ptr(dy), ptr(dx_f32), N, H, W, C, OH, OW,
                                             seg_dtype(dy), stream_ptr(stream)),
          "resize_bilinear_grad")
    return dx_f32


def spatial_reduce(x, y, scale, ws, stream=None):
    """y[n, 0, 0, c] = scale * sum_hw x[n, h, w, c] (x [N,H,W,C], y [N,1,1,C], padded C)."""
    N, H, W, C = x.shape
    assert y.shape[0] == N and y.shape[-1] == C
    wsp, _ = ws.ptr_size(4 * N * C)
    check(_lib.lib().seg_spatial_reduce(ptr(x), pixel_stride(x), ptr(y), N, H, W, C, float(scale),
                                        wsp, seg_dtype(x), stream_ptr(stream)), "spatial_reduce")
    return y


def spatial_broadcast(x, y, scale, stream=None):
    """y[n, h, w, c] = scale * x[n, 0, 0, c] (padded C)."""
    N, H, W, C = y.shape
    assert x.shape[0] == N and x.shape[-1] == C
    check(_lib.lib().seg_spatial_broadcast(ptr(x), ptr(y), pixel_stride(y), N, H, W, C, float(scale),
                                           seg_dtype(y), stream_ptr(stream)), "spatial_broadcast")
    return y


class ConcatPart(ctypes.Structure):
    """seg_concat_part (include/segkern.h)."""
    _fields_ = [("ptr", ctypes.c_void_p), ("ld", ctypes.c_int), ("channels", ctypes.c_int),
                ("accumulate", ctypes.c_int)]


def _parts(items):
    arr = (ConcatPart * len(items))()
    for e, (t, c, acc) in zip(arr, items):
        e.ptr, e.ld, e.channels, e.accumulate = ptr(t), pixel_stride(t), int(c), 1 if acc else 0
    return arr


def concat_fwd(parts, y, channels, stream=None):
    """tf.concat(axis=-1): parts = [(tensor, valid_channels)], y padded [.., round8(sum)]."""
    N, H, W, _ = y.shape
    arr = _parts([(t, c, False) for t, c in parts])
    check(_lib.lib().seg_concat_fwd(arr, len(parts), ptr(y), pixel_stride(y), round8(channels), N * H * W,
                                    seg_dtype(y), stream_ptr(stream)), "concat")
    return y


def concat_bwd(dy, parts, stream=None):
    """Split the concat gradient: parts = [(dst, valid_channels, accumulate)]."""
    N, H, W, _ = dy.shape
    arr = _parts(parts)
    check(_lib.lib().seg_concat_bwd(ptr(dy), pixel_stride(dy), arr, len(parts), N * H * W, seg_dtype(dy),
                                    stream_ptr(stream)), "concat_grad")


def copy_channels(x, y, stream=None):
    N, H, W, C = x.shape
    check(_lib.lib().seg_copy_channels(ptr(x), pixel_stride(x), ptr(y), pixel_stride(y), N * H * W,
                                       round8(C), seg_dtype(x), stream_ptr(stream)), "concat")
    return y


def prepare_input(img, x, stream=None):
    """fp32 or uint8 [N,H,W,c] -> padded compute tensor x [N,HP,WP,CP] (zeros outside)."""
    N, H, W, c = img.shape
    _, HP, WP, CP = x.shape
    fn = _lib.lib().seg_prepare_input_u8 if img.dtype == torch.uint8 else _lib.lib().seg_prepare_input
    if img.dtype not in (torch.uint8, torch.float32):
        raise ValueError(f"prepare_input: unsupported image dtype {img.dtype}")
    check(fn(ptr(img), ptr(x), N, H, W, c, HP, WP, CP, seg_dtype(x), stream_ptr(stream)), "prepare_input")
    return x


def augment(views, C, OH, OW, out, labels=False, stream=None):
    """seg_augment: `views` = [(src uint8 [H0,W0,C] device tensor, (y0, x0, h, w),
    flip, bc, contrast, bright)], out uint8 [n,OH,OW,C] (or [n,OH,OW] labels)."""
    n = len(views)
    arr = (_lib.SegAugView * max(n, 1))()
    for i, (src, (y0, x0, h, w), flip, bc, contrast, bright) in enumerate(views):
        if src.dtype != torch.uint8 or src.dim() != 3 or src.shape[2] != C or not src.is_contiguous():
            raise ValueError("augment: sources must be contiguous uint8 [H, W, C]")
        a = arr[i]
        a.src, a.H0, a.W0 = src.data_ptr(), src.shape[0], src.shape[1]
        a.x0, a.y0, a.w, a.h = x0, y0, w, h
        a.flip, a.bc, a.contrast, a.bright = int(flip), int(bc), float(contrast), int(bright)
    want = (n, OH, OW) if labels else (n, OH, OW, C)
    if tuple(out.shape) != want or out.dtype != torch.uint8 or not out.is_contiguous():
        raise ValueError(f"augment: out must be contiguous uint8 {want}")
    check(_lib.lib().seg_augment(arr, n, C, OH, OW, int(labels), ptr(out), stream_ptr(stream)), "augment")
    return out


def softmax_xent(logits, labels, dlogits, loss_sum, num_classes, valid_hw=None, grad_scale=1.0,
                 ws=None, stream=None):
    N, H, W, _ = logits.shape
    vh, vw = valid_hw if valid_hw is not None else (H, W)
    wsp, wss = (ws or Workspace(logits.device)).ptr_size(
        int(_lib.lib().seg_xent_workspace(N, H, W)))
    L = _lib.lib()
    if labels.dtype == torch.uint8:
        st = L.seg_softmax_xent_fwd_bwd(ptr(logits), pixel_stride(logits), ptr(labels), N, H, W,
                                        num_classes, vh, vw, float(grad_scale), ptr(loss_sum),
                                        ptr(dlogits), pixel_stride(dlogits), seg_dtype(logits),
                                        wsp, wss, stream_ptr(stream))
    else:
        st = L.seg_softmax_xent_soft_fwd_bwd(ptr(logits), pixel_stride(logits), ptr(labels), N, H,
                                             W, num_classes, vh, vw, float(grad_scale),
                                             ptr(loss_sum), ptr(dlogits), pixel_stride(dlogits),
                                             seg_dtype(logits), wsp, wss, stream_ptr(stream))
    check(st, "softmax_cross_entropy_with_logits")
    return loss_sum


def softmax(x, y, num_classes, stream=None):
    """tf.nn.softmax over the (padded) channel dim of NHWC x into y."""
    P = x.numel() // x.shape[-1]
    check(_lib.lib().seg_softmax(ptr(x), pixel_stride(x), int(num_classes), P, ptr(y), pixel_stride(y),
                                 seg_dtype(x), stream_ptr(stream)), "softmax")
    return y


def argmax(logits, pred, num_classes, stream=None):
    N, H, W, _ = logits.shape
    check(_lib.lib().seg_argmax(ptr(logits), pixel_stride(logits), num_classes, N * H * W,
                                ptr(pred), seg_dtype(logits), stream_ptr(stream)), "argmax")
    return pred


def confusion(pred, labels, conf, num_classes, valid_hw=None, stream=None):
    N, H, W = labels.shape[:3]
    vh, vw = valid_hw if valid_hw is not None else (H, W)
    check(_lib.lib().seg_confusion(ptr(pred), ptr(labels), N, H, W, vh, vw, num_classes, ptr(conf),
                                   stream_ptr(stream)), "confusion")
    return conf


def adam_tf1_step(p, g, m, v, lr, t, beta1=0.9, beta2=0.999, eps=1e-8, grad_scale=1.0,
                  stream=None):
    check(_lib.lib().seg_adam_tf1_step(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), float(lr),
                                       float(beta1), float(beta2), float(eps), int(t),
                                       float(grad_scale), stream_ptr(stream)), "adam")


class AdamSegment(ctypes.Structure):
    """seg_adam_segment (include/segkern.h)."""
    _fields_ = [("offset", ctypes.c_longlong), ("rs", ctypes.c_int), ("a", ctypes.c_int), ("b", ctypes.c_int),
                ("tile_begin", ctypes.c_int), ("rows_dst", ctypes.c_void_p), ("rows_ap", ctypes.c_int),
                ("rows_bp", ctypes.c_int), ("tr_dst", ctypes.c_void_p), ("tr_ap", ctypes.c_int),
                ("tr_bp", ctypes.c_int)]


class AdamPlan:
    """Device-resident segment table for adam_tf1_pack.  `segments` is a list of
    (offset, rs, a, b, rows, tr) with rows / tr = (tensor, a_pad, b_pad) or None;
    the tensors are kept alive by the plan."""

    def __init__(self, segments, device):
        arr = (AdamSegment * len(segments))()
        self.keep = []
        for i, (off, rs, a, b, rows, tr) in enumerate(segments):
            e = arr[i]
            e.offset, e.rs, e.a, e.b = off, rs, a, b
            if rows is not None:
                e.rows_dst, e.rows_ap, e.rows_bp = ptr(rows[0]), rows[1], rows[2]
                self.keep.append(rows[0])
            if tr is not None:
                e.tr_dst, e.tr_ap, e.tr_bp = ptr(tr[0]), tr[1], tr[2]
                self.keep.append(tr[0])
        total = _lib.lib().seg_adam_segments_plan(ctypes.byref(arr), len(segments))
        if total <= 0:
            raise ValueError(f"adam segment plan failed ({total})")
        self.total_tiles = total
        self.nsegs = len(segments)
        raw = bytes(memoryview(arr).cast("B"))
        self.table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)


def adam_tf1_pack(p, g, m, v, plan, lr, t, beta1=0.9, beta2=0.999, eps=1e-8, grad_scale=1.0,
                  dtype=BF16, stream=None):
    """TF1 Adam over every planned variable + packed compute copies (one launch)."""
    check(_lib.lib().seg_adam_tf1_pack(ptr(p), ptr(g), ptr(m), ptr(v), ptr(plan.table), plan.nsegs,
                                       plan.total_tiles, float(lr), float(beta1), float(beta2), float(eps),
                                       int(t), float(grad_scale), int(dtype), stream_ptr(stream)), "adam_pack")


def pack_segments(p, plan, dtype=BF16, stream=None):
    """Rewrite every planned variable's packed compute copies from p (no update)."""
    check(_lib.lib().seg_pack_segments(ptr(p), ptr(plan.table), plan.nsegs, plan.total_tiles, int(dtype),
                                       stream_ptr(stream)), "pack_segments")


def cast(x, y, stream=None):
    """Elementwise dtype conversion x -> y (same number of elements)."""
    assert x.numel() == y.numel()
    check(_lib.lib().seg_cast(ptr(x), seg_dtype(x), ptr(y), seg_dtype(y), x.numel(), stream_ptr(stream)), "cast")
    return y


def check_finite(g, flag, stream=None):
    """flag (int32 device scalar) = 1 if g holds an Inf / NaN."""
    check(_lib.lib().seg_check_finite(ptr(g), g.numel(), ptr(flag), stream_ptr(stream)), "check_finite")
    return flag


def axpy(y, x, alpha, stream=None):
    """y += alpha * x (fp32, same number of elements)."""
    assert y.dtype == torch.float32 and x.dtype == torch.float32 and y.numel() == x.numel()
    check(_lib.lib().seg_axpy(ptr(y), ptr(x), float(alpha), y.numel(), stream_ptr(stream)), "axpy")
    return y


def fill(y, value, stream=None):
    check(_lib.lib().seg_fill(ptr(y), y.numel(), float(value), seg_dtype(y), stream_ptr(stream)),
          "fill")
    return y
