"""Op-level parity of the round-2 C-ABI entry points against plain torch
fp32 references: seg_spatial_reduce / seg_spatial_broadcast (global average
pooling and the 1x1 -> HxW align_corners resize of DeepLab's image-pooling
branch, Network/model/DeepLabv3Plus.py:215-225) and seg_axpy (the
accumulate template's assign_add, Network/main.py:92-95).
Tolerances: fp32 sums 1e-5 relative; bf16 outputs one bf16 rounding (4e-3)."""
import numpy as np
import pytest
import torch

from oracle import tf1_ops as T
from semanticsegmentation_tensorflow_amd import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 7, 9, 8), (1, 128, 256, 512), (3, 1, 1, 24), (2, 33, 5, 2048)])
def test_spatial_reduce_mean_and_sum(dev, dtype, shape):
    if dtype == torch.float32 and shape[3] > 1024:
        pytest.skip("fp32 chunks: C <= 1024")
    N, H, W, C = shape
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(dtype)
    y = torch.empty(N, 1, 1, C, device=dev, dtype=dtype)
    ws = ops.Workspace(dev)
    for scale in (1.0 / (H * W), 1.0):
        ops.spatial_reduce(x, y, scale, ws)
        ref = x.float().sum(dim=(1, 2), keepdim=True) * scale
        tol = 1e-5 if dtype == torch.float32 else 4e-3
        err = (y.float() - ref).abs().max().item()
        assert err <= tol * ref.abs().max().item() + 1e-6, err
    # the oracle's align_corners resize from 1x1 is a broadcast; its gradient a spatial sum
    xo = torch.randn(N, 1, 1, C, dtype=torch.float64, requires_grad=True)
    yo = T.resize_bilinear(xo, (H, W))
    assert torch.equal(yo, xo.expand(N, H, W, C))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_spatial_broadcast(dev, dtype):
    N, H, W, C = 2, 17, 30, 256
    x = torch.randn(N, 1, 1, C, device=dev).to(dtype)
    full = torch.zeros(N, H, W, C + 16, device=dev, dtype=dtype)
    y = full[..., :C]                                  # strided destination (pixel stride C + 16)
    ops.spatial_broadcast(x, y, 0.25)
    ref = (x.float() * 0.25).expand(N, H, W, C)
    assert (y.float() - ref).abs().max().item() <= 4e-3 * ref.abs().max().item()
    assert full[..., C:].abs().max().item() == 0.0


def test_axpy(dev):
    n = 1_000_003
    y = torch.randn(n, device=dev)
    x = torch.randn(n, device=dev)
    ref = y + 1.5 * x
    ops.axpy(y, x, 1.5)
    np.testing.assert_allclose(y.cpu().numpy(), ref.cpu().numpy(), rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------------------------
# A-operand prologue (frozen BN + ReLU folded into the consuming conv):
# seg_conv2d_fwd_pro / seg_conv2d_bwd_filter_pro vs the oracle's
# conv2d(relu(batch_norm_frozen(x))) (Network/model/FCDenseNet.py:25-28)
# ---------------------------------------------------------------------------
from tests.gpu_utils import assert_close, from_dev, rnd, to_dev  # noqa: E402

# 1x1 cases run the LDS-DMA prologue kernels in 16-bit (igemm_nt2 192x64 / 192x128,
# igemm_tn2 at any channel count), 3x3 ones the register-staged kernels
PRO_CASES = [(2, 9, 11, 48, 64, 1), (1, 12, 10, 136, 64, 1), (1, 7, 9, 16, 24, 3), (2, 16, 20, 64, 16, 3),
             (1, 33, 41, 200, 136, 1), (2, 20, 30, 520, 64, 1), (1, 17, 19, 24, 8, 1)]
PRO_DT = {torch.float32: ops.F32, torch.bfloat16: ops.BF16, torch.float16: ops.F16}


def _pro_case(case, dtype, dev):
    N, H, W, C, K, R = case
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    w = torch.randn(R, R, C, K, generator=g, dtype=torch.float64) / np.sqrt(R * R * C)
    gamma = (1.0 + 0.3 * torch.randn(C, generator=g)).float()
    beta = (0.5 * torch.randn(C, generator=g)).float()
    xr, wr = rnd(x, dtype), rnd(w, dtype)
    # the device's BN output in the compute dtype (what the materialised path stores)
    a = rnd(T.relu(T.batch_norm_frozen(xr, gamma.double(), beta.double())), dtype)
    return x, w, gamma, beta, xr, wr, a


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", PRO_CASES)
def test_conv2d_fwd_with_bn_relu_prologue(dev, case, dtype):
    N, H, W, C, K, R = case
    x, w, gamma, beta, xr, wr, a = _pro_case(case, dtype, dev)
    ref = T.conv2d(a, wr)                                   # zero SAME padding of the BN output
    d = ops.conv_desc(N, H, W, C, K, R, R, 1, 1, "SAME", PRO_DT[dtype])
    wk = torch.empty(ops.packed_shape(R, R, C, K, ops.PACK_KRSC), dtype=dtype, device=dev)
    ops.pack_filter(w.float().to(dev).contiguous(), wk, ops.round8(C), ops.round8(K), ops.PACK_KRSC)
    y = torch.empty(N, H, W, d.K, dtype=dtype, device=dev)
    gd, bd = gamma.to(dev), beta.to(dev)
    ops.conv2d_fwd_pro(d, to_dev(x, dtype, dev), ops.prologue(gd, bd), wk, y)
    torch.cuda.synchronize()
    assert_close(from_dev(y, K), ref, dtype, f"conv fwd pro {case}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", PRO_CASES)
def test_conv2d_bwd_filter_with_bn_relu_prologue(dev, case, dtype):
    N, H, W, C, K, R = case
    x, w, gamma, beta, xr, wr, a = _pro_case(case, dtype, dev)
    g = torch.Generator().manual_seed(8)
    dy = rnd(torch.randn(N, H, W, K, generator=g, dtype=torch.float64), dtype)
    wv = wr.clone().requires_grad_(True)
    T.conv2d(a, wv).backward(dy)
    d = ops.conv_desc(N, H, W, C, K, R, R, 1, 1, "SAME", PRO_DT[dtype])
    dw = torch.zeros(R, R, C, K, device=dev)
    ops.conv2d_bwd_filter_pro(d, to_dev(x, dtype, dev), ops.prologue(gamma.to(dev), beta.to(dev)),
                              to_dev(dy, dtype, dev), dw)
    torch.cuda.synchronize()
    tol = 2e-5 if dtype == torch.float32 else 2e-3
    assert_close(dw.double().cpu(), wv.grad, torch.float32, f"conv wgrad pro {case}", tol)


# input gradient of the same folded convs carried through the BN(+ReLU)
# backward (seg_conv2d_bwd_data_bn) vs float64: dL/dx, dgamma, dbeta
BNB_CASES = [(2, 9, 11, 48, 64, 1), (1, 12, 10, 136, 64, 1), (1, 33, 41, 200, 136, 1), (2, 20, 30, 520, 64, 1),
             (1, 17, 19, 24, 8, 1), (2, 40, 52, 112, 64, 1)]


@pytest.fixture(params=[1, 0], ids=["stream", "bm256"])
def nt2bn_bm(request):
    """Both 1x1 forms: bn1x1_stream (K = 64; option bn1x1s) and igemm_nt2_bn
    (256-row tiles)."""
    ops.set_option("bn1x1s", request.param)
    yield request.param
    ops.set_option("bn1x1s", 1)


@pytest.mark.parametrize("accumulate", [False, True], ids=["write", "accumulate"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", BNB_CASES)
def test_conv2d_bwd_data_through_bn_relu(dev, case, dtype, accumulate, nt2bn_bm):
    N, H, W, C, K, R = case
    x, w, gamma, beta, xr, wr, a = _pro_case(case, dtype, dev)
    g = torch.Generator().manual_seed(9)
    dy = rnd(torch.randn(N, H, W, K, generator=g, dtype=torch.float64), dtype)
    # float64: a = relu(BN(x)), y = conv(a); backprop dy to x, gamma, beta
    xv = xr.clone().requires_grad_(True)
    gv, bv = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    av = T.relu(T.batch_norm_frozen(xv, gv, bv))
    T.conv2d(av, wr).backward(dy)
    d = ops.conv_desc(N, H, W, C, K, R, R, 1, 1, "SAME", PRO_DT[dtype])
    assert ops.conv_bwd_data_bn_workspace(d) > 0
    wh = torch.zeros(ops.packed_shape(R, R, C, K, ops.PACK_HWIO), dtype=dtype, device=dev)
    ops.pack_filter(w.float().to(dev).contiguous(), wh, ops.round8(C), ops.round8(K), ops.PACK_HWIO)
    # the input gradient lands in a channel slice of a wider buffer (concat gradient)
    old = rnd(torch.randn(N, H, W, C + 16, generator=g, dtype=torch.float64), dtype)
    wide = to_dev(old, dtype, dev) if accumulate else torch.full((N, H, W, C + 16), float("nan"), dtype=dtype,
                                                                   device=dev)
    dx = wide[..., 8:8 + C]
    dg, db = torch.full((C,), float("nan"), device=dev), torch.full((C,), float("nan"), device=dev)
    ops.conv2d_bwd_data_bn(d, to_dev(dy, dtype, dev), wh, to_dev(x, dtype, dev), gamma.to(dev), beta.to(dev), dx,
                           dg, db, accumulate=accumulate)
    torch.cuda.synchronize()
    want = xv.grad + (old[..., 8:8 + C] if accumulate else 0.0)
    assert_close(from_dev(wide[..., 8:8 + C].contiguous(), C), want, dtype, f"bn-dgrad dx {case}")
    if accumulate:   # the neighbouring channels of the shared buffer are untouched
        assert torch.equal(wide[..., :8].cpu(), to_dev(old, dtype, dev)[..., :8].cpu())
    assert_close(dg.double().cpu(), gv.grad, torch.float32, f"bn-dgrad dgamma {case}", 2e-3)
    assert_close(db.double().cpu(), bv.grad, torch.float32, f"bn-dgrad dbeta {case}", 2e-3)


# the 3x3 form (FC-DenseNet growth conv, 64 -> 16): the input gradient runs on
# conv_res16c and continues through the BN(+ReLU) that produced the conv's
# input and, with keep_prob < 1, the dropout of the conv before that BN; every
# tile height of the kernel (option res16c_bh: 8, 4 = the default)
BNB3_CASES = [(2, 21, 67, 64, 16), (1, 30, 70, 64, 16), (2, 9, 11, 32, 16)]


@pytest.fixture(params=[(4, 0), (8, 0), (4, 1), (8, 1)], ids=["bh4", "bh8", "bh4st", "bh8st"])
def res16c_bh(request):
    """Tile heights (option res16c_bh) and the staged 16-byte dx stores
    (option res16c_st)."""
    ops.set_option("res16c_bh", request.param[0])
    ops.set_option("res16c_st", request.param[1])
    yield request.param
    ops.set_option("res16c_bh", 4)
    ops.set_option("res16c_st", 1)


@pytest.mark.parametrize("kp", [1.0, 0.6], ids=["no-dropout", "dropout"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", BNB3_CASES)
def test_conv3x3_bwd_data_through_bn_relu_dropout(dev, case, dtype, kp, res16c_bh):
    from tests.test_gpu_ops import _np_uniform
    N, H, W, C, K = case
    x, w, gamma, beta, xr, wr, a = _pro_case((N, H, W, C, K, 3), dtype, dev)
    g = torch.Generator().manual_seed(10)
    dy = rnd(torch.randn(N, H, W, K, generator=g, dtype=torch.float64), dtype)
    xv = xr.clone().requires_grad_(True)
    gv, bv = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    T.conv2d(T.relu(T.batch_norm_frozen(xv, gv, bv)), wr).backward(dy)
    seed = 12345
    want = xv.grad
    if kp < 1.0:
        P = N * H * W
        u = np.array([[_np_uniform(seed, p * C + c) for c in range(C)] for p in range(P)], np.float32)
        mask = torch.from_numpy(np.floor(np.float32(kp) + u).astype(np.float64)).view(N, H, W, C)
        want = want / kp * mask
    d = ops.conv_desc(N, H, W, C, K, 3, 3, 1, 1, "SAME", PRO_DT[dtype])
    assert ops.conv_bwd_data_bn_workspace(d) > 0
    wh = torch.zeros(ops.packed_shape(3, 3, C, K, ops.PACK_HWIO), dtype=dtype, device=dev)
    ops.pack_filter(w.float().to(dev).contiguous(), wh, ops.round8(C), ops.round8(K), ops.PACK_HWIO)
    dx = torch.full((N, H, W, C), float("nan"), dtype=dtype, device=dev)
    dg, db = torch.full((C,), float("nan"), device=dev), torch.full((C,), float("nan"), device=dev)
    ops.conv2d_bwd_data_bn(d, to_dev(dy, dtype, dev), wh, to_dev(x, dtype, dev), gamma.to(dev), beta.to(dev), dx,
                           dg, db, dropout=(kp, seed) if kp < 1.0 else None)
    torch.cuda.synchronize()
    assert_close(from_dev(dx, C), want, dtype, f"bn3-dgrad dx {case}")
    assert_close(dg.double().cpu(), gv.grad, torch.float32, f"bn3-dgrad dgamma {case}", 2e-3)
    assert_close(db.double().cpu(), bv.grad, torch.float32, f"bn3-dgrad dbeta {case}", 2e-3)


# the streaming 1x1 kernel (conv1x1_stream: FC-DenseNet bottleneck convs,
# C <= 256 -> N <= 64) vs float64, with the bottleneck's dropout epilogue,
# the input as a channel slice of a wider concat buffer, pixel counts that
# leave ragged last tiles and give most blocks several tiles
S1_CASES = [(2, 130, 140, 48, 64), (1, 50, 61, 256, 64), (1, 40, 70, 112, 56), (2, 33, 35, 8, 16),
            (3, 97, 131, 200, 64)]


def _np_uniform_vec(seed, idx):
    """tests.test_gpu_ops._np_uniform over a uint64 index array (same hash)."""
    from tests.test_gpu_ops import _np_avalanche32
    M = np.uint64(0xFFFFFFFF)
    key = np.uint64(_np_avalanche32(((seed ^ (seed >> 32)) & 0xFFFFFFFF) ^ 0x632BE59B))
    idx = np.asarray(idx, dtype=np.uint64)
    q, j = idx >> np.uint64(3), idx & np.uint64(7)
    x = ((q & M) ^ (((q >> np.uint64(32)) * np.uint64(0x85EBCA6B)) & M)) & M
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M
    x ^= key
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M
    x ^= x >> np.uint64(16)
    x = (x + j * np.uint64(0x9E3779B9)) & M
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M
    x ^= x >> np.uint64(15)
    return ((x >> np.uint64(8)).astype(np.float64) / 16777216.0).astype(np.float32)


@pytest.fixture(params=[0, 2], ids=["st8", "st16"])
def s1x1_st(request):
    """conv1x1_stream's direct 8-byte and staged 16-byte stores (option s1x1_st)."""
    ops.set_option("s1x1_st", request.param)
    yield request.param
    ops.set_option("s1x1_st", 1)


@pytest.mark.parametrize("kp", [1.0, 0.2], ids=["no-dropout", "dropout"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", S1_CASES)
def test_conv1x1_stream_bn_relu_dropout(dev, case, dtype, kp, s1x1_st):
    from tests.test_gpu_ops import _np_uniform
    N, H, W, C, K = case
    x, w, gamma, beta, xr, wr, a = _pro_case((N, H, W, C, K, 1), dtype, dev)
    seed = 4242
    ref = T.conv2d(a, wr)
    if kp < 1.0:
        u = _np_uniform_vec(seed, np.arange(N * H * W * K, dtype=np.uint64))
        assert u[123] == np.float32(_np_uniform(seed, 123))
        mask = torch.from_numpy(np.floor(np.float32(kp) + u).astype(np.float64)).view(N, H, W, K)
        ref = ref / kp * mask
    d = ops.conv_desc(N, H, W, C, K, 1, 1, 1, 1, "SAME", PRO_DT[dtype])
    assert ops.conv_kernel_info(d, ops.OP_FWD_PRO)[0].startswith("conv1x1_stream")
    wk = torch.empty(ops.packed_shape(1, 1, C, K, ops.PACK_KRSC), dtype=dtype, device=dev)
    ops.pack_filter(w.float().to(dev).contiguous(), wk, ops.round8(C), ops.round8(K), ops.PACK_KRSC)
    wide = torch.zeros(N, H, W, C + 24, dtype=dtype, device=dev)
    wide[..., 16:16 + C] = to_dev(x, dtype, dev)
    y = torch.full((N, H, W, d.K), float("nan"), dtype=dtype, device=dev)
    epi = ops.epilogue(keep_prob=kp, seed=seed) if kp < 1.0 else None
    ops.conv2d_fwd_pro(d, wide[..., 16:16 + C], ops.prologue(gamma.to(dev), beta.to(dev)), wk, y, epi)
    torch.cuda.synchronize()
    assert_close(from_dev(y, K), ref, dtype, f"conv1x1_stream {case}")
    if kp < 1.0:   # the dropped positions are exactly the oracle's
        got = from_dev(y, K)
        assert bool((got[mask == 0] == 0).all())
        assert bool((mask[(got == 0) & (ref.abs() > 1e-3)] == 0).all())


# N = 256 k + a tail <= 128 on igemm_nt3 + igemm_nt2 (nt_nsplit): forward with
# bias + ReLU, and the input gradient with the ReluGrad mask, vs the float64
# oracle; the 256-aligned head is the same igemm_nt3 launch either way.
@pytest.mark.parametrize("C,K,op", [(256, 320, "fwd"), (256, 352, "fwd"), (320, 256, "bwd_data"),
                                    (560, 256, "bwd_data")])
def test_nt_nsplit_head_tail(dev, C, K, op):
    N, H, W = 2, 96, 96
    dtype = torch.bfloat16
    g = torch.Generator().manual_seed(31)
    d = ops.conv_desc(N, H, W, C, K, 1, 1, 1, 1, "SAME", ops.BF16)
    x64 = torch.randn(N, H, W, C, generator=g, dtype=torch.float64)
    w64 = torch.randn(1, 1, C, K, generator=g, dtype=torch.float64) / C ** 0.5
    dy64 = torch.randn(N, H, W, K, generator=g, dtype=torch.float64)
    mask64 = torch.relu(torch.randn(N, H, W, C, generator=g, dtype=torch.float64))
    b = (torch.randn(K, generator=g) * 0.1).to(dev)
    ws = ops.Workspace(dev)
    outs = {}
    for ns in (0, 1):
        ops.set_option("nt_nsplit", ns)
        try:
            if op == "fwd":
                name = ops.conv_kernel_info(d, ops.OP_FWD)[0]
                wk = torch.empty(ops.packed_shape(1, 1, C, K, ops.PACK_KRSC, C), dtype=dtype, device=dev)
                ops.pack_filter(w64.float().to(dev), wk, C, K, ops.PACK_KRSC)
                y = torch.full((N, H, W, K), float("nan"), dtype=dtype, device=dev)
                ops.conv2d_fwd(d, x64.to(dev, dtype), wk, y, ops.epilogue(bias=b, relu=True), ws)
            else:
                name = ops.conv_kernel_info(d, ops.OP_BWD_DATA)[0]
                wh = torch.empty(ops.packed_shape(1, 1, C, K, ops.PACK_HWIO, C), dtype=dtype, device=dev)
                ops.pack_filter(w64.float().to(dev), wh, C, K, ops.PACK_HWIO)
                y = torch.full((N, H, W, C), float("nan"), dtype=dtype, device=dev)
                ops.conv2d_bwd_data(d, dy64.to(dev, dtype), wh, y, ws, epi=ops.epilogue(relu_mask=mask64.to(dev, dtype)))
            torch.cuda.synchronize()
        finally:
            ops.set_option("nt_nsplit", 1)
        assert name.startswith("igemm_nt3"), name
        outs[ns] = y.clone()
    assert torch.equal(outs[0][..., :256], outs[1][..., :256])
    xr, wr = x64.to(dtype).double(), w64.to(dtype).double()
    if op == "fwd":
        ref = torch.relu(T.conv2d(xr, wr, 1, "SAME", 1) + b.double().cpu())
    else:
        xa = torch.zeros(N, H, W, C, dtype=torch.float64, requires_grad=True)
        (T.conv2d(xa, wr, 1, "SAME", 1) * dy64.to(dtype).double()).sum().backward()
        ref = torch.where(mask64.to(dtype).double() > 0, xa.grad, torch.zeros_like(xa.grad))
    for ns in (0, 1):
        got = outs[ns].double().cpu()
        err = (got - ref).abs().max().item() / ref.abs().max().item()
        assert err < 1.2e-2, (ns, err)
