"""Debug: tap-dense tconv forward intermediate Z vs torch (bf16/f32, nt variants)."""
import sys
import torch
sys.path.insert(0, ".")
from semanticsegmentation_tensorflow_amd import ops
from oracle import tf1_ops as tf

dev = torch.device("cuda:0")
N, IH, IW, Ci, OH, OW, Co, k, s = 1, 2, 3, 16, 16, 24, 2, 16, 8
g = torch.Generator().manual_seed(4)
x = torch.randn(N, IH, IW, Ci, generator=g, dtype=torch.float64)
w = torch.randn(k, k, Co, Ci, generator=g, dtype=torch.float64) / 8
for v in (1, 2):
    ops.set_option("igemm_nt_variant", v)
    for dt, tdt in ((ops.F32, torch.float32), (ops.BF16, torch.bfloat16)):
        d = ops.tconv_desc(N, IH, IW, Ci, OH, OW, Co, k, k, s, "SAME", dt)
        ap = ops.tconv_filter_apad(d)
        wp = torch.empty(ops.packed_shape(k, k, Co, Ci, ops.PACK_TCONV_FWD, ap), dtype=tdt, device=dev)
        ops.pack_filter(w.float().to(dev).contiguous(), wp, ap, 16, ops.PACK_TCONV_FWD)
        xd = torch.zeros(N, IH, IW, 16, dtype=tdt, device=dev)
        xd[..., :Ci] = x.to(tdt).to(dev)
        y = torch.zeros(N, OH, OW, 8, dtype=tdt, device=dev)
        ws = ops.Workspace(dev)
        ops.tconv2d_fwd(d, xd, wp, y, None, ws)
        torch.cuda.synchronize()
        Z = ws.buf[: N * IH * IW * 512 * (2 if tdt == torch.bfloat16 else 4)].view(tdt).view(N * IH * IW, 512).double().cpu()
        xr = x.to(tdt).double().reshape(-1, Ci)
        wr = w.to(tdt).double().reshape(k * k * Co, Ci)
        Zr = xr @ wr.T
        ez = (Z - Zr).abs().max().item() / Zr.abs().max().item()
        ref = tf.conv2d_transpose(x.to(tdt).double(), w.to(tdt).double(), (N, OH, OW, Co), s)
        ey = (y[..., :Co].double().cpu() - ref).abs().max().item() / ref.abs().max().item()
        wpd = wp.double().cpu().reshape(k * k * ap, 16)[:, :Ci]
        ew = (wpd - wr).abs().max().item()
        print(f"variant {v} {tdt}: Z rel err {ez:.3e}  y rel err {ey:.3e}  pack err {ew:.3e}")
        if ez > 1e-2:
            bad = ((Z - Zr).abs() > 1e-2 * Zr.abs().max()).nonzero()
            print("bad entries", bad[:10].tolist(), len(bad))

# exact replica of tests/test_gpu_ops.py::test_tconv2d_fwd_bias_residual case 3, bf16
import math
from tests.gpu_utils import to_dev, from_dev, rnd, rel_err
for v in (1, 2):
    ops.set_option("igemm_nt_variant", v)
    for tdt in (torch.float32, torch.bfloat16):
        g = torch.Generator().manual_seed(4)
        x = torch.randn(N, IH, IW, Ci, generator=g, dtype=torch.float64)
        w = torch.randn(k, k, Co, Ci, generator=g, dtype=torch.float64) / math.sqrt(Ci * 4)
        b = torch.randn(Co, generator=g, dtype=torch.float64) * 0.1
        g = torch.Generator().manual_seed(5)
        res = rnd(torch.randn(N, OH, OW, Co, generator=g, dtype=torch.float64), tdt)
        ref0 = tf.conv2d_transpose(rnd(x, tdt), rnd(w, tdt), (N, OH, OW, Co), s)
        ref = ref0 + b.float().double() + res
        d = ops.tconv_desc(N, IH, IW, Ci, OH, OW, Co, k, k, s, "SAME", ops.F32 if tdt == torch.float32 else ops.BF16)
        ap = ops.tconv_filter_apad(d)
        wp = torch.empty(ops.packed_shape(k, k, Co, Ci, ops.PACK_TCONV_FWD, ap), dtype=tdt, device=dev)
        ops.pack_filter(w.float().to(dev).contiguous(), wp, ap, 16, ops.PACK_TCONV_FWD)
        for mode in ("none", "bias", "res", "both"):
            y = torch.full((N, OH, OW, d.K), float("nan"), dtype=tdt, device=dev)
            resd = to_dev(res, tdt, dev)
            epi = None if mode == "none" else ops.epilogue(bias=b.float().to(dev) if mode in ("bias", "both") else None,
                                                           residual=resd if mode in ("res", "both") else None)
            ops.tconv2d_fwd(d, to_dev(x, tdt, dev), wp, y, epi)
            torch.cuda.synchronize()
            r = ref0 + (b.float().double() if mode in ("bias", "both") else 0) + (res if mode in ("res", "both") else 0)
            print(v, tdt, mode, f"{rel_err(from_dev(y, Co), r):.3e}")

ops.set_option("igemm_nt_variant", 2)
tdt = torch.float32
d = ops.tconv_desc(N, IH, IW, Ci, OH, OW, Co, k, k, s, "SAME", ops.F32)
y = torch.full((N, OH, OW, d.K), float("nan"), dtype=tdt, device=dev)
bb = torch.tensor([1.0, 2.0], device=dev)
e = ops.epilogue(bias=bb)
print("epi fields", [(f[0], getattr(e, f[0])) for f in e._fields_][:6])
ops.tconv2d_fwd(d, to_dev(x, tdt, dev), wp.float() if wp.dtype != tdt else wp, y, e)
ops.tconv2d_fwd(d, to_dev(x, tdt, dev), wp.float(), y, e)
torch.cuda.synchronize()
y0 = torch.full((N, OH, OW, d.K), float("nan"), dtype=tdt, device=dev)
ops.tconv2d_fwd(d, to_dev(x, tdt, dev), wp.float(), y0, None)
torch.cuda.synchronize()
diff = (y - y0)[0].cpu()
print("bias added ch0 unique", diff[..., 0].unique()[:10].tolist())
print("bias added ch1 unique", diff[..., 1].unique()[:10].tolist())
