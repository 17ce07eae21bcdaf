"""GPU diagnostic (not collected by pytest): layer-by-layer comparison of the
bf16 device path against the oracle with bf16-emulated forward rounding.
    python tests/diag_bf16.py"""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from oracle import models as M, tf1_ops as T
from semanticsegmentation_tensorflow_amd import tf
from tests.model_inputs import he_weights, synthetic_batch
from tests.test_gpu_fcn import build_fcn

N, H, W = 2, 64, 96
q = lambda t: t.to(torch.bfloat16).to(torch.float64)
shapes = M.fcn_param_shapes(3, 2)
wts = he_weights(shapes, 1)
img, lab = synthetic_batch(N, H, W, 2)
dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"

# ---- oracle with hooks on every conv pre-activation
wref = {k: (torch.from_numpy(v).bfloat16().double() if (v.ndim == 4 and dt == "bf16") else torch.from_numpy(v).double()).requires_grad_(True) for k, v in wts.items()}
zs, acts = {}, {}
def conv_layer(x, name):
    z = T.bias_add(T.conv2d(x, wref[f"{name}/weights"]), wref[f"{name}/biases"])
    z.retain_grad(); zs[name] = z
    a = T.relu(z)
    return q(a) if dt == "bf16" else a
h = torch.from_numpy(img).double()
for name, _, _ in M.FCN_CONVS[:14]:
    h = conv_layer(h, name); acts[name] = h
    if name in M.POOL_AFTER:
        h = T.max_pool2x2(h); acts[M.POOL_AFTER[name]] = h
h = conv_layer(h, "conv6"); acts["conv6"] = h
h = conv_layer(h, "conv7"); acts["conv7"] = h
c8 = conv_layer(h, "conv8"); acts["conv8"] = c8
def deconv(x, name, shp, res):
    z = T.bias_add(T.conv2d_transpose(x, wref[f"{name}/weights"], shp, 2), wref[f"{name}/biases"]) + res
    z.retain_grad(); zs[name] = z
    return q(z) if dt == "bf16" else z
f1 = deconv(c8, "conv_t1", tuple(acts["pool4"].shape), acts["pool4"]); acts["conv_t1"] = f1
f2 = deconv(f1, "conv_t2", tuple(acts["pool3"].shape), acts["pool3"]); acts["conv_t2"] = f2
lg = T.bias_add(T.conv2d_transpose(f2, wref["conv_t3/weights"], (N, H, W, 2), 8), wref["conv_t3/bias"])
lg = q(lg) if dt == "bf16" else lg
lg.retain_grad()
loss = T.mean_softmax_xent(lg, T.one_hot(torch.from_numpy(lab), 2))
loss.backward()

# ---- device
image, labels, keep, pred, logits, loss_t, train_step = build_fcn(H, W)
sess = tf.Session(compute_dtype=dt)
sess.run(tf.global_variables_initializer())
for k, v in wts.items():
    sess.assign(k, v)
sess.run([loss_t, train_step], feed_dict={image: img, labels: lab, keep: 1.0})
plan = [p for p in sess.plans.values() if p.train][0]
names = [n for n, _, _ in M.FCN_CONVS] + ["conv8"]
convs = [n for n in plan.nodes if n.kind == "conv"]
tconvs = [n for n in plan.nodes if n.kind == "tconv"]
def rl2(a, b):
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
print("loss dev/oracle", sess.run(loss_t, feed_dict={image: img, labels: lab, keep: 1.0}), loss.item())
for nm, n in list(zip(names, convs)) + list(zip(["conv_t1", "conv_t2"], tconvs)):
    C = plan.shapes[id(n.output)][3]
    y = plan.buf[id(n.output)][..., :C].double().cpu().numpy()
    ya = acts[nm].detach().numpy()
    dz_key = ("dz", id(n.output))
    if n.kind == "conv" and dz_key in plan.tmp:
        dz = plan.tmp[dz_key][..., :C].double().cpu().numpy()
    else:
        dz = None
    # oracle d(loss)/dz  (z = pre-relu); device dz = dy*(y>0) -> same quantity
    gz = zs[nm].grad.numpy() if zs[nm].grad is not None else None
    msg = f"{nm:8s} fwd relL2={rl2(y, ya):.2e} |y|={np.linalg.norm(ya):.3e}"
    if dz is not None and gz is not None:
        msg += f"  dz relL2={rl2(dz, gz):.2e} |dz|={np.linalg.norm(gz):.3e}"
        flips = ((y > 0) != (ya > 0)).mean()
        msg += f" reluflip={flips:.2e}"
    print(msg)
