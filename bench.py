#!/usr/bin/env python
"""Headline benchmark: FCN training images/sec on synthetic KITTI-shaped
375x1242 2-class batches (BASELINE.json config C2 at N=1, C4 for N>1).

One "step" = one sess.run(train_step) of the reference's FCN.py training
graph (forward, softmax-xent loss, backward, TF1 Adam on all 138.9 M
parameters) over a batch of 4 images per GPU that are already resident in
HBM.  375x1242 is zero-padded to 384x1248 (the reference cannot run
375x1242 through FCN); the loss is masked to 375x1242; FLOPs
are counted at the executed shape.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

Rank 0 prints ONE JSON line.  Extra objects: "roofline" (dominant kernel,
HIP-event timed inside this run) and "cpu_baseline" (the CPU oracle
restatement timed on this host's cores, N=1 only).
"""
import argparse
import json
import os
import re
import sys
import time

# HIP hardware queues per process: left as the environment sets them (the GPU
# box exports GPU_MAX_HW_QUEUES=4, HIP's own default); the value in effect is
# recorded in the result line.  The Session's stream layout is sized for 4
# (DESIGN.md section 6).
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "train images/sec on KITTI 375×1242 2-class at 1/2/4/8 MI355X; mIoU parity"
PEAK = {"bf16": 2.5e15, "f16": 2.5e15, "f32": 157.3e12}   # dense MFMA peaks (MI355X_MICROARCH.md)
DEFAULT_DTYPE = {"fcn": "bf16", "fcdensenet": "bf16", "deeplab": "f16"}   # C5: "fp16 with fp32 accum"
HBM_PEAK = 8.0e12                                  # HBM3E bytes/s (MI355X_MICROARCH.md)
FCN_TRAIN_FLOP_PER_IMG = 1348.97e9                 # SURVEY.md 8d at 384x1248, C_in=3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); default 1, or WORLD_SIZE when started by torchrun")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="fcn", choices=["fcn", "fcdensenet", "deeplab"],
                    help="fcn = config C2/C4 (headline); fcdensenet = config C3 (U-Net); "
                         "deeplab = config C5 (atrous + ASPP + bilinear, 1024x2048 Cityscapes-shaped)")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (fcn 4, fcdensenet 8, deeplab 2)")
    ap.add_argument("--height", type=int, default=None, help="375 (KITTI); deeplab 1024")
    ap.add_argument("--width", type=int, default=None, help="1242 (KITTI); deeplab 2048")
    ap.add_argument("--dtype", default=None, choices=["bf16", "f16", "f32"],
                    help="compute dtype (default: bf16; f16 + dynamic loss scaling for --model deeplab, config C5)")
    ap.add_argument("--keep-prob", type=float, default=None,
                    help="fcn 0.8 (FCN.py:395), fcdensenet 0.2 (FCDenseNet.py:13)")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--dp-mode", default="allreduce", choices=["allreduce", "zero"],
                    help="gradient exchange at N > 1: all-reduce + every rank's Adam (default: the shorter "
                         "post-backward critical path, DESIGN.md section 6) or ZeRO-1 (reduce-scatter, "
                         "sharded Adam, all-gather)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--no-extra", action="store_true", help="skip the C3 / C5 side lines")
    ap.add_argument("--extra-steps", type=int, default=5)
    ap.add_argument("--kernel-table", action="store_true", help="print per-launch timings to stderr")
    ap.add_argument("--no-fold-bn", action="store_true",
                    help="A/B: keep FC-DenseNet's BatchNorm+ReLU as separate passes (no conv prologue)")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the two rocprofv3 --pmc child passes (FETCH_SIZE / WRITE_SIZE) behind roofline.traffic")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-miou", action="store_true", help="skip the mIoU parity probe")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the KITTI data-pipeline rate probe")
    ap.add_argument("--no-fuse-adam", action="store_true",
                    help="do not fuse TF1 Adam into the conv6/conv7 filter-gradient epilogue")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="seg_set_option kernel knob (A/B runs; repeatable)")
    ap.add_argument("--schedule", action="append", default=[], metavar="NAME=VALUE",
                    help="Session schedule attribute for A/B runs (side_wgrad, main_wgrad, fused_delay, "
                         "fuse_pool, fuse_grad_sum; repeatable)")
    ap.add_argument("--force-dp", action="store_true",
                    help="data-parallel Session over an RCCL ('nccl') process group even at world size 1 "
                         "(e.g. torchrun --nproc-per-node 1): the C4 per-rank step, all-reduces included")
    ap.add_argument("--force-collectives", action="store_true",
                    help="with --force-dp at world size 1: issue the bucket collectives anyway (the per-rank path "
                         "of a world > 1 job minus the wire time, as the dp_mode probe line)")
    ap.add_argument("--no-dp-probe", action="store_true",
                    help="N=1: skip the side line that re-times the step through a world-1 RCCL data-parallel Session")
    ap.add_argument("--no-inference", action="store_true", help="skip the inference-latency line")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank path (no GPU): --gpus N starts N rank processes over "
                         "gloo, each times K trivial steps, rank 0 prints the line with n_gpus = the world size")
    ap.add_argument("--overlap-optimizer", action="store_true",
                    help="per-layer Adam on a side stream as gradients become final (measured slower: the "
                         "HBM-bound update steals CUs from the MFMA-bound backward)")
    return ap.parse_args()


def pad32(x):
    return (x + 31) // 32 * 32


def synthetic(batch, H, W, HP, WP, seed, device):
    """Images: integers uniform in [0,255] (uint8 PNG fed raw, FCN.py:395);
    labels: a lower-image 'road' trapezoid + 5% pixel noise, uint8 class index
    (process_gt_image, FCN.py:195-201)."""
    import torch
    g = torch.Generator(device=device).manual_seed(seed)
    img = torch.zeros(batch, HP, WP, 3, dtype=torch.float32, device=device)
    img[:, :H, :W] = torch.randint(0, 256, (batch, H, W, 3), generator=g, device=device).float()
    yy = torch.arange(HP, device=device).view(HP, 1).float()
    xx = torch.arange(WP, device=device).view(1, WP).float()
    half = (yy - H * 0.45).clamp(min=0) / (H * 0.55) * (W * 0.45) + W * 0.05
    road = ((yy > H * 0.45) & ((xx - W / 2).abs() < half)).to(torch.uint8)
    lab = road.expand(batch, HP, WP).clone()
    noise = torch.rand(batch, HP, WP, generator=g, device=device) < 0.05
    lab = torch.where(noise, 1 - lab, lab)
    lab[:, H:, :] = 0
    lab[:, :, W:] = 0
    return img, lab.contiguous()


def cpu_baseline(H, W, HP, WP, steps, model="fcn"):
    """The oracle's FCN (or FC-DenseNet) forward+backward (torch-CPU fp32) on this host."""
    import numpy as np
    import torch
    from oracle import models as M
    from oracle import tf1_ops as T
    # every core this job is allotted: the GPU box gives one GPU's job 16 CPUs
    # (OMP_NUM_THREADS=16 there; nproc / os.cpu_count() report the whole host)
    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    shapes = {"fcn": M.fcn_param_shapes, "fcdensenet": M.fcdensenet_param_shapes,
              "deeplab": M.deeplab_param_shapes}[model](3, 2)
    fwd = {"fcn": M.fcn_forward, "fcdensenet": M.fcdensenet_forward, "deeplab": M.deeplab_forward}[model]
    p = {k: torch.from_numpy((rng.standard_normal(s, dtype=np.float32) * 0.01).astype(np.float32)
                             ).requires_grad_(True)
         for k, s in shapes.items()}
    x = torch.zeros(1, HP, WP, 3)
    x[:, :H, :W] = torch.from_numpy(rng.integers(0, 256, (1, H, W, 3)).astype(np.float32))
    lab = torch.zeros(1, HP, WP, dtype=torch.long)
    lab[:, H // 2:, W // 4:3 * W // 4] = 1
    mask = torch.zeros(1, HP, WP)
    mask[:, :H, :W] = 1
    y1 = T.one_hot(lab, 2, torch.float32)

    def step():
        for v in p.values():
            v.grad = None
        _, logits = fwd(p, x)
        T.mean_softmax_xent(logits, y1, mask).backward()

    step()                              # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = (time.perf_counter() - t0) / steps
    return {"value": round(1.0 / dt, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"oracle {dict(fcn='FCN', fcdensenet='FC-DenseNet', deeplab='DeepLab-ASPP')[model]} "
                      f"fwd+bwd, torch-CPU fp32, "
                      f"1 image {HP}x{WP}" + (f" ({H}x{W} padded)" if (H, W) != (HP, WP) else "") + ", "
                      f"1 warm-up + {steps} timed steps, {dt:.2f} s/step"}


def miou_parity(sess, pred, image, keep, img, lab, H, W, model):
    """mIoU of the trained model's class map on the benchmark batch (device,
    masked to HxW), and -- on image 0 -- the CPU oracle's class map from the
    same fp32 master weights (float64, bf16-rounded at the device's rounding
    points): agreement of the two maps and both mIoUs."""
    import numpy as np
    import torch
    from oracle import models as M
    from semanticsegmentation_tensorflow_amd import evaluate as E
    from semanticsegmentation_tensorflow_amd import ops
    pr = sess.run(pred, feed_dict={image: img, keep: 1.0}, as_numpy=False)
    m = E.MeanIoU(2, img.device, (H, W)).update(pr, lab)
    miou, _ = m.result()
    out = {"miou": round(miou, 5), "miou_images": int(img.shape[0])}
    if model != "fcn":
        return out
    names = M.fcn_param_shapes(3, 2)
    p = {k: torch.from_numpy(sess.variable_value(k)).double() for k in names}
    if sess.cdt == ops.BF16:   # bf16 compute: the device sees bf16 filters / input
        p = {k: (v.to(torch.bfloat16).double() if v.dim() == 4 else v) for k, v in p.items()}
    x0 = img[:1].double().cpu()
    t0 = time.perf_counter()
    with torch.no_grad():
        q = (lambda t: t.to(torch.bfloat16).double()) if sess.cdt == ops.BF16 else None
        rp, _ = M.fcn_forward(p, x0, quant=q)
    dt = time.perf_counter() - t0
    gp = pr[:1].reshape(rp.shape).cpu()
    agree = (gp[:, :H, :W] == rp[:, :H, :W]).double().mean().item()
    mo = E.MeanIoU(2, img.device, (H, W)).update(rp.to(img.device).reshape(1, *lab.shape[1:]), lab[:1])
    mg = E.MeanIoU(2, img.device, (H, W)).update(gp.to(img.device).reshape(1, *lab.shape[1:]), lab[:1])
    out.update({"image0_miou_device": round(mg.result()[0], 5), "image0_miou_oracle": round(mo.result()[0], 5),
                "image0_class_map_agreement": round(agree, 6),
                "oracle": f"oracle FCN forward, float64 (bf16 rounding points), {dt:.1f} s"})
    return out


def pipeline_rate(H, W, device, threads=16, seconds=2.0):
    """KITTI input pipeline (gen_batch_function, FCN.py:235-307) rates on this
    box: native PNG decode of 375x1242 RGBA merge + RGB gt files on `threads`
    host threads, and the GPU augmentation (3 samples per file: bc_img
    original, crop, flip; PIL-exact bilinear resize to HxW; labels)."""
    import io
    import random
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    import torch
    from PIL import Image

    from semanticsegmentation_tensorflow_amd import data
    rng = np.random.default_rng(7)
    yy, xx = np.mgrid[0:375, 0:1242]
    img = np.stack([(xx * 0.2 + yy * 0.3) % 256, (xx * 0.1) % 256, (yy * 0.5) % 256, np.full_like(xx, 255)], -1)
    img = (img + rng.integers(-8, 8, img.shape)).clip(0, 255).astype(np.uint8)
    gt = np.zeros((375, 1242, 3), np.uint8)
    gt[:] = (255, 0, 0)
    gt[220:, 300:900] = (255, 0, 255)
    pngs = []
    for a, mode in ((img, "RGBA"), (gt, "RGB")):
        b = io.BytesIO()
        Image.fromarray(a, mode).save(b, "PNG")
        pngs.append(b.getvalue())
    pair = lambda _: (data.png_decode(pngs[0]), data.png_decode(pngs[1]))   # noqa: E731
    n = 0
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(pair, range(threads)))
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            list(ex.map(pair, range(4 * threads)))
            n += 4 * threads
        files_per_s = n / (time.perf_counter() - t0)
    dec = [(torch.from_numpy(img).to(device), torch.from_numpy(gt).to(device)) for _ in range(4)]
    r = random.Random(1)
    data.augment_batch(dec, (H, W), r, device)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    s.record()
    for _ in range(reps):
        data.augment_batch(dec, (H, W), r, device)
    e.record()
    torch.cuda.synchronize()
    aug = 12 * reps / (s.elapsed_time(e) * 1e-3)
    return {"host_decode_files_per_s": round(files_per_s, 1), "host_threads": threads,
            "gpu_augment_samples_per_s": round(aug, 1), "samples_per_file": 3,
            "sustained_samples_per_s": round(min(3 * files_per_s, aug), 1),
            "note": f"375x1242 RGBA merge + RGB gt PNG pairs -> {H}x{W} samples + labels"}


def inference_latency(device, dtype, H=375, W=1242, images=30):
    """Per-image inference time the way the reference reports it
    (Network/utils/utils.py:63-89, averaged over 30 images in
    Network/main.py:200-206): one image per sess.run of tf.nn.softmax(logits)
    with keep_prob 1.0.  Two figures: `device_ms_per_img` -- the image
    resident in HBM, the softmax map left on the device (kernel time plus
    launch overhead, synchronised per image); `gen_test_output_ms_per_img` --
    evaluate.gen_test_output (numpy image in, numpy softmax out: host copies
    included, the reference's loop body without PNG decode / resize)."""
    import numpy as np
    import torch
    from semanticsegmentation_tensorflow_amd import evaluate as E
    from semanticsegmentation_tensorflow_amd import graph as G
    from semanticsegmentation_tensorflow_amd import tf
    from semanticsegmentation_tensorflow_amd.fcn import FCN
    HP, WP = pad32(H), pad32(W)
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, HP, WP, 3], name="input_image")
    keep = tf.placeholder(tf.float32, name="keep_probability")
    _, logits = FCN(image, keep, 2).create()
    softmax = tf.nn.softmax(logits)
    sess = tf.Session(compute_dtype=dtype, seed=0)
    sess.run(tf.global_variables_initializer())
    imgs, _ = synthetic(images, H, W, HP, WP, 4321, device)
    for i in range(3):                                    # plan compile + warm-up
        sess.run(softmax, feed_dict={image: imgs[i:i + 1], keep: 1.0}, as_numpy=False)
    torch.cuda.synchronize()
    t = []
    for i in range(images):
        t0 = time.perf_counter()
        sess.run(softmax, feed_dict={image: imgs[i:i + 1], keep: 1.0}, as_numpy=False)
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    host = imgs.cpu().numpy()
    t2 = [pt for _, _, _, pt in E.gen_test_output(sess, softmax, keep, image, host, (HP, WP))]
    del sess
    torch.cuda.empty_cache()
    return {"batch": 1, "images": images, "image": f"{H}x{W} -> {HP}x{WP}", "dtype": dtype,
            "fetch": "tf.nn.softmax(logits), keep_prob 1.0 (Network/utils/utils.py:81)",
            "device_ms_per_img": round(1e3 * float(np.mean(t)), 3),
            "device_ms_per_img_min": round(1e3 * float(np.min(t)), 3),
            "gen_test_output_ms_per_img": round(1e3 * float(np.mean(t2)), 3),
            "note": "device: image resident in HBM, softmax left on the device, synchronised per image; "
                    "gen_test_output: numpy image in / numpy softmax out per image (host copies included)"}


def kernel_symbol(name):
    """rocprof symbol pattern of a seg_conv_kernel_info family name (the main
    kernel; its split-K reducer launches are attributed to it separately)."""
    fam, rest = name.split("<", 1)
    a = rest.rstrip(">").split(",")
    bm, bn = a[1], a[2]
    # dtype-templated kernels appear mangled (`_ZN3seg10conv_halo2ILi16E...`)
    if fam == "conv_halo4":
        return r"conv_halo4[<I]"
    if fam == "conv_halo":
        return r"conv_halo2[<I]" if bn == "256" else r"conv_halo(_duo)?[<I]"
    if fam in ("igemm_nt3", "igemm_tn3"):
        return fam + "<"
    if fam == "igemm_nt2_bn":   # the BatchNorm-backward instantiation (last template flag)
        return rf"igemm_nt2I\w*Li{bm}ELi{bn}E\w*Lb0ELb1EEEv"
    if fam == "igemm_nt2":
        return rf"igemm_nt2I\w*Li{bm}ELi{bn}E"
    if fam == "igemm_tn2":
        return rf"igemm_tn2(<{bm}, {bn},|I\w*Li{bm}ELi{bn}E)"
    if fam == "wgrad_halo":
        return rf"wgrad_halo(<\d+, {bn},|ILi\d+ELi{bn}E)"
    # family names whose kernel symbol differs from the family name
    return {"conv_res64": r"conv_res64[<I]", "conv_c8": r"conv_c8_fwd", "wgrad_c8": r"wgrad_c8",
            "igemm_nt": r"igemm_ntI", "igemm_tn": r"igemm_tnI",
            "bn1x1_stream": r"bn1x1_dgrad_stream", "conv1x1_stream": r"conv1x1_stream",
            "conv_res16c_bn": r"conv_res16cIDF16[b_]Lb1E", "smallk_nt": r"smallk_nt_k",
            "igemm_nt2_pro": r"igemm_nt2I\w*Lb1ELb0EEEv", "igemm_tn2_pro": r"igemm_tn2I\w*Lb1EEEv",
            }.get(fam, re.escape(fam))


def pmc_traffic(argv, symbol, out_dir):
    """HBM bytes per launch of the dominant kernel from two separate rocprofv3
    --pmc passes over a child run of this benchmark (one warm-up + one timed
    step; only the last step's dispatches are used).  Corrections per
    MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB;
    on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced streaming
    read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  A
    launch's split-K reducer dispatches are attributed to it."""
    import csv
    import shutil
    import signal
    import subprocess
    res = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out_dir, ctr.lower())
        shutil.rmtree(d, ignore_errors=True)
        cmd = ["rocprofv3", "--pmc", ctr, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run",
               "--", sys.executable, os.path.abspath(__file__)] + argv + ["--pmc-child"]
        env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
        p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env,
                             start_new_session=True)
        try:
            p.wait(timeout=180)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            raise RuntimeError(f"rocprofv3 --pmc {ctr} timed out")
        path = None
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    path = os.path.join(root, f)
        if p.returncode != 0 or path is None:
            raise RuntimeError(f"rocprofv3 --pmc {ctr} failed (rc={p.returncode})")
        rows = list(csv.DictReader(open(path)))
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        starts = [i for i, r in enumerate(rows) if "prepare_input" in r["Kernel_Name"]]
        step = rows[starts[-1]:]
        pat = re.compile(symbol)
        total, launches, inside = 0.0, 0, False
        for r in step:
            k = r["Kernel_Name"]
            if pat.search(k):
                launches += 1
                inside = True
                total += float(r["Counter_Value"])
            elif inside and "splitk_reduce" in k:
                total += float(r["Counter_Value"])
            else:
                inside = False
        if launches == 0:
            raise RuntimeError(f"no dispatch of {symbol} in the PMC pass")
        res[ctr] = total * 1024.0 / launches * (2.0 if ctr == "FETCH_SIZE" else 1.0)
        res["launches"] = launches
    return res


DEFAULTS = {  # per model: (H, W, batch per GPU, keep_prob)
    "fcn": (375, 1242, 4, 0.8),            # C2 (C4 under torchrun); FCN.py:395 keep_prob 0.8
    "fcdensenet": (375, 1242, 8, 0.2),     # C3; FCDenseNet.py KEEP_PROB
    "deeplab": (1024, 2048, 2, 0.9),       # C5, Cityscapes-shaped
}
WORKLOAD = {"fcn": "FCN (reference Network/model/FCN.py topology)",
            "fcdensenet": "FC-DenseNet 'U-Net' (reference Network/model/FCDenseNet.py topology)",
            "deeplab": "DeepLab-style atrous VGG16 + ASPP (rates 6/12/18, image pooling) + bilinear x8 "
                       "(semanticsegmentation_tensorflow_amd/deeplab.py; config C5)"}


SCHEDULE = {}     # --schedule overrides, applied to every Session build_train_graph makes


def build_train_graph(model, H, W, dtype, dp=None, fuse_adam=True, overlap_optimizer=False, fold_bn=True):
    """The benchmarked training graph and Session: `model`'s builder on a
    [None, HP, WP, 3] image placeholder (H x W zero-padded to multiples of
    32), softmax-xent masked to H x W, tf.train.AdamOptimizer(1e-4).minimize
    (Network/model/FCN.py:312-340).  The full-size parity tests
    (tests/test_gpu_fullsize.py) build their step through this function, so
    they run exactly the launch plan bench.py times."""
    from semanticsegmentation_tensorflow_amd import graph as G
    from semanticsegmentation_tensorflow_amd import tf
    from semanticsegmentation_tensorflow_amd.deeplab import DeepLabASPP
    from semanticsegmentation_tensorflow_amd.fcdensenet import FCDenseNet
    from semanticsegmentation_tensorflow_amd.fcn import FCN
    HP, WP = pad32(H), pad32(W)
    G.reset_default_graph()
    image = tf.placeholder(tf.float32, [None, HP, WP, 3], name="input_image")
    labels = tf.placeholder(tf.uint8, [None, HP, WP], name="annotation")
    keep = tf.placeholder(tf.float32, name="keep_probability")
    if model == "fcn":
        pred, logits = FCN(image, keep, 2).create()
    elif model == "deeplab":
        pred, logits = DeepLabASPP(image, keep, 2)
    else:
        pred, logits = FCDenseNet(image, keep, 2)
    loss = tf.reduce_mean(tf.nn.softmax_cross_entropy_with_logits(logits=logits, labels=labels,
                                                                   valid_hw=(H, W)))
    train_step = tf.train.AdamOptimizer(1e-4).minimize(loss)
    sess = tf.Session(compute_dtype=dtype, seed=0, data_parallel=dp, overlap_optimizer=overlap_optimizer,
                      fuse_adam=fuse_adam)
    sess.fold_bn = fold_bn
    for k, v in SCHEDULE.items():
        if not hasattr(sess, k):
            raise ValueError(f"--schedule: no Session attribute {k!r}")
        setattr(sess, k, v)
    sess.run(tf.global_variables_initializer())
    return {"sess": sess, "image": image, "labels": labels, "keep": keep, "pred": pred, "logits": logits,
            "loss": loss, "train_step": train_step, "HP": HP, "WP": WP}


def measure(model, B, H, W, kp, steps, warmup, dtype, device, dp=None, rank=0, fuse_adam=True,
            overlap_optimizer=False, want_miou=False, fold_bn=True):
    """Build `model`'s training graph, run `warmup` + `steps` timed train steps
    on a synthetic batch resident in HBM, then one more step with HIP events
    around every conv launch (on its launch stream) for the per-kernel
    roofline.  Returns the measurement dict (no printing)."""
    import torch
    import torch.distributed as dist
    from semanticsegmentation_tensorflow_amd import ops

    world = dp.world if dp is not None else 1
    g = build_train_graph(model, H, W, dtype, dp, fuse_adam, overlap_optimizer, fold_bn)
    sess, image, labels, keep, pred, loss, train_step = (g[k] for k in ("sess", "image", "labels", "keep", "pred",
                                                                        "loss", "train_step"))
    HP, WP = g["HP"], g["WP"]
    img, lab = synthetic(B, H, W, HP, WP, 1234 + rank, device)
    feed = {image: img, labels: lab, keep: kp}

    for _ in range(warmup):
        sess.run(train_step, feed_dict=feed)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        sess.run(train_step, feed_dict=feed)
    torch.cuda.synchronize()
    if dp:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dp:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    out = {"elapsed": elapsed, "loss": float(sess.run(loss, feed_dict=feed)), "HP": HP, "WP": WP}
    if want_miou:
        try:
            out["miou"] = miou_parity(sess, pred, image, keep, img, lab, H, W, model)
        except Exception as exc:  # report, never crash the headline line
            out["miou"] = {"error": repr(exc)}

    # ---- per-kernel timing (HIP events on the launch stream) for the roofline
    sess.timer = []
    # a spin kernel first, so the host has queued the whole step before the GPU
    # reaches it: the event pairs then bracket device time only (the timed
    # step's per-launch event records slow the host; on a step of many small
    # launches -- C3 -- the GPU would otherwise catch up and the host's gaps
    # would land inside the spans)
    torch.cuda._sleep(int(4e8))
    sess.run(train_step, feed_dict=feed)
    torch.cuda.synchronize()
    per = {}
    step_conv_flops = 0.0
    rows = []
    esz = 4 if dtype == "f32" else 2
    for desc, op, s_ev, e_ev in sess.timer:
        name, splits, flops = ops.conv_kernel_info(desc, op)
        ms = s_ev.elapsed_time(e_ev)
        step_conv_flops += flops
        # algorithmic HBM bytes: input + output activations once, the filter once
        # (fp32 filter gradient for the wgrad ops)
        nbytes = esz * (desc.N * desc.H * desc.W * desc.c_valid + desc.N * desc.OH * desc.OW * desc.k_valid) \
            + (4 if op in (ops.OP_BWD_FILTER, ops.OP_TBWD_FILTER, ops.OP_BWD_FILTER_PRO) else esz) \
            * desc.R * desc.S * desc.c_valid * desc.k_valid
        if op == ops.OP_BWD_DATA_BN:        # + the BN input read to re-derive the mask / dgamma
            nbytes += esz * desc.N * desc.H * desc.W * desc.c_valid
        rows.append((name, op, splits, flops, ms, desc.N, desc.H, desc.W, desc.c_valid, desc.k_valid, desc.R))
        a = per.setdefault(name, [0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += flops
        a[2] += ms
        a[3] += nbytes
    sess.timer = None
    # the same per-launch timing with the filter gradients serialised on the
    # compute stream: each kernel alone on the chip (in the timed step the
    # side-stream filter gradients share the CUs with the input-gradient chain)
    alone = {}
    side_mode = getattr(sess, "side_wgrad", 0)
    if side_mode:
        sess.side_wgrad = 0
        sess.timer = []
        torch.cuda._sleep(int(4e8))
        sess.run(train_step, feed_dict=feed)
        torch.cuda.synchronize()
        for desc, op, s_ev, e_ev in sess.timer:
            name = ops.conv_kernel_info(desc, op)[0]
            a = alone.setdefault(name, [0, 0.0])
            a[0] += 1
            a[1] += s_ev.elapsed_time(e_ev)
        sess.timer = None
        sess.side_wgrad = side_mode
    # the dominant family: the most time in the serialized step (each kernel
    # alone on the chip; in the overlapped step two families of similar time
    # swap between runs), or in the step itself when no side stream exists
    rank_by = {k: v for k, v in alone.items() if k in per} or {k: (v[0], v[2]) for k, v in per.items()}
    dname = max(rank_by.items(), key=lambda kv: kv[1][1])[0]
    dn, dflops, dms, dbytes = per[dname]
    # the dominant family re-timed in-step with events around ITS launches
    # only (every other launch un-instrumented, as in the timed steps): the
    # figure the line reports, comparable with the kernel durations of the
    # timed steps in a rocprofv3 kernel trace (tools/timed_stats.py)
    all_ev_ms = dms / dn
    reps = max(1, min(steps, 5))
    sess.timer = []
    seen = {}

    def is_dominant(d, o):
        k = (id(d), o)
        if k not in seen:
            seen[k] = ops.conv_kernel_info(d, o)[0] == dname
        return seen[k]
    sess.timer_match = is_dominant
    torch.cuda._sleep(int(4e8))
    for _ in range(reps):
        sess.run(train_step, feed_dict=feed)
    torch.cuda.synchronize()
    ev = [s_ev.elapsed_time(e_ev) for _, _, s_ev, e_ev in sess.timer]
    sess.timer, sess.timer_match = None, None
    timing_mode = "all_events"
    if len(ev) == dn * reps:
        dms = sum(ev) / reps
        timing_mode = "family"
    achieved = (dflops / dn) / (dms / dn * 1e-3)
    peak = PEAK[dtype]
    # roofline bound of the dominant kernel group from its arithmetic intensity
    hbm_bound = dflops / dbytes < peak / HBM_PEAK
    if hbm_bound:
        roof = {"bound": "hbm", "kernel": dname, "achieved": round(dbytes / dn / (dms / dn * 1e-3) / 1e9, 1),
                "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": round(dbytes / (dms * 1e-3) / HBM_PEAK, 4),
                "traffic": None, "launches_per_step": dn, "algorithmic_bytes_per_launch": round(dbytes / dn),
                "algorithmic_gflop_per_launch": round(dflops / dn / 1e9, 3), "mfma_frac": round(achieved / peak, 4),
                "avg_launch_ms": round(dms / dn, 4)}
    else:
        roof = {"bound": "mfma", "kernel": dname, "achieved": round(achieved / 1e12, 2),
                "peak": round(peak / 1e12, 1), "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "traffic": None, "launches_per_step": dn, "algorithmic_gflop_per_launch": round(dflops / dn / 1e9, 3),
                "algorithmic_bytes_per_launch": round(dbytes / dn), "avg_launch_ms": round(dms / dn, 4)}
    roof["all_events_avg_launch_ms"] = round(all_ev_ms, 4)
    roof["timing_mode"] = timing_mode
    if timing_mode == "family":
        roof["timing"] = (f"HIP events (hipEventDisableSystemFence: no cache flush in the interval) on the launch "
                          f"stream around the {dn} launches per step of this family only, {reps} train steps after "
                          f"the timed ones; all_events_avg_launch_ms: the same with every conv launch of the step "
                          f"bracketed")
    else:
        roof["timing"] = (f"HIP events around EVERY conv launch of one train step (the family-only re-timing "
                          f"recorded {len(ev)} events, not {dn} x {reps}, and was discarded)")
    if dname in alone and alone[dname][1] > 0:
        an, ams = alone[dname]
        if hbm_bound:
            ach = dbytes / an / (ams / an * 1e-3)
            roof["alone"] = {"achieved": round(ach / 1e9, 1), "frac": round(ach / HBM_PEAK, 4)}
        else:
            ach = dflops / an / (ams / an * 1e-3)
            roof["alone"] = {"achieved": round(ach / 1e12, 2), "frac": round(ach / peak, 4)}
        roof["alone"].update({"avg_launch_ms": round(ams / an, 4), "note": (
            "the same launches timed in a step with the filter gradients serialised on the compute stream "
            "(the kernel alone on the chip); the headline step runs them on the side stream, sharing the CUs")})
    ms_per_step = elapsed / steps * 1e3
    step_flops = FCN_TRAIN_FLOP_PER_IMG * B if (model == "fcn" and (HP, WP) == (384, 1248)) else step_conv_flops
    out.update({"value": B * world * steps / elapsed, "ms_per_step": ms_per_step, "roofline": roof,
                "step_mfma_frac": step_flops / (ms_per_step * 1e-3) / peak,
                "conv_gflop_per_step": step_conv_flops / 1e9, "rows": rows, "groups": per})
    if dtype == "f16":
        out["loss_scaling"] = {"kind": "dynamic" if sess.dynamic_scale else "fixed", "scale": sess.loss_scale,
                               "skipped_steps": sess.skipped_steps}
    del sess
    torch.cuda.empty_cache()
    return out


def extra_config(model, dtype, device, steps, warmup):
    """C3 / C5 measured in the same run as the headline (a reported side line;
    the headline metric stays C2)."""
    H, W, B, kp = DEFAULTS[model]
    dtype = DEFAULT_DTYPE[model] if dtype is None else dtype
    m = measure(model, B, H, W, kp, steps, warmup, dtype, device)
    return {"config": {"workload": WORKLOAD[model], "batch": B, "image": f"{H}x{W} -> {m['HP']}x{m['WP']}",
                       "keep_prob": kp},
            "value": round(m["value"], 3), "unit": "images/s", "steps": steps, "warmup": warmup,
            "ms_per_step": round(m["ms_per_step"], 3), "dtype": dtype,
            "step_mfma_frac": round(m["step_mfma_frac"], 4), "roofline": m["roofline"],
            **({"loss_scaling": m["loss_scaling"]} if "loss_scaling" in m else {})}


def init_rccl(device):
    """torch.distributed over RCCL ('nccl' on ROCm); a world-1 group when not
    launched by torchrun."""
    import torch.distributed as dist
    if dist.is_initialized():
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dist.init_process_group("nccl", device_id=device)


def dp_probe(args, B, H, W, kp, device):
    """The headline step re-timed through the data-parallel Session over a
    world-1 RCCL process group with the collectives forced on: config C4's
    per-rank step minus the wire time -- every bucket reduce-scattered over
    RCCL from the side stream as backward produces it, TF1 Adam on the rank's
    slices (ZeRO-1), the all-gather of the updated parameters and the repack
    of the compute copies (the conv6 / conv7 filter-gradient + Adam fusion is
    off: a collective sits between gradient and update)."""
    import torch
    import torch.distributed as dist
    from semanticsegmentation_tensorflow_amd.dp import DataParallel
    own = not dist.is_initialized()
    init_rccl(device)
    dp = DataParallel(bucket_mb=args.bucket_mb, force_collectives=True, shard_optimizer=args.dp_mode == "zero")
    m = measure(args.model, B, H, W, kp, args.steps, args.warmup, args.dtype, device, dp, 0)
    exchange = ("zero1 (reduce-scatter, sharded Adam, all-gather)" if args.dp_mode == "zero"
                else "all-reduce per bucket during backward, every rank's Adam")
    backend, world, nb = dist.get_backend(), dist.get_world_size(), len(dp.buckets)
    if own:
        # the group exists for this probe only: its RCCL proxy thread would
        # otherwise keep polling beside the side lines (C3 measured 197 instead
        # of 214 img/s after it) and the CPU baseline
        torch.cuda.synchronize()
        dist.destroy_process_group()
    return {"backend": backend, "world": world, "bucket_mb": args.bucket_mb,
            "buckets": nb, "exchange": exchange,
            "value": round(m["value"], 3), "unit": "images/s", "ms_per_step": round(m["ms_per_step"], 3),
            "note": "same workload as the headline; collectives forced on at world 1 (a real world-1 job "
                    "skips them and runs the single-process plan)"}


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) started without torchrun: start N rank
    processes of this script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE =
    N, rendezvous on 127.0.0.1), and exit with the worst rank's status.  The
    parent never initialises the GPU (torch.cuda.device_count() does not on
    this image) and prints nothing on stdout: rank 0 prints the line.  N above
    the visible device count is an error.  If a rank fails, the others are
    terminated (by PID) rather than left waiting in a collective."""
    import signal
    import subprocess
    n = args.gpus
    if not args.dry_run:
        import torch
        vis = torch.cuda.device_count()
        if n > vis:
            print(f"bench.py: --gpus {n} but {vis} GPU(s) visible", file=sys.stderr)
            return 2
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            if p.poll() is None:
                continue
            live.remove(p)
            rc = max(rc, abs(p.returncode))
            if p.returncode != 0:
                for q in live:
                    q.send_signal(signal.SIGTERM)
    return rc


def dry_run(args):
    """The multi-rank reporting path without a GPU: gloo process group, W + K
    steps of a small all-reduce (the step's gradient exchange stand-in),
    barrier-bracketed timing, MAX over ranks, rank 0 prints the line."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    g = torch.ones(1 << 16)

    def step():
        if world > 1:
            dist.all_reduce(g)
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    B = args.batch or DEFAULTS[args.model][2]
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps({"metric": METRIC, "value": round(B * world * args.steps / elapsed, 3), "unit": "images/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": None, "data": "synthetic",
                          "dry_run": True, "config": {"workload": "dry run (gloo, no GPU)", "global_batch": B * world,
                                                      "parallelism": f"dp{world}"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main():
    args = parse()
    if args.gpus is None:   # torchrun without --gpus: one rank per process it started
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.dry_run:
        sys.exit(dry_run(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:   # only an explicit --gpus can disagree with the launcher
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dp = None
    from semanticsegmentation_tensorflow_amd.session import side_stream_for
    side_stream_for(device)     # before RCCL takes hardware queues (session.side_stream_for)
    if world > 1 or args.force_dp:
        init_rccl(device)
        from semanticsegmentation_tensorflow_amd.dp import DataParallel
        dp = DataParallel(bucket_mb=args.bucket_mb, shard_optimizer=args.dp_mode == "zero",
                          force_collectives=args.force_collectives)
        world = dist.get_world_size()     # what RCCL saw

    from semanticsegmentation_tensorflow_amd import ops
    for kv in args.option:
        name, val = kv.split("=")
        ops.set_option(name, int(val))
    for kv in args.schedule:
        name, val = kv.split("=")
        SCHEDULE[name] = float(val) if "." in val else int(val)
    dH, dW, dB, dkp = DEFAULTS[args.model]
    if args.dtype is None:
        args.dtype = DEFAULT_DTYPE[args.model]
    H, W = args.height or dH, args.width or dW
    B = args.batch or dB
    kp = args.keep_prob if args.keep_prob is not None else dkp
    m = measure(args.model, B, H, W, kp, args.steps, args.warmup, args.dtype, device, dp, rank,
                fuse_adam=not args.no_fuse_adam, overlap_optimizer=args.overlap_optimizer,
                want_miou=rank == 0 and not args.no_miou and not args.pmc_child, fold_bn=not args.no_fold_bn)
    if args.pmc_child:
        return
    HP, WP = m["HP"], m["WP"]
    if args.kernel_table and rank == 0:
        for r in m["rows"]:
            print("KERNEL %-26s op=%d split=%-3d GF=%8.2f ms=%8.3f TF/s=%7.1f N=%d %dx%d C=%d K=%d R=%d"
                  % (r[0], r[1], r[2], r[3] / 1e9, r[4], r[3] / r[4] / 1e9, *r[5:]), file=sys.stderr)
        for k, (n, f, ms, b) in sorted(m["groups"].items(), key=lambda kv: -kv[1][2]):
            print(f"GROUP {k}: launches={n} ms={ms:.3f} TF/s={f / ms / 1e9:.1f} GB/s={b / ms / 1e6:.0f}",
                  file=sys.stderr)
    dname = m["roofline"]["kernel"]
    result = {
        "metric": METRIC,
        "value": round(m["value"], 3),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(m["ms_per_step"], 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic",
        "config": {
            "workload": WORKLOAD[args.model] + f" train step: fwd + softmax-xent + bwd + TF1 Adam, {H}x{W}x3"
                        + (f" zero-padded to {HP}x{WP}" if (HP, WP) != (H, W) else ""),
            "global_batch": B * world,
            "batch_per_gpu": B,
            "image": f"{H}x{W} -> {HP}x{WP}",
            "parallelism": f"dp{world}",
            "dp_mode": args.dp_mode if world > 1 else None,
            "keep_prob": kp,
        },
        "roofline": m["roofline"],
        "step_mfma_frac": round(m["step_mfma_frac"], 4),
        "conv_gflop_per_step_measured": round(m["conv_gflop_per_step"], 2),
        "loss_after": round(m["loss"], 5),
        "miou_parity": m.get("miou"),
        "env": {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES")},
    }
    if "loss_scaling" in m:
        result["loss_scaling"] = m["loss_scaling"]
    # the world-1 RCCL probe right after the headline: after the CPU baseline
    # its host-heavy step shared the host with that run's still-spinning OpenMP
    # threads and lost ~10 % (495 vs 548 img/s in round 5)
    if world == 1 and dp is None and args.model == "fcn" and not args.no_dp_probe:
        try:
            result["dp_mode"] = dp_probe(args, B, H, W, kp, device)
        except Exception as exc:  # report, never crash the headline line
            result["dp_mode"] = {"error": repr(exc)}
    if rank == 0 and world == 1 and not args.no_pipeline and args.model == "fcn":
        try:
            result["data_pipeline"] = pipeline_rate(H, W, device)
        except Exception as exc:  # report, never crash the headline line
            result["data_pipeline"] = {"error": repr(exc)}
    if rank == 0 and world == 1 and not args.no_traffic:
        try:
            argv = [a for a in sys.argv[1:] if a not in ("--kernel-table",)]
            argv = argv + ["--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-traffic", "--no-miou",
                           "--no-pipeline", "--no-extra", "--no-dp-probe", "--no-inference"]
            t = pmc_traffic(argv, kernel_symbol(dname), os.path.join(ROOT, "gpurun_out", "bench_pmc"))
            result["roofline"]["traffic"] = round(t["FETCH_SIZE"] + t["WRITE_SIZE"])
            result["roofline"]["traffic_detail"] = {
                "unit": "bytes per launch", "fetch_x2": round(t["FETCH_SIZE"]), "write": round(t["WRITE_SIZE"]),
                "symbol": kernel_symbol(dname), "launches": t["launches"],
                "note": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE, separate passes; FETCH_SIZE doubled (gfx950)"}
        except Exception as exc:  # report, never crash the headline line
            result["roofline"]["traffic_error"] = repr(exc)
    if rank == 0 and world == 1 and args.model == "fcn" and not args.no_inference and not args.pmc_child:
        try:
            result["inference"] = inference_latency(device, args.dtype, H, W)
        except Exception as exc:  # report, never crash the headline line
            result["inference"] = {"error": repr(exc)}
    if rank == 0 and world == 1 and args.model == "fcn" and not args.no_extra:
        # C3 and C5 in the same run (side lines; the headline stays C2)
        for key, model in (("c3_fcdensenet", "fcdensenet"), ("c5_deeplab", "deeplab")):
            try:
                result[key] = extra_config(model, None, device, args.extra_steps, 3)
            except Exception as exc:  # report, never crash the headline line
                result[key] = {"error": repr(exc)}
                continue
            if args.no_traffic:
                continue
            try:   # HBM traffic of that config's dominant kernel, same two PMC passes
                roof = result[key]["roofline"]
                sym = kernel_symbol(roof["kernel"])
                argv = ["--model", model, "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-traffic",
                        "--no-miou", "--no-pipeline", "--no-extra", "--no-dp-probe", "--no-inference"]
                t = pmc_traffic(argv, sym, os.path.join(ROOT, "gpurun_out", "bench_pmc_" + model))
                roof["traffic"] = round(t["FETCH_SIZE"] + t["WRITE_SIZE"])
                roof["traffic_detail"] = {
                    "unit": "bytes per launch", "fetch_x2": round(t["FETCH_SIZE"]), "write": round(t["WRITE_SIZE"]),
                    "symbol": sym, "launches": t["launches"],
                    "note": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE, separate passes; FETCH_SIZE doubled (gfx950)"}
            except Exception as exc:
                result[key]["roofline"]["traffic_error"] = repr(exc)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(H, W, HP, WP, args.cpu_steps, args.model)
            if args.model == "fcn":
                # the FCN driver's own default training shape (Network/model/FCN.py:24)
                result["cpu_baseline_160x576"] = cpu_baseline(160, 576, 160, 576, args.cpu_steps, "fcn")
        except Exception as exc:  # report, never crash the headline line
            result["cpu_baseline"] = {"value": None, "error": repr(exc)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
