"""the data-parallel Session through RCCL on the GPU.

One process, world 1 over the 'nccl' (RCCL) backend with the collectives
forced on (tests/workers/dp_rccl_worker.py): the ZeRO-1 reduce-scatter +
sharded Adam + all-gather, and the all-reduce path, issued from the Session's
side stream beside the side-stream filter gradients and their deferred split-K
reductions -- a stream-ordering mistake there would corrupt C4's gradients.
Every Session schedule attribute value (side_wgrad 0 / 1 / 2, main_wgrad 0 /
1 / 2 / 3, fused_delay 0 / 6, fuse_pool, fuse_grad_sum) runs, single-process
and data-parallel, and each step's gradients, parameters and Adam m / v are
checked against the default single-process step (which fuses the conv6 /
conv7 update into their filter-gradient epilogues):
* gradients vs the default step: fp32 within 1e-5 of each variable's max;
  bf16 within relative L2 2e-2 (un-fusing pool / gradient sums reorders bf16
  roundings), and bit-identical for a schedule that only moves launches
  between streams;
* the update vs float64 TF1 Adam (t = 1) of the step's OWN gradient:
  parameters within 1e-6 + 1e-5 * max, m 1e-5 / v 1e-4 relative (the
  fused-update kernel's documented tolerances, tests/test_gpu_ops.py) -- so
  the sharded update and its all-gather are checked exactly, not through
  gradient noise.
Network/model/FCN.py:334-340 (loss, Adam), Network/main.py:29-34 (the
reference is single-device)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from tests.workers.dp_rccl_worker import CASES

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STREAM_ONLY = {"sp_bf16_serial", "sp_bf16_side1", "sp_bf16_mw2"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _adam1(p0, g):
    """TF1 Adam, first step, float64."""
    lr_t = 1e-4 * np.sqrt(1 - 0.999) / (1 - 0.9)
    m = 0.1 * g
    v = 0.001 * g * g
    return p0 - lr_t * m / (np.sqrt(v) + 1e-8), m, v


@pytest.mark.timeout(300)
def test_dp_rccl_world1_every_schedule(dev, tmp_path):
    from oracle import models as M
    from tests.model_inputs import he_weights
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-u", "-m", "tests.workers.dp_rccl_worker", str(_free_port()),
                        str(tmp_path)], cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=280)
    assert p.returncode == 0, p.stdout[-4000:]
    w0 = he_weights(M.fcn_param_shapes(3, 2), 91)
    res = {tag: dict(np.load(os.path.join(tmp_path, tag + ".npz"))) for tag, _, _, _ in CASES}
    for tag, dtype, mode, sched in CASES:
        ref = res["ref_" + dtype]
        r = res[tag]
        for name in w0:
            if tag in STREAM_ONLY:
                for q in ("g:", "p:", "m:", "v:"):
                    assert np.array_equal(r[q + name], ref[q + name]), (tag, q, name)
                continue
            g, gr = r["g:" + name].astype(np.float64), ref["g:" + name].astype(np.float64)
            if dtype == "f32":
                assert np.abs(g - gr).max() <= 1e-5 * max(np.abs(gr).max(), 1e-30), (tag, name)
            else:
                rel = np.linalg.norm(g - gr) / max(np.linalg.norm(gr), 1e-30)
                assert rel <= 2e-2, (tag, name, rel)
            pe, me, ve = _adam1(w0[name].astype(np.float64), g)
            pd = r["p:" + name].astype(np.float64)
            assert np.abs(pd - pe).max() <= 1e-6 + 1e-5 * np.abs(pe).max(), (tag, name)
            np.testing.assert_allclose(r["m:" + name], me, rtol=1e-5, atol=1e-12, err_msg=f"{tag} {name} m")
            np.testing.assert_allclose(r["v:" + name], ve, rtol=1e-4, atol=1e-20, err_msg=f"{tag} {name} v")
