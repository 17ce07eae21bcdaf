"""Which hardware queue do the Session's compute and side streams land on
once an RCCL process group exists?  Run under `rocprofv3 --kernel-trace` and
read Queue_Id: python tools/queue_probe.py {none,late,early,prio}."""
import os
import sys

import torch
import torch.distributed as dist

mode = sys.argv[1]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def work(s, tag):
    with torch.cuda.stream(s):
        a = torch.full((2048, 2048), 1e-3, device=dev)
        for _ in range(2):
            a = a @ a
    torch.cuda.synchronize()
    print(tag, "stream", s.cuda_stream, flush=True)


side = None
if mode == "early":
    side = torch.cuda.Stream(device=dev)
    work(side, "early-side")
if mode != "none":
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29573")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    dist.init_process_group("nccl", device_id=dev)
if side is None:
    side = torch.cuda.Stream(device=dev, priority=-1 if mode == "prio" else 0)
work(torch.cuda.current_stream(dev), "compute")
work(side, "side")
if dist.is_initialized():
    dist.destroy_process_group()
