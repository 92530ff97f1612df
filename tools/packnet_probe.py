"""Probe: eager PackNet01 forward / backward timings per phase on the GPU (cold MIOpen caches)."""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.argv = ["bench.py", "--depth-net", "PackNet01", "--batch", "6"]
import bench  # noqa: E402
import __graft_entry__  # noqa: E402

__graft_entry__.build()
args = bench.parse()
dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False


def log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


model = bench.build_model(args, dev)
net = model.depth_net
x = torch.rand(6, 3, 192, 640, device=dev)
for it in range(3):
    t = time.perf_counter()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = net(x)
    torch.cuda.synchronize()
    log(f"fwd {it}: {time.perf_counter() - t:.2f} s")
    t = time.perf_counter()
    sum(o.float().mean() for o in out["inv_depths"]).backward()
    torch.cuda.synchronize()
    log(f"bwd {it}: {time.perf_counter() - t:.2f} s")
