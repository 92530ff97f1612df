"""RCCL all_reduce captured inside a HIP graph (world size 1 process group over nccl=RCCL): the
capture machinery bench.py --comm graph relies on at N > 1."""
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
x = torch.arange(1 << 20, device=dev, dtype=torch.float32)
dist.all_reduce(x)           # warm (communicator init outside capture)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    with torch.cuda.graph(g, stream=s):
        x.mul_(2.0)
        dist.all_reduce(x)
        x.add_(1.0)
x.copy_(torch.arange(1 << 20, device=dev, dtype=torch.float32))
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
ref = torch.arange(1 << 20, device=dev, dtype=torch.float32)
for _ in range(3):
    ref = ref * 2 + 1
assert torch.equal(x, ref), (x[:4], ref[:4])
print("[rccl-capture] OK: all_reduce captured and replayed 3x", flush=True)
dist.destroy_process_group()
