"""Where the ATen layout / dtype copies of the ResNetSAN01 + PoseNet step come from: one forward +
backward under bf16 autocast (channels_last nets, fused epilogues as in bench.py) profiled with
python stacks; prints every copy / cat / fill kernel's aten op and the stack that launched it.
python tools/diag_copies.py"""
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
import bench  # noqa: E402
import packnet_sfm_amd  # noqa: E402,F401
from packnet_sfm_amd.networks.depth.ResNetSAN01 import ResNetSAN01  # noqa: E402
from packnet_sfm_amd.networks.pose.PoseNet import PoseNet  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
depth = bench.to_channels_last(ResNetSAN01(version="18A").to(dev).train())
pose = bench.to_channels_last(PoseNet(nb_ref_imgs=2).to(dev).train())
cl = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
ims = [cl(torch.rand(4, 3, 192, 640, device=dev)) for _ in range(3)]


def step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        sig = depth(ims[0])["inv_depths"]
        p = pose(ims[0], ims[1:])
    loss = sum(s.float().mean() for s in sig) + p.float().square().mean()
    loss.backward()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
for e in prof.key_averages(group_by_stack_n=6):
    k = e.key
    if any(w in k for w in ("copy", "cat", "fill_", "to_copy", "contiguous", "zero_")) and e.device_time_total > 0:
        print(f"{e.count:3d} x {e.device_time_total / max(e.count, 1):7.1f} us  {k}")
        for fr in (e.stack or [])[:6]:
            print("        ", fr)
