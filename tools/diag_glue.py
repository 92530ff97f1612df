"""ATen glue kernels of a depth + pose step (bf16 weights as the graph trainer keeps them, bf16
autocast, channels_last): torch.profiler op table with input shapes for every copy / cat / cast /
elementwise / reduce op.  python tools/diag_glue.py [packnet-san|resnet-san]"""
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")
import bench  # noqa: E402
import packnet_sfm_amd  # noqa: E402,F401
from packnet_sfm_amd.networks.pose.PoseNet import PoseNet  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "packnet-san"
dev = torch.device("cuda")
torch.manual_seed(0)
if which == "packnet-san":
    from packnet_sfm_amd.networks.depth.PackNetSAN01 import PackNetSAN01
    depth, B = PackNetSAN01(version="1A", dropout=0.5).to(dev), 6
else:
    from packnet_sfm_amd.networks.depth.ResNetSAN01 import ResNetSAN01
    depth, B = ResNetSAN01(version="18A").to(dev), 4
pose = PoseNet(nb_ref_imgs=2).to(dev)
for m in (depth, pose):
    m.train()
    bench.to_channels_last(m)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
cl = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
ims = [cl(torch.rand(B, 3, 192, 640, device=dev)) for _ in range(3)]


def step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        sig = depth(ims[0])["inv_depths"]
        p = pose(ims[0], ims[1:])
    loss = sum(s.float().mean() for s in sig) + p.float().square().mean()
    loss.backward()


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    step()
    torch.cuda.synchronize()
words = ("copy", "cat", "to_copy", "add", "mul", "sub", "div", "sum", "mean", "pad", "clone", "contiguous", "fill",
         "zero", "where", "elu", "sigmoid", "pixel", "reshape", "cumsum", "interpolate", "upsample")
rows = []
for e in prof.key_averages(group_by_input_shape=True):
    if e.key.startswith("aten::") and any(w in e.key for w in words) and e.device_time_total > 0:
        rows.append((e.device_time_total, e.count, e.key, str(e.input_shapes)[:150]))
for t, n, k, sh in sorted(rows, reverse=True)[:60]:
    print(f"{t:9.1f} us {n:4d} x  {k:28s} {sh}")
