"""(1) What reference cycles does one eager training step leave behind (objects only the garbage
collector frees — a cycle through a tensor with a grad_fn keeps that step's autograd graph)?
(2) Run-to-run spread of the eager bf16 step's gradients under several settings."""
import collections
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
__graft_entry__.build()
import bench  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False


class A:
    depth_net, pose_net, batch, height, width = "ResNetSAN01", "PoseNet", 2, 64, 192


torch.manual_seed(0)
m = bench.to_channels_last(bench.build_model(A, dev))
b = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)


def step(model, amp=True):
    for p in model.parameters():
        p.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
        out = model(b)
    out["loss"].sum().backward()
    torch.cuda.synchronize()
    return {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}


step(m)
gc.collect()
gc.set_debug(gc.DEBUG_SAVEALL)
step(m)
n = gc.collect()
types = collections.Counter(type(o).__name__ for o in gc.garbage)
print(f"[cycles] {n} unreachable objects after one step: {types.most_common(25)}", flush=True)
for o in gc.garbage:
    if type(o).__name__ in ("BackwardCFunction",) or "Backward" in type(o).__name__:
        print("[cycles] autograd node in a cycle:", type(o).__name__, flush=True)
        break
for o in gc.garbage:
    if isinstance(o, dict) and len(o) < 40:
        print("[cycles] dict keys:", list(o.keys())[:20], flush=True)
gc.set_debug(0)
gc.garbage.clear()
gc.collect()


def spread(tag, **kw):
    amp = kw.pop("amp", True)
    m.overlap_pose_net = kw.pop("overlap", True)
    det = kw.pop("det", False)
    torch.backends.cudnn.deterministic = kw.pop("cudnn_det", False)
    torch.use_deterministic_algorithms(det, warn_only=True)
    g1, g2 = step(m, amp), step(m, amp)
    rel = sorted(float((g1[k] - g2[k]).norm() / g2[k].norm().clamp_min(1e-30)) for k in g1)
    print(f"[spread] {tag}: median {rel[len(rel) // 2]:.2e}  max {rel[-1]:.2e}", flush=True)


spread("bf16 default")
spread("bf16 cudnn.deterministic", cudnn_det=True)
spread("fp32 cudnn.deterministic", cudnn_det=True, amp=False)
spread("bf16 pose net on the current stream", overlap=False)
spread("bf16 deterministic algorithms", det=True)
spread("bf16 deterministic + current stream", det=True, overlap=False)
spread("fp32", amp=False)
spread("fp32 deterministic + current stream", amp=False, det=True, overlap=False)
