"""Composed pack layer fwd + bwd at one PackNet shape, N iterations, with per-kernel-group HIP-event
timing (for rocprofv3 PMC passes and A/B of k_pc_conv / k_pc_wgrad variants).
  python tools/pc_layer_run.py [--shape B,C,H,W,d,k] [--iters N] [--lib PATH]..."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="6,64,192,640,8,5")
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--lib", action="append", default=[])
ap.add_argument("--reps", type=int, default=1)
a = ap.parse_args()
import __graft_entry__  # noqa: E402
__graft_entry__.build()
from packnet_sfm_amd import _hip  # noqa: E402
from packnet_sfm_amd.networks.layers.packnet import packconv  # noqa: E402

B, C, H, W, d, k = (int(v) for v in a.shape.split(","))
g = torch.Generator().manual_seed(0)
x = torch.randn(B, C, H, W, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=torch.channels_last)
W2 = (torch.randn(C, 4 * C * d, k, k, generator=g) / (4 * C * d * k * k) ** 0.5).cuda().requires_grad_(True)
w3 = (torch.randn(d, 1, 3, 3, 3, generator=g) / 27 ** 0.5).cuda().requires_grad_(True)
b3 = (0.3 * torch.randn(d, generator=g)).cuda().requires_grad_(True)
gy = torch.randn(B, C, H // 2, W // 2, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=torch.channels_last)
x.requires_grad_(True)


def ev(fn, n):
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[len(ts) // 2]


for _ in range(a.reps):
    for lib in a.lib or [None]:
        if lib:
            _hip.LIB_PATH = lib
            _hip._lib = None
        y = packconv.PackConvFn.apply(x, W2, w3, b3, k)
        y.backward(gy)
        torch.cuda.synchronize()
        ref = (y.float().clone(), x.grad.float().clone(), W2.grad.clone())
        x.grad = W2.grad = w3.grad = b3.grad = None
        tf = ev(lambda: packconv.PackConvFn.apply(x, W2, w3, b3, k), a.iters)
        tb = ev(lambda: packconv.PackConvFn.apply(x, W2, w3, b3, k).backward(gy), a.iters)
        print(f"{lib or 'in-tree'} {(B, C, H, W, d, k)}: fwd {tf:.0f} us, fwd+bwd {tb:.0f} us, "
              f"|y| {float(ref[0].norm()):.6e} |dx| {float(ref[1].norm()):.6e} |dW2| {float(ref[2].norm()):.6e}",
              flush=True)
