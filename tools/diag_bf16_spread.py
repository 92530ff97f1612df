#!/usr/bin/env python3
"""Where does the run-to-run spread of the bf16 training step's gradients come from?

Runs the bench's default network step (ResNetSAN01 + PoseNet, bf16 autocast, channels_last, MIOpen
find as bench.py) eagerly three times on the same batch and weights, and an fp32 run with
deterministic MIOpen solvers, and compares stage by stage:
  1. the forward: sigmoid maps and pose vectors (bitwise?);
  2. the loss's gradients w.r.t. them (dL/dsig, dL/dpose: the HIP kernels, deterministic);
  3. every parameter gradient, in backward order (heads first), relative L2 difference — eager
     vs eager (the spread) and bf16 vs the fp32 deterministic step (the bf16 step's error).
Also re-runs the backward with MIOpen restricted to deterministic solvers in bf16, to separate
solver non-determinism from bf16 arithmetic.
  python tools/diag_bf16_spread.py [--batch 4] [--height 192] [--width 640]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--height", type=int, default=192)
ap.add_argument("--width", type=int, default=640)
args = ap.parse_args()

import __graft_entry__  # noqa: E402
__graft_entry__.build()
import bench  # noqa: E402

dev = torch.device("cuda:0")


class A:
    depth_net, pose_net, batch, height, width = "ResNetSAN01", "PoseNet", args.batch, args.height, args.width
    min_depth, max_depth = 0.5, 80.0


torch.manual_seed(0)
model = bench.to_channels_last(bench.build_model(A, dev))
batch = bench.synthetic_batch(args.batch, args.height, args.width, dev, seed=0, channels_last=True)
names = [n for n, _ in model.named_parameters()]


def run(amp, deterministic, benchmark=True):
    torch.backends.cudnn.benchmark = benchmark
    torch.backends.cudnn.deterministic = deterministic
    model.zero_grad(set_to_none=True)
    kept = {}
    d_fwd, p_fwd = model.depth_net.forward, model.pose_net.forward

    def depth_fwd(*a, **k):
        o = d_fwd(*a, **k)
        o = dict(o, inv_depths=[t.clone() for t in o["inv_depths"]])
        for t in o["inv_depths"]:
            t.retain_grad()
        kept["inv"] = o["inv_depths"]
        return o

    def pose_fwd(*a, **k):
        v = p_fwd(*a, **k)
        v.retain_grad()
        kept["vec"] = v
        return v
    model.depth_net.forward, model.pose_net.forward = depth_fwd, pose_fwd
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
            out = model(batch)
        out["loss"].sum().backward()
    finally:
        del model.depth_net.forward, model.pose_net.forward
    torch.cuda.synchronize()
    return {"loss": float(out["loss"]),
            "sig": [t.detach().float().clone() for t in kept["inv"]],
            "dsig": [t.grad.float().clone() for t in kept["inv"]],
            "vec": kept["vec"].detach().float().clone(), "dvec": kept["vec"].grad.float().clone(),
            "grads": {n: (p.grad.detach().float().clone() if p.grad is not None else None)
                      for n, p in model.named_parameters()}}


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def compare(tag, x, y):
    print(f"--- {tag}: loss {x['loss']:.9f} vs {y['loss']:.9f}")
    for i, (a, b) in enumerate(zip(x["sig"], y["sig"])):
        print(f"  sigmoid scale {i}: bitwise {torch.equal(a, b)}  rel {rel(a, b):.2e}")
    print(f"  pose vec: bitwise {torch.equal(x['vec'], y['vec'])}  rel {rel(x['vec'], y['vec']):.2e}")
    for i, (a, b) in enumerate(zip(x["dsig"], y["dsig"])):
        print(f"  dL/dsig scale {i}: bitwise {torch.equal(a, b)}  rel {rel(a, b):.2e}")
    print(f"  dL/dvec: bitwise {torch.equal(x['dvec'], y['dvec'])}  rel {rel(x['dvec'], y['dvec']):.2e}")
    rows = []
    for n in reversed(names):   # backward order: heads first
        a, b = x["grads"][n], y["grads"][n]
        if a is None or b is None:
            continue
        rows.append((n, torch.equal(a, b), rel(a, b)))
    r = sorted(v for _, _, v in rows)
    print(f"  parameter gradients: {sum(e for _, e, _ in rows)}/{len(rows)} bitwise, rel L2 median "
          f"{r[len(r) // 2]:.2e}, max {r[-1]:.2e}")
    first = next(((n, v) for n, e, v in rows if not e), None)
    print(f"  first non-bitwise gradient in backward order: {first}")
    print("   first 12 in backward order:")
    for n, e, v in rows[:12]:
        print(f"   {n:60s} bitwise {e!s:5s} rel {v:.2e}")
    print("   largest 8:")
    for n, e, v in sorted(rows, key=lambda t: -t[2])[:8]:
        print(f"   {n:60s} bitwise {e!s:5s} rel {v:.2e}")


b1, b2 = run(True, False), run(True, False)
compare("bf16 eager vs bf16 eager (MIOpen find, fast solvers)", b1, b2)
d1, d2 = run(True, True, benchmark=False), run(True, True, benchmark=False)
compare("bf16 eager vs bf16 eager (deterministic solvers)", d1, d2)
f32 = run(False, True, benchmark=False)
compare("bf16 (fast solvers) vs fp32 deterministic", b1, f32)
compare("bf16 (deterministic solvers) vs fp32 deterministic", d1, f32)
