"""Micro-benchmark of the fused normalisation epilogues (psfm_netops) against the reference op
chain (MIOpen BatchNorm + ReLU / GroupNorm + ReLU) at the ResNet18-SAN / PoseNet layer shapes of
the bench workload (B=4, 192x640).  Meant to run under rocprofv3 --kernel-trace (per-kernel,
per-grid durations via tools/summarize_trace.py --grid); also prints HIP-event wall per layer.
  python tools/netops_bench.py [--lib path/to/libpsfm_hip.so] [--iters 30] [--mode fused|ref]"""
import argparse
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--mode", default="fused", choices=["fused", "ref"])
args = ap.parse_args()
import packnet_sfm_amd  # noqa: E402,F401
from packnet_sfm_amd import _hip  # noqa: E402
if args.lib:
    _hip.LIB_PATH = args.lib
from packnet_sfm_amd.networks.layers import fused as FU  # noqa: E402

FU.FUSE.update(bias=args.mode == "fused", gn=args.mode == "fused", bn=args.mode == "fused")
dev = torch.device("cuda:0")
BN_SHAPES = [(4, 64, 96, 320), (4, 64, 48, 160), (4, 128, 24, 80), (4, 256, 12, 40), (4, 512, 6, 20)]
GN_SHAPES = [(4, 16, 96, 320), (4, 32, 48, 160), (4, 64, 24, 80), (4, 128, 12, 40), (4, 256, 6, 20)]
g = torch.Generator(device="cpu").manual_seed(0)


def cl(t):
    return t.contiguous(memory_format=torch.channels_last)


for kind, shapes in (("bn", BN_SHAPES), ("gn", GN_SHAPES)):
    for shape in shapes:
        C = shape[1]
        x = cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16).requires_grad_(True)
        dy = cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16)
        if kind == "bn":
            m = nn.BatchNorm2d(C).to(dev).train()
            fn = (lambda: FU.bn_act(x, m, relu=True)) if args.mode == "fused" else \
                (lambda: torch.relu(m(x)))
        else:
            m = nn.GroupNorm(16, C).to(dev)
            b = torch.zeros(C, device=dev, dtype=torch.bfloat16, requires_grad=True)
            fn = (lambda: FU.gn_act(x, b, m, relu=True)) if args.mode == "fused" else \
                (lambda: torch.relu(m(x + b.view(1, -1, 1, 1))))
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.mode == "ref"):
            for _ in range(3):
                fn().backward(dy)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn().backward(dy)
            e1.record()
        torch.cuda.synchronize()
        print(f"{args.mode} {kind} {str(shape):22s} fwd+bwd {1000 * e0.elapsed_time(e1) / args.iters:8.1f} us (eager)",
              flush=True)
