"""Fused GroupNorm + ELU (psfm_gn_act) at the layer shapes of a PackNet step: records every
gn_act call of one forward of the configured depth net, then times each distinct shape's forward
(stats + apply) and backward (stats + apply) between HIP events, and prints
the algorithmic HBM bytes per pass and the fraction of 8 TB/s.
  python tools/gn_bench.py [--depth-net PackNet01] [--batch 6] [--iters 20]
Algorithmic bytes (bf16 activations, 2 B/elem; residual r where the layer has one):
  fwd: stats reads x (+r), apply reads x (+r) and writes y          -> (2 + 2r + 1) * 2 B/elem
  bwd: stats reads dy, x (+r), apply reads dy, x (+r), writes dx (+dr) -> (4 + 2r + 1 + r) * 2 B/elem"""
import argparse
import collections
import faulthandler
import json
import os
import sys

import torch

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--depth-net", default="PackNet01")
ap.add_argument("--batch", type=int, default=6)
ap.add_argument("--height", type=int, default=192)
ap.add_argument("--width", type=int, default=640)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--lib", default=None)
ap.add_argument("--net", default="depth", choices=["depth", "pose"], help="record the depth or the pose net's GN calls")
ap.add_argument("--eager", action="store_true", help="time eager calls (default: HIP-graph replays of --iters calls)")
# capture-crash bisection (tools/diag_gn_capture.py): drop one step of the sequence
ap.add_argument("--max-shapes", type=int, default=0, help="stop after this many shapes (0: all)")
ap.add_argument("--no-live-grad", action="store_true", help="no grad-enabled call kept alive before the timing")
ap.add_argument("--no-events", action="store_true", help="create the timing events after the capture")
ap.add_argument("--fwd-only", action="store_true", help="time the forward only")
args = ap.parse_args()
import __graft_entry__  # noqa: E402

__graft_entry__.build()
from packnet_sfm_amd import _hip  # noqa: E402

if args.lib:
    _hip.LIB_PATH, _hip._lib = args.lib, None
import bench  # noqa: E402
from packnet_sfm_amd.networks.layers import fused as FU  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False


class A:
    depth_net, pose_net, batch, height, width = args.depth_net, "PoseNet", args.batch, args.height, args.width


# layer shapes from one forward of the net on the CPU at batch 1 (no MIOpen kernels to build on a
# cold box); the batch is applied below
model = bench.build_model(A, torch.device("cpu"))
calls = collections.OrderedDict()
orig = FU.gn_act


def rec(x, bias, gn, relu=True, act=None, residual=None):
    key = (tuple(x.shape), residual is not None, bias is not None, int(gn.num_groups), act)
    calls[key] = calls.get(key, 0) + 1
    return orig(x, bias, gn, relu=relu, act=act, residual=residual)


for mod in list(sys.modules.values()):
    if getattr(mod, "gn_act", None) is orig and mod is not FU:
        mod.gn_act = rec
FU.gn_act = rec
b = bench.synthetic_batch(1, args.height, args.width, torch.device("cpu"), seed=0)
with torch.no_grad():
    if args.net == "depth":
        model.depth_net(b["rgb"])
    else:
        model.pose_net(b["rgb"], b["rgb_context"])
print(f"{sum(calls.values())} gn_act calls, {len(calls)} shapes", flush=True)


# ONE stream for the recorded forwards, the warm-ups and the captures.  The round-3 segfault in
# capture_end (profiles/r03/cap/gn_bench_graph_crash.log, line 119 = the BACKWARD timing) was the
# backward of a forward that ran on the default stream, captured on torch.cuda.graph's own stream:
# the autograd engine runs each backward op on its forward's stream, so those launches went to a
# stream outside the capture (HIP then crashes at capture end instead of refusing the launch;
# tools/diag_gn_capture.py --capture-bwd reproduces it, --bwd-on-capture-stream passes bit-exactly).
cs = torch.cuda.Stream()


def timed(fn):
    """Per-call GPU time: a HIP graph of args.iters calls replayed between two HIP events (no host
    launch gaps; --eager: back-to-back eager calls, an upper bound for small shapes)."""
    s = cs
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    if not args.no_events:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if args.eager:
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
    else:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=cs):
            for _ in range(args.iters):
                fn()
        g.replay()
        if args.no_events:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / args.iters


tot = collections.Counter()
for ishape, ((shape, has_res, has_bias, ng, act), n) in enumerate(calls.items()):
    if args.max_shapes and ishape >= args.max_shapes:
        break
    shape = (args.batch,) + shape[1:]
    N, C, H, W = shape
    gn = torch.nn.GroupNorm(ng, C).to(dev)
    x = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x) if has_res else None
    bias = torch.randn(C, device=dev) if has_bias else None
    if not args.no_live_grad:
        xg = x.detach().requires_grad_(True)
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):   # the backward then runs (and is captured) on cs
            y = orig(xg, bias, gn, act=act, residual=r)
            dy = torch.randn_like(y)
        torch.cuda.current_stream().wait_stream(cs)
    with torch.no_grad():   # the forward-only call (eval), as a training step's forward costs the same
        fwd_us = timed(lambda: orig(x, bias, gn, act=act, residual=r))
    bwd_us = 0.0 if (args.fwd_only or args.no_live_grad) else \
        timed(lambda: torch.autograd.grad(y, xg, dy, retain_graph=True))
    el = x.numel()
    rr = 1 if has_res else 0
    fb, bb = (3 + 2 * rr) * 2 * el, (5 + 3 * rr) * 2 * el
    line = {"shape": shape, "res": has_res, "bias": has_bias, "calls_per_fwd": n,
            "fwd_us": round(fwd_us, 2), "fwd_frac": round(fb / (fwd_us * 1e-6) / 8e12, 3),
            "bwd_us": round(bwd_us, 2), "bwd_frac": round(bb / (bwd_us * 1e-6) / 8e12, 3) if bwd_us else None}
    tot["fwd_us"] += n * fwd_us
    tot["bwd_us"] += n * bwd_us
    tot["bytes"] += n * (fb + bb)
    print(json.dumps(line), flush=True)
print(json.dumps({"total_fwd_us": round(tot["fwd_us"], 1), "total_bwd_us": round(tot["bwd_us"], 1)}))
