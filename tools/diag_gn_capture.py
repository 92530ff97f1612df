#!/usr/bin/env python3
"""Bisect the HIP-graph capture segfault of tools/gn_bench.py: its first shape,
[6, 64, 192, 640] + conv bias, 20 forward-only psfm_gn_act calls captured under no_grad, crashed in
torch.cuda.graphs capture_end (profiles/r03/cap/gn_bench_graph_crash.log), while the same capture in
tools/diag_capture_fwd.py passed.  Each flag adds one thing gn_bench does before its capture:

  --live-grad    a grad-enabled gn_act call on the same shape whose autograd graph stays alive, and
                 dy = randn_like(y) (gn_bench.py:111-113)
  --cpu-model    the PackNet01 + PoseNet model built and its depth net run on the CPU first, with
                 gn_act wrapped by a recorder in every module that imported it (gn_bench.py:50-70)
  --no-bench     torch.backends.cudnn.benchmark = False (gn_bench.py:37)
  --side-warmup  the warm-up calls on a side stream (gn_bench.py:80-86) instead of the current one
  --keep         keep the captured calls' outputs alive (tools/diag_capture_fwd.py does; gn_bench's
                 timed() drops them, so their blocks are freed and re-used inside the capture)
  --drop-all     drop the LAST captured call's output too (default keeps it, to compare the replay)
  --events       create two timing events before the capture (gn_bench.py:87) and record them
                 around a second replay

  --capture-bwd  capture `torch.autograd.grad(y, xg, dy, retain_graph=True)` x iters instead of the
                 forward (what gn_bench.py:119 — the crashing line — actually times); y from a forward
                 run BEFORE the capture on the default stream, as gn_bench does
  --bwd-on-capture-stream  with --capture-bwd: run that forward on the stream the graph then captures on

One configuration per process (a segfault ends it); prints OK on a clean capture + replay."""
import argparse
import faulthandler
import os
import sys

import torch

faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--live-grad", action="store_true")
ap.add_argument("--cpu-model", action="store_true")
ap.add_argument("--no-bench", action="store_true")
ap.add_argument("--side-warmup", action="store_true")
ap.add_argument("--keep", action="store_true")
ap.add_argument("--drop-all", action="store_true")
ap.add_argument("--capture-bwd", action="store_true")
ap.add_argument("--bwd-on-capture-stream", action="store_true")
ap.add_argument("--torch-chain", action="store_true", help="with --capture-bwd: torch's own GroupNorm + ELU ops")
ap.add_argument("--events", action="store_true")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--shape", default="6,64,192,640")
args = ap.parse_args()
import __graft_entry__  # noqa: E402

__graft_entry__.build()
from packnet_sfm_amd.networks.layers import fused as FU  # noqa: E402

dev = torch.device("cuda:0")
if args.no_bench:
    torch.backends.cudnn.benchmark = False
orig = FU.gn_act
if args.cpu_model:
    import bench

    class A:
        depth_net, pose_net, batch, height, width = "PackNet01", "PoseNet", 1, 192, 640

    model = bench.build_model(A, torch.device("cpu"))
    seen = []

    def rec(x, bias, gn, relu=True, act=None, residual=None):
        seen.append(tuple(x.shape))
        return orig(x, bias, gn, relu=relu, act=act, residual=residual)

    for mod in list(sys.modules.values()):
        if getattr(mod, "gn_act", None) is orig and mod is not FU:
            mod.gn_act = rec
    FU.gn_act = rec
    b = bench.synthetic_batch(1, 192, 640, torch.device("cpu"), seed=0)
    with torch.no_grad():
        model.depth_net(b["rgb"])
    print(f"cpu model: {len(seen)} gn_act calls", flush=True)
shape = tuple(int(v) for v in args.shape.split(","))
C = shape[1]
gn = torch.nn.GroupNorm(16, C).to(dev)
x = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
bias = torch.randn(C, device=dev)
keep = None
if args.capture_bwd:
    if args.torch_chain:   # the reference op chain (autocast-style fp32 GN on the bf16 input)
        orig = lambda x_, b_, gn_, act=None: torch.nn.functional.elu(gn_(x_.float() + b_.view(1, -1, 1, 1)))  # noqa: E731
    cs = torch.cuda.Stream()
    xg = x.detach().requires_grad_(True)
    dy = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if args.torch_chain:
        dy = dy.float()
    if args.bwd_on_capture_stream:
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            y = orig(xg, bias, gn, act=FU.ACT_ELU)
        torch.cuda.current_stream().wait_stream(cs)
    else:
        y = orig(xg, bias, gn, act=FU.ACT_ELU)
    ref = torch.autograd.grad(y, xg, dy, retain_graph=True)[0].clone()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cs):
        for _ in range(args.iters - 1):
            torch.autograd.grad(y, xg, dy, retain_graph=True)
        out = torch.autograd.grad(y, xg, dy, retain_graph=True)[0]
    g.replay()
    torch.cuda.synchronize()
    ok = torch.equal(out, ref)
    print(f"OK backward capture + replay ({vars(args)}), dx equals eager: {ok}", flush=True)
    sys.exit(0 if ok else 1)
if args.live_grad:
    xg = x.detach().requires_grad_(True)
    y = orig(xg, bias, gn, act=FU.ACT_ELU)
    keep = (y, xg, torch.randn_like(y))
with torch.no_grad():
    fn = lambda: orig(x, bias, gn, act=FU.ACT_ELU)  # noqa: E731
    ref = fn().clone()
    if args.side_warmup:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(s)
    else:
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    if args.events:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        if args.keep:
            outs = [fn() for _ in range(args.iters)]
        elif args.drop_all:
            for _ in range(args.iters):
                fn()
            outs = []
        else:
            for _ in range(args.iters - 1):
                fn()
            outs = [fn()]
    g.replay()
    if args.events:
        e0.record()
        g.replay()
        e1.record()
    torch.cuda.synchronize()
ok = all(torch.equal(o, ref) for o in outs)
print(f"OK capture + replay ({vars(args)}), outputs equal eager: {ok}", flush=True)
sys.exit(0 if ok else 1)
