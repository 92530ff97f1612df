"""Micro-benchmark of the fused pack/unpack Conv3d (include/psfm_pack3d.h) on PackNet01's five pack
and five unpack shapes at B=6, 192x640, bf16 channels_last: per-call GPU time from HIP events
around graph replays.  --lib PATH (repeatable) A/Bs alternative builds in one process."""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", action="append", default=[])
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--net", default="packnet", choices=["packnet", "packnet-san"],
                help="packnet: PackNet01 (d=8, n1=64); packnet-san: PackNetSAN01 (d=4, n1=32)")
ap.add_argument("--only", default="", help="run only the case with this key (e.g. pack64x192x640)")
ap.add_argument("--dx", default="", help="comma list of PSFM_P3D_DX forms to A/B (mfma, cl); empty: the default")
ap.add_argument("--fwd", default="", help="comma list of PSFM_P3D_FWD forms to A/B (mfma, valu); empty: the default")
ap.add_argument("--dw", default="", help="comma list of PSFM_P3D_DW forms to A/B (mfma, generic); empty: the default")
args = ap.parse_args()
__graft_entry__.build()
from packnet_sfm_amd import _hip  # noqa: E402
from packnet_sfm_amd.networks.layers.packnet import pack3d as P  # noqa: E402

dev = torch.device("cuda:0")
B = 6
if args.net == "packnet":
    D = 8
    PACK = [(64, 192, 640), (64, 96, 320), (128, 48, 160), (256, 24, 80), (512, 12, 40)]
    UNPACK = [(256, 6, 20), (128, 12, 40), (64, 24, 80), (32, 48, 160), (32, 96, 320)]  # conv2d outputs
else:
    D = 4
    PACK = [(32, 192, 640), (64, 96, 320), (128, 48, 160), (256, 24, 80), (512, 12, 40)]
    UNPACK = [(512, 6, 20), (256, 12, 40), (128, 24, 80), (64, 48, 160), (32, 96, 320)]
cases = [(0, c) for c in PACK] + [(1, c) for c in UNPACK]


def timed(fn, iters):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / iters


for lib, form, dwf, fwf in [(lb, f, w, fw) for lb in (args.lib or [None]) for f in args.dx.split(",")
                            for w in args.dw.split(",") for fw in args.fwd.split(",")]:
    for k, v in (("PSFM_P3D_DX", form), ("PSFM_P3D_DW", dwf), ("PSFM_P3D_FWD", fwf)):
        if v:
            os.environ[k] = v
        else:
            os.environ.pop(k, None)
    if lib:
        _hip.LIB_PATH = lib
        _hip._lib = None
    res, tot = {}, [0.0, 0.0, 0.0]
    for mode, (C, H, W) in cases:
        if args.only and args.only != f"{'pack' if mode == 0 else 'unpack'}{C}x{H}x{W}":
            continue
        x = torch.randn(B, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(D, 1, 3, 3, 3, device=dev) * 0.2
        b = torch.randn(D, device=dev) * 0.1
        y = torch.empty(P._out_shape(mode, x, 2, D), device=dev, dtype=x.dtype, memory_format=torch.channels_last)
        gy = torch.randn(y.shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gx = torch.empty_like(x)
        gw = torch.empty(D, 27, device=dev)
        gb = torch.empty(D, device=dev)
        d = P._desc(mode, x, y, 2, D)
        ws = torch.empty(max(_hip.lib().psfm_p3d_ws_floats(ctypes.byref(d)), 1), device=dev)
        wf = w.reshape(D, 27).contiguous()
        L, st = _hip.lib(), lambda: _hip.stream(dev)
        t_f = timed(lambda: L.psfm_p3d_fwd(ctypes.byref(d), _hip.ptr(x), _hip.ptr(wf), _hip.ptr(b), _hip.ptr(y), st()), args.iters)
        t_x = timed(lambda: L.psfm_p3d_bwd(ctypes.byref(d), _hip.ptr(x), _hip.ptr(wf), _hip.ptr(gy), _hip.ptr(gx), None, None, None,
                                           st()), args.iters)
        t_w = timed(lambda: L.psfm_p3d_bwd(ctypes.byref(d), _hip.ptr(x), _hip.ptr(wf), _hip.ptr(gy), None, _hip.ptr(gw), _hip.ptr(gb),
                                           _hip.ptr(ws), st()), args.iters)
        key = f"{'pack' if mode == 0 else 'unpack'}{C}x{H}x{W}"
        res[key] = [round(t_f, 1), round(t_x, 1), round(t_w, 1)]
        tot = [tot[0] + t_f, tot[1] + t_x, tot[2] + t_w]
    res["total_fwd_bwdx_bwdw_us"] = [round(t, 1) for t in tot]
    print(lib or "default", "dx=" + (form or "default"), "dw=" + (dwf or "default"), "fwd=" + (fwf or "default"), json.dumps(res), flush=True)
