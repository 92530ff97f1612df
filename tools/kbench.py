"""Photometric-kernel micro-benchmark (B=4, 192x640, 2 contexts, 4 full-res scales): per-kernel
durations from HIP events, fwd+bwd of MultiViewPhotometricLoss only.  Optional: --lib PATH loads an
alternative build of libpsfm_hip.so (A/B of kernel variants in one process)."""
import argparse
import json
import sys

import torch

import os  # noqa: E402
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
import golden_util as gu  # noqa: E402
import __graft_entry__  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", action="append", default=[])
ap.add_argument("--iters", type=int, default=30)
ap.add_argument("--B", type=int, default=4)
ap.add_argument("--H", type=int, default=192)
ap.add_argument("--W", type=int, default=640)
ap.add_argument("--paths", default="k12,k1k2")
ap.add_argument("--prio", default="", help="comma list of PSFM_K12_PRIO modes to run (K12 wave-pair balance)")
ap.add_argument("--reps", type=int, default=1, help="repeat the whole lib x prio sweep (interleaved A/B)")
ap.add_argument("--noisy", action="store_true",
                help="i.i.d. U[0, 2] per-pixel sigmoid maps (what a random-init PackNetSAN01's InvDepth heads "
                     "produce: sigmoid / min_depth, no spatial smoothness) instead of smooth maps in [0.01, 0.2]")
args = ap.parse_args()
__graft_entry__.build()
from packnet_sfm_amd import _hip  # noqa: E402
from packnet_sfm_amd.geometry.pose import Pose  # noqa: E402
from packnet_sfm_amd.losses import _hip_photometric as HP  # noqa: E402
from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss  # noqa: E402

dev = torch.device("cuda:0")
B, H, W = args.B, args.H, args.W
g = torch.Generator().manual_seed(0)
image = gu.smooth_texture(g, B, 3, H, W).to(dev)
ctx = [gu.smooth_texture(g, B, 3, H, W).to(dev) for _ in range(2)]
K = gu.kitti_K(B, H, W).to(dev)
vec = gu.pose_vecs(g, B, 2).to(dev)
if args.noisy:
    sigs = [(2.0 * torch.rand(B, 1, H, W, generator=g)).to(dev).requires_grad_(True) for _ in range(4)]
else:
    sigs = [gu.sigmoid_maps(g, B, H, W).to(dev).requires_grad_(True) for _ in range(4)]
poses = [Pose.from_vec(vec[:, j], "euler") for j in range(2)]
fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                              photometric_reduce_op="min", automask_loss=True, clip_loss=0.0,
                              min_depth=0.5, max_depth=80.0)
results = {}
runs = [(lib, pm) for _ in range(args.reps) for lib in (args.lib or [None])
        for pm in (args.prio.split(",") if args.prio else [None])]
for lib, pm in runs:
    if lib:
        _hip.LIB_PATH = lib
        _hip._lib = None
    if pm is not None:
        os.environ["PSFM_K12_PRIO"] = pm
    for fused in [p == "k12" for p in args.paths.split(",")]:
        HP.FUSED_GRAD = fused
        for _ in range(2):
            fn(image, ctx, sigs, K, K, poses)["loss"].sum().backward()
        torch.cuda.synchronize()
        HP.KERNEL_TIMING["record"] = rec = []
        out = fn(image, ctx, sigs, K, K, poses)
        out["loss"].sum().backward()
        HP.KERNEL_TIMING["record"] = None
        res = {k: round(v, 2) for k, v in HP.graph_replay_times_us(rec, dev, reps=10, iters=args.iters).items()}
        res["total_us"] = round(sum(res.values()), 2)
        res["loss"] = float(out["loss"].detach())
        tag = (lib or "default") + (" k12" if fused else " k1k2") + (f" prio{pm}" if pm is not None else "")
        results[tag] = res
        print(tag, json.dumps(res), flush=True)
