"""The fisheye multires case with its coarse sigmoid maps nearest-upsampled to full resolution
(the same loss): per-pixel dL/dsig of several library builds against the float64 oracle, around a
region (--rows, --cols) of scale --scale."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", action="append", default=[])
ap.add_argument("--scale", type=int, default=1)
ap.add_argument("--rows", default="1,7")
ap.add_argument("--cols", default="32,41")
a = ap.parse_args()
import __graft_entry__  # noqa: E402
__graft_entry__.build()
import golden_util as gu  # noqa: E402
from oracle import photometric_oracle as O  # noqa: E402
from packnet_sfm_amd import _hip  # noqa: E402
from packnet_sfm_amd.geometry.pose import Pose  # noqa: E402
from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss  # noqa: E402

tag = "_multires"
z = gu.load_golden("fisheye_small")
T = lambda x: torch.from_numpy(np.ascontiguousarray(x))  # noqa: E731
img, ctx = T(z[f"image{tag}"]), [T(z[f"ctx0{tag}"]), T(z[f"ctx1{tag}"])]
H, W = img.shape[-2:]
intr = {k: T(z[f"intr_{k}"]) for k in ("k", "s", "div", "ux", "uy")}
pvec = T(z[f"pvec{tag}"])
full = [F.interpolate(T(z[f"sig{i}{tag}"]).float(), size=(H, W), mode="nearest") for i in range(4)]
r0, r1 = (int(v) for v in a.rows.split(","))
c0, c1 = (int(v) for v in a.cols.split(","))
np.set_printoptions(precision=3, linewidth=220, suppress=True)
# float64 oracle
sd = [f.double().requires_grad_(True) for f in full]
loss = O.photometric_loss(img.double(), [c.double() for c in ctx], sd, {k: v.double() for k, v in intr.items()},
                          {k: v.double() for k, v in intr.items()}, [O.pose_vec_to_mat(pvec[:, j].double()) for j in range(2)],
                          None, num_scales_=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                          photometric_reduce_op="min", automask_loss=True, min_depth=0.5, max_depth=80.0)
loss[0].sum().backward()
ref = sd[a.scale].grad[0, 0, r0:r1, c0:c1].numpy() * 1e5
print("fp64 oracle x1e5\n", ref)
dev = torch.device("cuda:0")
for lib in a.lib or [None]:
    if lib:
        _hip.LIB_PATH = lib
        _hip._lib = None
    sigs = [f.to(dev).requires_grad_(True) for f in full]
    vec = pvec.to(dev)
    fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                  photometric_reduce_op="min", automask_loss=True, clip_loss=0.0, min_depth=0.5,
                                  max_depth=80.0)
    di = {k: v.to(dev) for k, v in intr.items()}
    out = fn(img.to(dev), [c.to(dev) for c in ctx], sigs, di, di, [Pose.from_vec(vec[:, j], "euler") for j in range(2)])
    out["loss"].sum().backward()
    g = sigs[a.scale].grad[0, 0, r0:r1, c0:c1].cpu().numpy() * 1e5
    print(f"{lib or 'in-tree'} x1e5 (minus fp64)\n", g - ref, flush=True)
