"""K12's dL/dsig planes (before grad_finish) of the fisheye multires case (each scale at its own
resolution, the images resized) per library build (--lib), against the first build: where they differ."""
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
a = ap.parse_args()
import __graft_entry__  # noqa: E402
__graft_entry__.build()
import golden_util as gu  # noqa: E402
from packnet_sfm_amd import _hip  # noqa: E402
from packnet_sfm_amd.geometry.pose import Pose  # noqa: E402
from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss  # noqa: E402

tag = "_multires"
z = gu.load_golden("fisheye_small")
T = lambda x: torch.from_numpy(np.ascontiguousarray(x))  # noqa: E731
dev = torch.device("cuda:0")
img, ctx = T(z[f"image{tag}"]).to(dev), [T(z[f"ctx0{tag}"]).to(dev), T(z[f"ctx1{tag}"]).to(dev)]
H, W = img.shape[-2:]
intr = {k: T(z[f"intr_{k}"]).to(dev) for k in ("k", "s", "div", "ux", "uy")}
vec = T(z[f"pvec{tag}"]).to(dev)
coarse = [T(z[f"sig{i}{tag}"]).to(dev) for i in range(4)]
full = [F.interpolate(c, size=(H, W), mode="nearest") for c in coarse]


def planes(sigs):
    fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                  photometric_reduce_op="min", automask_loss=True, clip_loss=0.0, min_depth=0.5,
                                  max_depth=80.0)
    s = [t.clone().requires_grad_(True) for t in sigs]
    out = fn(img, ctx, s, intr, intr, [Pose.from_vec(vec[:, j], "euler") for j in range(2)])
    torch.cuda.synchronize()
    c = out["loss"].grad_fn.calls
    return [g.clone() for cc in c for g in cc.gsig], float(out["loss"])


np.set_printoptions(precision=3, linewidth=220, suppress=True)
first = None
for lib in a.lib or [None]:
    if lib:
        _hip.LIB_PATH = lib
        _hip._lib = None
    pc, lc = planes(coarse)
    print(f"== {lib}: loss {lc:.9f}")
    if first is not None:
        for i, (x, y) in enumerate(zip(pc, first)):
            d = (x - y).abs()
            print(f"  plane {i} {tuple(x.shape)}: max diff {float(d.max()):.3e} at {np.unravel_index(int(d.argmax()), d.shape)}; "
                  f"{int((d > 1e-3 * float(y.abs().max())).sum())} px over 1e-3 max", flush=True)
            if float(d.max()) > 1e-3 * float(y.abs().max()):
                b, _, r, cc = np.unravel_index(int(d.argmax()), d.shape)
                sl = (b, 0, slice(max(r - 3, 0), r + 4), slice(max(cc - 3, 0), cc + 4))
                print("   first x1e5\n", y[sl].cpu().numpy() * 1e5)
                print("   this - first x1e5\n", (x - y)[sl].cpu().numpy() * 1e5)
    else:
        first = pc
