"""dL/dpose and dL/dsig of the kitti full-res photometric case (test_kitti_full_res_golden) through K12
for each given library, against each other and the float64 oracle.
  python tools/diag_k12_pose.py LIB..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_util as gu  # noqa: E402
from packnet_sfm_amd import _hip  # noqa: E402
from oracle import photometric_oracle as O  # noqa: E402

B, H, W = 1, 192, 640
z = gu.load_golden("loss_kitti_1img")
g = torch.Generator().manual_seed(int(z["seed"]))
image = gu.smooth_texture(g, B, 3, H, W)
ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
K = gu.kitti_K(B, H, W)
vec = gu.pose_vecs(g, B, 2)
sigs = [gu.sigmoid_maps(g, B, H, W) for _ in range(4)]
mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(2)]
s64 = [s.detach().double().requires_grad_(True) for s in sigs]
v64 = vec.detach().double().requires_grad_(True)
m64 = [O.pose_vec_to_mat(v64[:, j]) for j in range(2)]
O.photometric_loss(image.double(), [c.double() for c in ctx], s64, K.double(), K.double(), m64, None)[0].sum().backward()
ref_pose = v64.grad.numpy()
print("oracle fp64 dpose", ref_pose.reshape(-1), flush=True)
res = {}
for lib in sys.argv[1:]:
    _hip.LIB_PATH = os.path.abspath(lib)
    _hip._lib = None
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    dev = torch.device("cuda")
    s_d = [s.to(dev).requires_grad_(True) for s in sigs]
    v_d = vec.to(dev).requires_grad_(True)
    fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                  photometric_reduce_op="min", automask_loss=True, clip_loss=0.0,
                                  min_depth=0.5, max_depth=80.0)
    out = fn(image.to(dev), [c.to(dev) for c in ctx], s_d, K.to(dev), K.to(dev),
             [Pose.from_vec(v_d[:, j], "euler") for j in range(2)], mask=torch.ones(B, 1, H, W, device=dev))
    out["loss"].sum().backward()
    gp = v_d.grad.cpu().double().numpy()
    scale = np.abs(ref_pose).max()
    print(lib, "loss", float(out["loss"]), "dpose rel err vs fp64 per entry", (np.abs(gp - ref_pose) / scale).reshape(-1).round(5), flush=True)
    res[lib] = (gp, [s.grad.cpu().double().numpy() for s in s_d])
    for i in range(4):
        e = np.abs(res[lib][1][i] - s64[i].grad.numpy())
        print(f"   dsig{i}: max err / max {e.max() / np.abs(s64[i].grad.numpy()).max():.3e}, px > 1e-3 max: {(e > 1e-3 * np.abs(s64[i].grad.numpy()).max()).sum()}")
libs = list(res)
if len(libs) == 2:
    a, b = res[libs[0]], res[libs[1]]
    print("lib vs lib dpose rel", (np.abs(a[0] - b[0]) / np.abs(ref_pose).max()).reshape(-1).round(5))
    for i in range(4):
        e = np.abs(a[1][i] - b[1][i]).reshape(-1)
        idx = np.argsort(-e)[:5]
        print(f"   dsig{i} lib vs lib: max {e.max():.3e} at {[(int(k) // W, int(k) % W) for k in idx]}, px differing > 1e-3 max: {(e > 1e-3 * np.abs(a[1][i]).max()).sum()}")
