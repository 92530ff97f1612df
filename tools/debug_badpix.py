"""Unflagged pixels where the HIP dL/dsig differs from the oracle (B=4 192x640 parity case):
print the fp64 diagnostics at each (candidate margins, distance of the warp coordinates to an
integer, |warp - target|, SSIM values) to see which discontinuity they sit on."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
__graft_entry__.build()
import golden_util as gu  # noqa: E402
from oracle import photometric_oracle as O  # noqa: E402
from packnet_sfm_amd.geometry.pose import Pose  # noqa: E402
from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss  # noqa: E402

torch.set_num_threads(16)
dev = torch.device("cuda:0")
B, H, W = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (4, 192, 640)
if len(sys.argv) > 4 and sys.argv[4] == "k1k2":   # the unfused K1 forward / K2 + K3 backward
    from packnet_sfm_amd.losses import _hip_photometric as HP
    HP.FUSED_GRAD = False
g = torch.Generator().manual_seed(4000 + B * 7 + H)
image = gu.smooth_texture(g, B, 3, H, W)
ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
K = gu.kitti_K(B, H, W)
K[:, 0, 2] += torch.linspace(-0.02, 0.02, B) * W
vec = gu.pose_vecs(g, B, 2)
sigs = [gu.sigmoid_maps(g, B, H, W) for _ in range(4)]
mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(2)]
s_c = [s.clone().requires_grad_(True) for s in sigs]
O.photometric_loss(image, ctx, s_c, K, K, mats, None)[0].sum().backward()
sens, ties = O.sensitive_pixels(image, ctx, sigs, K, mats, 0.5, 80.0, return_ties=True)
s_d = [s.to(dev).requires_grad_(True) for s in sigs]
v_d = vec.to(dev)
fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                              photometric_reduce_op="min", automask_loss=True, clip_loss=0.0, min_depth=0.5,
                              max_depth=80.0)
fn(image.to(dev), [c.to(dev) for c in ctx], s_d, K.to(dev), K.to(dev),
   [Pose.from_vec(v_d[:, j], "euler") for j in range(2)])["loss"].sum().backward()
torch.cuda.synchronize()
# fp64 diagnostics (and the oracle's gradient in float64)
img = image.double()
s64 = [s.double().requires_grad_(True) for s in sigs]
O.photometric_loss(img, [c.double() for c in ctx], s64, K.double(), K.double(), [m.double() for m in mats],
                   None)[0].sum().backward()
for i in range(4):
    got, ref = s_d[i].grad.cpu().double(), s_c[i].grad.double()
    lim = 1e-3 * ref.abs().max()
    bad = ((got - ref).abs() > lim) & ((got - s64[i].grad).abs() > lim) & ~sens[i]
    idx = bad.nonzero().tolist()
    print(f"scale {i}: {len(idx)} unflagged bad pixels, lim {float(lim):.3e}")
    s = sigs[i].double()
    depth = 1.0 / (1.0 / (O.sigmoid_to_depth(s, 0.5, 80.0) + 1e-8)).clamp(min=1e-6)
    X = O.lift(depth, K.double())
    cands, coords, l1s, ssims = [], [], [], []
    for c, T in zip(ctx, mats):
        gr = O.project_to_grid(X, K.double(), T.double())
        coords.append(((gr[..., 0] + 1) / 2 * (W - 1), (gr[..., 1] + 1) / 2 * (H - 1)))
        w = O.synthesize(c.double(), depth, K.double(), K.double(), T.double())
        l1s.append((w - img).abs())
        ssims.append(O.ssim_map(w, img))
        cands.append(O.photometric_map(w, img, 0.85, 1e-4, 9e-4))
        cands.append(O.photometric_map(c.double(), img, 0.85, 1e-4, 9e-4))
    allc = torch.cat(cands, 1)
    for (b, _, y, x) in idx[:12]:
        v = allc[b, :, y, x]
        srt = v.sort()[0]
        near = allc[b, :, max(y - 2, 0):y + 3, max(x - 2, 0):x + 3]
        nsrt = near.sort(0)[0]
        min_margin_nb = float((nsrt[1] - nsrt[0]).min())
        print(f"  px b{b} y{y} x{x}: got {float(got[b,0,y,x]):+.4e} ref {float(ref[b,0,y,x]):+.4e} "
              f"fp64 {float(s64[i].grad[b,0,y,x]):+.4e} "
              f"err/lim {float((got[b,0,y,x]-ref[b,0,y,x]).abs()/lim):.1f}  cands {[round(float(t), 6) for t in v]} "
              f"margin {float(srt[1]-srt[0]):.2e} min margin 5x5 {min_margin_nb:.2e}  "
              f"frac(ix) {[round(float(cx[b,y,x] - cx[b,y,x].round()), 7) for cx, _ in coords]} "
              f"frac(iy) {[round(float(cy[b,y,x] - cy[b,y,x].round()), 7) for _, cy in coords]} "
              f"min|w-I| {[float(l[b,:,y,x].min()) for l in l1s]} ssim {[[round(float(t), 5) for t in s_[b,:,y,x]] for s_ in ssims]}",
              flush=True)
