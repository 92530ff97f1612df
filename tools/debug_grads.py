"""GPU debug: gradient sensitivity.  Compares HIP grads, CPU-oracle grads and the same oracle
run with ATen on the GPU (control for inherent fp32 near-tie sensitivity of min/argmin)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import golden_util as gu  # noqa: E402
from oracle import photometric_oracle as O  # noqa: E402
import __graft_entry__  # noqa: E402

__graft_entry__.build()
from packnet_sfm_amd.geometry.pose import Pose  # noqa: E402
from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss  # noqa: E402

dev = torch.device("cuda:0")


def oracle(image, ctx, sigs, K, vec, device):
    s = [x.clone().to(device).requires_grad_(True) for x in sigs]
    v = vec.clone().to(device).requires_grad_(True)
    out = O.photometric_loss(image.to(device), [c.to(device) for c in ctx], s, K.to(device), K.to(device),
                             [O.pose_vec_to_mat(v[:, j]) for j in range(len(ctx))], None)
    out[0].sum().backward()
    return out, [x.grad.double().cpu() for x in s], v.grad.double().cpu()


def hip(image, ctx, sigs, K, vec):
    s = [x.clone().to(dev).requires_grad_(True) for x in sigs]
    v = vec.clone().to(dev).requires_grad_(True)
    fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                  photometric_reduce_op="min", automask_loss=True, clip_loss=0.0,
                                  min_depth=0.5, max_depth=80.0)
    out = fn(image.to(dev), [c.to(dev) for c in ctx], s, K.to(dev), K.to(dev),
             [Pose.from_vec(v[:, j], "euler") for j in range(len(ctx))])
    out["loss"].sum().backward()
    return out, [x.grad.double().cpu() for x in s], v.grad.double().cpu()


def report(name, ga, gb, va, vb):
    errs = []
    for i, (a, b) in enumerate(zip(ga, gb)):
        d = (a - b).abs()
        l2 = float((a - b).norm() / b.norm())
        frac = float((d > 1e-3 * b.abs().max()).double().mean())
        errs.append(f"s{i}: maxrel {float(d.max() / b.abs().max()):.2e} l2 {l2:.2e} frac>1e-3 {frac:.2e}")
    print(f"[{name}] " + " | ".join(errs))
    print(f"[{name}] pose maxrel {float((va - vb).abs().max() / vb.abs().max()):.2e} "
          f"l2 {float((va - vb).norm() / vb.norm()):.2e}")


for (B, H, W, seed) in [(2, 24, 80, 0), (1, 192, 640, 2024)]:
    if seed == 0:
        z = gu.load_golden("loss_default")
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
        image, ctx, K, vec = T(z["image"]), [T(z["ctx0"]), T(z["ctx1"])], T(z["K"]), T(z["vec"])
        sigs = [T(z[f"sig{i}"]) for i in range(4)]
    else:
        g = torch.Generator().manual_seed(seed)
        image = gu.smooth_texture(g, B, 3, H, W)
        ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
        K = gu.kitti_K(B, H, W)
        vec = gu.pose_vecs(g, B, 2)
        sigs = [gu.sigmoid_maps(g, B, H, W) for _ in range(4)]
    print(f"=== B={B} {H}x{W}")
    oc, gc, vc = oracle(image, ctx, sigs, K, vec, "cpu")
    og, gg, vg = oracle(image, ctx, sigs, K, vec, dev)
    oh, gh, vh = hip(image, ctx, sigs, K, vec)
    print("loss cpu", float(oc[0]), "aten-gpu", float(og[0]), "hip", float(oh["loss"]))
    report("aten-gpu vs cpu", gg, gc, vg, vc)
    report("hip vs cpu", gh, gc, vh, vc)
    report("hip vs aten-gpu", gh, gg, vh, vg)
    if seed == 0:
        a, b = gh[3], gc[3]
        d = (a - b).abs()
        idx = np.unravel_index(int(d.argmax()), d.shape)
        print("max err s3 at", idx, "hip", float(a[idx]), "cpu", float(b[idx]))
