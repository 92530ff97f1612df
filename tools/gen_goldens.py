#!/usr/bin/env python3
"""Generate golden fixtures for the photometric hot path FROM THE REFERENCE.

Runs only in the build container (the reference is not on the GPU box).
It imports `/root/reference/packnet_sfm` as-is and drives its own functions;
the only harness pieces are the ones SURVEY.md §8(c) records:

  * stub modules for `cv2`, `yacs`, `torchvision`, `termcolor` (imported by the
    reference's utility modules, never called on this path);
  * `warp_ref_image` overridden to build a pinhole `Camera(K).scaled(s)` per
    scale (the fork hard-wires FisheyeCamera and `.to(get_device())`, which
    cannot run on a pinhole K nor on CPU: SURVEY.md §0.3 b-d);
  * `mask` passed explicitly (the fork multiplies by `None` otherwise, §0.3e);
  * `SelfSupModel.forward` called without `masks=` (§0.3a).

Every arithmetic line (Camera, Pose, view_synthesis, SSIM, calc_photometric_loss,
reduce_photometric_loss, calc_smoothness_loss, sigmoid_to_depth_linear, the
networks) is the reference's own code.  Outputs: `tests/golden/*.npz`.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_goldens.py
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))
import golden_util as gu  # noqa: E402

OUT = gu.GOLDEN_DIR


def _install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    mod("cv2")
    yacs = mod("yacs")
    cfgmod = mod("yacs.config", CfgNode=type("CfgNode", (dict,), {}))
    yacs.config = cfgmod
    tv = mod("torchvision")
    tvt = mod("torchvision.transforms")
    tvu = mod("torchvision.utils", save_image=lambda *a, **k: None)
    tv.transforms, tv.utils = tvt, tvu
    mod("termcolor", colored=lambda s, *a, **k: s)


_install_stubs()
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

from packnet_sfm.geometry.camera import Camera  # noqa: E402
from packnet_sfm.geometry.pose import Pose  # noqa: E402
from packnet_sfm.geometry.camera_utils import view_synthesis  # noqa: E402
from packnet_sfm.losses import multiview_photometric_loss as mpl  # noqa: E402
from packnet_sfm.utils.image import match_scales  # noqa: E402
from packnet_sfm.utils.depth import inv2depth, compute_depth_metrics  # noqa: E402
from packnet_sfm.utils.post_process_depth import (  # noqa: E402
    sigmoid_to_depth_linear, sigmoid_to_inv_depth)


class HarnessLoss(mpl.MultiViewPhotometricLoss):
    """Reference loss with the pinhole warp override."""

    def warp_ref_image(self, inv_depths, ref_image, K, ref_K, pose, image_size=None):
        B, _, H, W = ref_image.shape
        cams, ref_cams = [], []
        for i in range(self.n):
            _, _, DH, DW = inv_depths[i].shape
            s = DW / float(W)
            cams.append(Camera(K=K.float()).scaled(s))
            ref_cams.append(Camera(K=ref_K.float(), Tcw=pose).scaled(s))
        depths = [inv2depth(inv_depths[i]) for i in range(self.n)]
        ref_images = match_scales(ref_image, inv_depths, self.n)
        return [view_synthesis(ref_images[i], depths[i], ref_cams[i], cams[i],
                               padding_mode=self.padding_mode) for i in range(self.n)]

    def reduce_photometric_loss(self, photometric_losses):
        # capture per-scale reduced maps for debugging, then defer to reference
        if self.photometric_reduce_op == "min":
            self.captured_min = [torch.cat(l, 1).min(1, True)[0].detach()
                                 for l in photometric_losses[: self.n]]
        return super().reduce_photometric_loss(photometric_losses)


class _FisheyeTgt:
    """Target fisheye camera for the reference's view_synthesis: reconstruct in the camera frame
    (identity pose).  The fork's FisheyeCamera.reconstruct/project(frame='w') apply a Pose to a
    [B,3,N] tensor, which Pose.transform_points rejects: the harness applies the
    reference's own Pose to the 4-D point map instead and calls the reference's frame='c' math."""

    def __init__(self, cam):
        self.cam = cam

    def reconstruct(self, depth, frame="w"):
        return self.cam.reconstruct(depth, frame="c")


class _FisheyeRef:
    def __init__(self, cam, pose):
        self.cam, self.pose = cam, pose

    def project(self, X, frame="w"):
        return self.cam.project(self.pose @ X, frame="c")


class HarnessFisheyeLoss(HarnessLoss):
    """The fork's own fisheye warp_ref_image (:131-195: per-scale centre (c + 0.5) s - 0.5, k / s /
    div unchanged, FisheyeCamera per scale) with the §0.3c / §0.3d workarounds above."""

    def warp_ref_image(self, inv_depths, ref_image, intrinsics, ref_intrinsics, pose, image_size=None):
        from packnet_sfm.geometry.camera import FisheyeCamera
        B, _, H, W = ref_image.shape
        warped = []
        depths = [inv2depth(inv_depths[i]) for i in range(self.n)]
        ref_images = match_scales(ref_image, inv_depths, self.n)
        for i in range(self.n):
            _, _, DH, DW = inv_depths[i].shape
            sw, sh = DW / float(W), DH / float(H)

            def scaled(c):
                return {"k": c["k"].clone(), "s": c["s"].clone(), "div": c["div"].clone(),
                        "ux": (c["ux"].clone() + 0.5) * sw - 0.5, "uy": (c["uy"].clone() + 0.5) * sh - 0.5}
            cam = FisheyeCamera(intrinsics=scaled(intrinsics), image_size=(DH, DW))
            ref_cam = FisheyeCamera(intrinsics=scaled(ref_intrinsics), image_size=(DH, DW))
            warped.append(view_synthesis(ref_images[i], depths[i], _FisheyeRef(ref_cam, pose), _FisheyeTgt(cam),
                                         padding_mode=self.padding_mode))
        return warped


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


# ----------------------------------------------------------------------------------------------------------------------
def gen_geom():
    g = torch.Generator().manual_seed(11)
    B, H, W = 2, 24, 80
    K = gu.kitti_K(B, H, W)
    vec = gu.pose_vecs(g, B, 1)[:, 0]
    depth = 1.0 + 29.0 * torch.rand(B, 1, H, W, generator=g)
    ref = gu.smooth_texture(g, B, 3, H, W)
    pose = Pose.from_vec(vec, "euler")
    cam = Camera(K=K)
    ref_cam = Camera(K=K, Tcw=pose)
    X = cam.reconstruct(depth, frame="w")
    coords = ref_cam.project(X, frame="w")
    warped = view_synthesis(ref, depth, ref_cam, cam, padding_mode="zeros")
    # scaled camera (half resolution)
    Ks = Camera(K=K).scaled(0.5).K
    np.savez_compressed(os.path.join(OUT, "geom_small.npz"),
                        K=np32(K), vec=np32(vec), depth=np32(depth), ref=np32(ref),
                        pose_mat=np32(pose.mat), points=np32(X), coords=np32(coords),
                        warped=np32(warped), K_half=np32(Ks))


def gen_ssim():
    g = torch.Generator().manual_seed(12)
    x = gu.smooth_texture(g, 2, 3, 24, 80)
    y = gu.smooth_texture(g, 2, 3, 24, 80)
    loss = HarnessLoss(num_scales=1, ssim_loss_weight=0.85, photometric_reduce_op="min",
                       automask_loss=True, clip_loss=0.0, C1=1e-4, C2=9e-4)
    ssim = mpl.SSIM(x, y, C1=1e-4, C2=9e-4)
    ssim_c = loss.SSIM(x, y)
    photo = loss.calc_photometric_loss([x], [y], None)[0]
    np.savez_compressed(os.path.join(OUT, "ssim_small.npz"), x=np32(x), y=np32(y),
                        ssim=np32(ssim), ssim_clamped=np32(ssim_c), photo=np32(photo))


# ----------------------------------------------------------------------------------------------------------------------
LOSS_CASES = {
    # name: (loss kwargs, extra)
    "default": dict(kw=dict(), mask="ones"),
    "mindepth0": dict(kw=dict(min_depth=0.0), mask="ones"),
    "no_automask": dict(kw=dict(automask_loss=False), mask="ones"),
    "reduce_mean": dict(kw=dict(automask_loss=False, photometric_reduce_op="mean"), mask="ones"),
    "rand_mask": dict(kw=dict(), mask="rand"),
    "clip": dict(kw=dict(clip_loss=0.5), mask="ones"),
    "l1_only": dict(kw=dict(ssim_loss_weight=0.0), mask="ones"),
    "multires": dict(kw=dict(), mask="ones", multires=True),
    "one_ctx": dict(kw=dict(), mask="ones", nctx=1),
    "wide_motion": dict(kw=dict(), mask="ones", motion=8.0),
    # ProgressiveScaling (loss_base.py:10-49, used at :372): thresholds [0.25, 0.5, 0.75, 1.0] would
    # give n = 3 / 2, but the reference tests them with is_list() (utils/types.py:21-23), which is
    # False for the np.float32 array it builds: n stays num_scales (pinned here, `n_used`)
    "progressive_p03": dict(kw=dict(progressive_scaling=0.25), mask="ones", progress=0.3),
    "progressive_p06": dict(kw=dict(progressive_scaling=0.25), mask="ones", progress=0.6),
}

BASE_KW = dict(num_scales=4, ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001,
               C1=1e-4, C2=9e-4, photometric_reduce_op="min", disp_norm=True, clip_loss=0.0,
               progressive_scaling=0.0, padding_mode="zeros", automask_loss=True,
               min_depth=0.5, max_depth=80.0)


def run_loss_case(name, case, B=2, H=24, W=80, seed=100):
    g = torch.Generator().manual_seed(seed + sum(map(ord, name)))
    kw = {**BASE_KW, **case["kw"]}
    nctx = case.get("nctx", 2)
    S = kw["num_scales"]
    image = gu.smooth_texture(g, B, 3, H, W)
    ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(nctx)]
    K = gu.kitti_K(B, H, W)
    vec = gu.pose_vecs(g, B, nctx)
    vec[:, :, :3] *= case.get("motion", 1.0)
    if case.get("multires"):
        sig = [gu.sigmoid_maps(g, B, H >> i, W >> i) for i in range(S)]
    else:
        sig = [gu.sigmoid_maps(g, B, H, W) for _ in range(S)]
    if case["mask"] == "ones":
        mask = torch.ones(B, 1, H, W)
    else:
        mask = (torch.rand(B, 1, H, W, generator=g) > 0.3).float()

    sig_p = [s.clone().requires_grad_(True) for s in sig]
    vec_p = vec.clone().requires_grad_(True)
    poses = [Pose.from_vec(vec_p[:, j], "euler") for j in range(nctx)]
    loss_fn = HarnessLoss(**kw)
    progress = case.get("progress", 0.0)
    out = loss_fn(image, ctx, sig_p, K, K, poses, progress=progress, mask=mask)
    out["loss"].sum().backward()
    res = dict(image=np32(image), K=np32(K), vec=np32(vec), mask=np32(mask),
               progress=np.float64(progress), n_used=np.int64(loss_fn.n),
               loss=np32(out["loss"]),
               photometric_loss=np32(out["metrics"]["photometric_loss"]),
               smoothness_loss=np32(out["metrics"]["smoothness_loss"]),
               grad_vec=np32(vec_p.grad))
    for j in range(nctx):
        res[f"ctx{j}"] = np32(ctx[j])
    for i in range(S):
        res[f"sig{i}"] = np32(sig[i])
        # scales beyond ProgressiveScaling's n get no gradient in the reference (None -> zeros)
        res[f"grad_sig{i}"] = np32(sig_p[i].grad) if sig_p[i].grad is not None else np.zeros_like(np32(sig[i]))
        if hasattr(loss_fn, "captured_min") and i < len(loss_fn.captured_min):
            res[f"min{i}"] = np32(loss_fn.captured_min[i])
    res["kwargs_keys"] = np.array(sorted(kw.keys()))
    res["kwargs_vals"] = np.array([repr(kw[k]) for k in sorted(kw.keys())])
    return res


def gen_losses(only=None):
    for name, case in LOSS_CASES.items():
        if only and name not in only:
            continue
        res = run_loss_case(name, case)
        np.savez_compressed(os.path.join(OUT, f"loss_{name}.npz"), **res)
        print(f"  loss_{name}: loss={float(res['loss'][0]):.6f}")


def gen_kitti_1img():
    """B=1, 192x640: scalars, grad norms and sampled pixels (inputs re-generated from seed)."""
    B, H, W, S = 1, 192, 640, 4
    g = torch.Generator().manual_seed(2024)
    image = gu.smooth_texture(g, B, 3, H, W)
    ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
    K = gu.kitti_K(B, H, W)
    vec = gu.pose_vecs(g, B, 2)
    sig = [gu.sigmoid_maps(g, B, H, W) for _ in range(S)]
    sig_p = [s.clone().requires_grad_(True) for s in sig]
    vec_p = vec.clone().requires_grad_(True)
    poses = [Pose.from_vec(vec_p[:, j], "euler") for j in range(2)]
    loss_fn = HarnessLoss(**BASE_KW)
    out = loss_fn(image, ctx, sig_p, K, K, poses, progress=0.0, mask=torch.ones(B, 1, H, W))
    out["loss"].sum().backward()
    idx = torch.randint(0, H * W, (64,), generator=torch.Generator().manual_seed(7))
    res = dict(seed=np.int64(2024), loss=np32(out["loss"]),
               photometric_loss=np32(out["metrics"]["photometric_loss"]),
               smoothness_loss=np32(out["metrics"]["smoothness_loss"]),
               grad_vec=np32(vec_p.grad), sample_idx=idx.numpy().astype(np.int64))
    for i in range(S):
        gflat = sig_p[i].grad.reshape(-1)
        res[f"grad_sig{i}_norm"] = np.float64(gflat.double().norm())
        res[f"grad_sig{i}_sum"] = np.float64(gflat.double().sum())
        res[f"grad_sig{i}_samples"] = np32(gflat[idx])
        res[f"min{i}_mean"] = np.float64(loss_fn.captured_min[i].double().mean())
        res[f"min{i}_samples"] = np32(loss_fn.captured_min[i].reshape(-1)[idx])
    np.savez_compressed(os.path.join(OUT, "loss_kitti_1img.npz"), **res)
    print(f"  loss_kitti_1img: loss={float(res['loss'][0]):.6f}")


# per-element network-gradient parity: the gradient arriving at the depth net's
# raw inverse-depth outputs and at the pose net's output vector, and the full gradients of a few
# layers (inverse-depth heads, one pack / unpack Conv3d, the PoseNet head) — a test feeds the same
# upstream gradients into the build's nets and compares these layers element by element
FULL_GRAD_PATTERNS = ("disp1_layer.", "disp2_layer.", "disp3_layer.", "disp4_layer.", "pack1.conv3d.",
                      "unpack1.conv3d.", "pose_pred.")


def _retain_net_outputs(model):
    kept = {}
    d_fwd, p_fwd = model.depth_net.forward, model.pose_net.forward

    def depth_fwd(*a, **k):
        o = d_fwd(*a, **k)
        if "inv" not in kept and o["inv_depths"][0].requires_grad:
            # clones: the coarse maps are also used INSIDE the net (upsampled into the next decoder
            # stage); the gradient of the clone is the one arriving from outside (the loss) only
            o = dict(o, inv_depths=[t.clone() for t in o["inv_depths"]])
            for t in o["inv_depths"]:
                t.retain_grad()
            kept["inv"] = o["inv_depths"]
        return o

    def pose_fwd(*a, **k):
        v = p_fwd(*a, **k)
        if "vec" not in kept and v.requires_grad:
            v.retain_grad()
            kept["vec"] = v
        return v
    model.depth_net.forward, model.pose_net.forward = depth_fwd, pose_fwd
    return kept


def _net_grad_fixture(model, kept):
    res = {f"up_inv{i}": np32(t.grad) for i, t in enumerate(kept["inv"])}
    res["up_vec"] = np32(kept["vec"].grad)
    names = []
    for net in ("depth_net", "pose_net"):
        for n, p in getattr(model, net).named_parameters():
            if p.grad is not None and any(k in n for k in FULL_GRAD_PATTERNS):
                assert p.numel() <= 4096, (n, p.shape)
                names.append(f"{net}.{n}")
                res[f"full_grad:{net}.{n}"] = np32(p.grad)
    res["full_grad_names"] = np.array(names)
    return res


def gen_step_packnet():
    """SelfSupModel(PackNet01 '1A' + PoseNet) forward+backward, B=1, 64x192."""
    from packnet_sfm.models.SelfSupModel import SelfSupModel
    from packnet_sfm.networks.depth.PackNet01 import PackNet01
    from packnet_sfm.networks.pose.PoseNet import PoseNet

    B, H, W = 1, 64, 192
    torch.manual_seed(0)
    model = SelfSupModel(**{**BASE_KW, "upsample_depth_maps": True, "rotation_mode": "euler"})
    model.add_depth_net(PackNet01(version="1A"))
    model.add_pose_net(PoseNet(nb_ref_imgs=2))
    model._photometric_loss = HarnessLoss(**BASE_KW)   # pinhole warp override (§8c step 3)
    gu.det_init_(model.depth_net)
    gu.det_init_(model.pose_net)
    model.train()
    g = torch.Generator().manual_seed(77)
    rgb = gu.smooth_texture(g, B, 3, H, W)
    ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
    K = gu.kitti_K(B, H, W)
    batch = dict(rgb=rgb, rgb_context=ctx, rgb_original=rgb, rgb_context_original=ctx,
                 intrinsics=K, distortion_coeffs=K, mask=torch.ones(B, 1, H, W))
    kept = _retain_net_outputs(model)
    out = model(batch, progress=0.0)
    out["loss"].sum().backward()
    names, norms = [], []
    for net in ("depth_net", "pose_net"):
        for n, p in sorted(getattr(model, net).named_parameters()):
            if p.grad is not None and p.dim() >= 2:
                names.append(f"{net}.{n}")
                norms.append(float(p.grad.double().norm()))
    sel = list(range(0, len(names), max(1, len(names) // 16)))[:16]
    inv0 = out["inv_depths"][0]
    res = dict(loss=np32(out["loss"]),
               photometric_loss=np32(out["metrics"]["photometric_loss"]),
               smoothness_loss=np32(out["metrics"]["smoothness_loss"]),
               inv0_sum=np.float64(inv0.double().sum()), inv0_abs=np.float64(inv0.double().abs().sum()),
               inv0_samples=np32(inv0.reshape(-1)[::997]),
               pose_mats=np32(torch.stack([p.mat for p in out["poses"]], 1)),
               grad_names=np.array([names[i] for i in sel]),
               grad_norms=np.array([norms[i] for i in sel], dtype=np.float64),
               **_net_grad_fixture(model, kept))
    np.savez_compressed(os.path.join(OUT, "step_packnet_tiny.npz"), **res)
    print(f"  step_packnet_tiny: loss={float(res['loss'][0]):.6f}")


def gen_step_packnet_san():
    """SelfSupModel(PackNetSAN01 '1A' RGB path + PoseNet) forward+backward, B=1, 64x192 — the depth
    net of BASELINE configs 3 and 5.  Harness stub: `MinkowskiEncoder` (the SAN LiDAR branch, which
    needs the absent MinkowskiEngine and is never called without input_depth) is replaced by a
    parameter-free module.  dropout=None (the YAMLs' 0.5 makes the training forward random)."""
    import torch.nn as nn
    stub = types.ModuleType("packnet_sfm.networks.layers.minkowski_encoder")
    stub.MinkowskiEncoder = lambda *a, **k: nn.Module()
    sys.modules["packnet_sfm.networks.layers.minkowski_encoder"] = stub
    from packnet_sfm.models.SelfSupModel import SelfSupModel
    from packnet_sfm.networks.depth.PackNetSAN01 import PackNetSAN01
    from packnet_sfm.networks.pose.PoseNet import PoseNet

    B, H, W = 1, 64, 192
    torch.manual_seed(0)
    model = SelfSupModel(**{**BASE_KW, "upsample_depth_maps": True, "rotation_mode": "euler"})
    model.add_depth_net(PackNetSAN01(version="1A", dropout=None))
    model.add_pose_net(PoseNet(nb_ref_imgs=2))
    model._photometric_loss = HarnessLoss(**BASE_KW)   # pinhole warp override (§8c step 3)
    gu.det_init_(model.depth_net)
    gu.det_init_(model.pose_net)
    model.train()
    g = torch.Generator().manual_seed(78)
    rgb = gu.smooth_texture(g, B, 3, H, W)
    ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
    K = gu.kitti_K(B, H, W)
    batch = dict(rgb=rgb, rgb_context=ctx, rgb_original=rgb, rgb_context_original=ctx,
                 intrinsics=K, distortion_coeffs=K, mask=torch.ones(B, 1, H, W))
    kept = _retain_net_outputs(model)
    out = model(batch, progress=0.0)
    out["loss"].sum().backward()
    names, norms = [], []
    for net in ("depth_net", "pose_net"):
        for n, p in sorted(getattr(model, net).named_parameters()):
            if p.grad is not None and p.dim() >= 2:
                names.append(f"{net}.{n}")
                norms.append(float(p.grad.double().norm()))
    sel = list(range(0, len(names), max(1, len(names) // 16)))[:16]
    grads_fixture = _net_grad_fixture(model, kept)
    inv = out["inv_depths"]
    model.depth_net.eval()
    with torch.no_grad():
        ev = model.depth_net(rgb)["inv_depths"]
    res = dict(loss=np32(out["loss"]),
               photometric_loss=np32(out["metrics"]["photometric_loss"]),
               smoothness_loss=np32(out["metrics"]["smoothness_loss"]),
               inv_sums=np.array([float(t.double().sum()) for t in inv]),
               inv_shapes=np.array([list(t.shape) for t in inv]),
               inv0_samples=np32(inv[0].reshape(-1)[::997]),
               eval_len=np.int64(len(ev)), eval_inv0_sum=np.float64(ev[0].double().sum()),
               pose_mats=np32(torch.stack([p.mat for p in out["poses"]], 1)),
               param_names=np.array([n for n, _ in model.depth_net.named_parameters()]),
               param_count=np.int64(sum(p.numel() for p in model.depth_net.parameters())),
               grad_names=np.array([names[i] for i in sel]),
               grad_norms=np.array([norms[i] for i in sel], dtype=np.float64), **grads_fixture)
    np.savez_compressed(os.path.join(OUT, "step_packnet_san_tiny.npz"), **res)
    print(f"  step_packnet_san_tiny: loss={float(res['loss'][0]):.6f} params={int(res['param_count'])}")


def gen_fisheye():
    """FisheyeCamera (VADAS) geometry + the photometric loss on fisheye cameras (24x80, B=2)."""
    from packnet_sfm.geometry.camera import FisheyeCamera
    g = torch.Generator().manual_seed(41)
    B, H, W = 2, 24, 80
    intr = gu.vadas_intrinsics(B, H, W)
    vec = gu.pose_vecs(g, B, 1)[:, 0] * 0.5
    depth = 2.0 + 28.0 * torch.rand(B, 1, H, W, generator=g)
    ref = gu.smooth_texture(g, B, 3, H, W)
    pose = Pose.from_vec(vec, "euler")
    cam = FisheyeCamera(intrinsics=intr, image_size=(H, W))
    Xc = cam.reconstruct(depth, frame="c")
    coords = FisheyeCamera(intrinsics=intr, image_size=(H, W)).project(pose @ Xc, frame="c")
    warped = view_synthesis(ref, depth, _FisheyeRef(FisheyeCamera(intrinsics=intr, image_size=(H, W)), pose),
                            _FisheyeTgt(cam), padding_mode="zeros")
    res = dict(vec=np32(vec), depth=np32(depth), ref=np32(ref), points=np32(Xc), coords=np32(coords),
               warped=np32(warped), **{f"intr_{k}": np32(v) for k, v in intr.items()})
    # loss: full-res 4 scales and a multi-resolution case, with gradients
    for tag, multires in (("", False), ("_multires", True)):
        gl = torch.Generator().manual_seed(43 + int(multires))
        image = gu.smooth_texture(gl, B, 3, H, W)
        ctx = [gu.smooth_texture(gl, B, 3, H, W) for _ in range(2)]
        pv = gu.pose_vecs(gl, B, 2) * 0.5
        sig = [gu.sigmoid_maps(gl, B, H >> (i if multires else 0), W >> (i if multires else 0)) for i in range(4)]
        sig_p = [t.clone().requires_grad_(True) for t in sig]
        pv_p = pv.clone().requires_grad_(True)
        fn = HarnessFisheyeLoss(**BASE_KW)
        out = fn(image, ctx, sig_p, intr, intr, [Pose.from_vec(pv_p[:, j], "euler") for j in range(2)],
                 progress=0.0, mask=torch.ones(B, 1, H, W))
        out["loss"].sum().backward()
        res.update({f"image{tag}": np32(image), f"ctx0{tag}": np32(ctx[0]), f"ctx1{tag}": np32(ctx[1]),
                    f"pvec{tag}": np32(pv), f"loss{tag}": np32(out["loss"]),
                    f"photometric_loss{tag}": np32(out["metrics"]["photometric_loss"]),
                    f"smoothness_loss{tag}": np32(out["metrics"]["smoothness_loss"]),
                    f"grad_vec{tag}": np32(pv_p.grad)})
        for i in range(4):
            res[f"sig{i}{tag}"] = np32(sig[i])
            res[f"grad_sig{i}{tag}"] = np32(sig_p[i].grad)
        print(f"  fisheye{tag}: loss={float(out['loss']):.6f}")
    np.savez_compressed(os.path.join(OUT, "fisheye_small.npz"), **res)


def gen_decoders():
    """ResNet-side heads of BASELINE configs 1/2 that the reference can pin without torchvision:
    DepthDecoder (networks/layers/resnet/depth_decoder.py:16-64: 5 up-stages, skips, sigmoid heads)
    and PoseDecoder (pose_decoder.py:13-53) with det_init_ weights, fed seeded encoder features;
    forward outputs and, for a seeded upstream gradient, the input-feature gradients, every bias
    gradient and the full weight gradients of the small layers, plus all gradient norms."""
    from packnet_sfm.networks.layers.resnet.depth_decoder import DepthDecoder
    from packnet_sfm.networks.layers.resnet.layers import disp_to_depth
    from packnet_sfm.networks.layers.resnet.pose_decoder import PoseDecoder
    feats, up_disp, up_pose = gu.decoder_inputs()
    res = {"seed": np.int64(91)}
    dec = DepthDecoder(np.array([64, 64, 128, 256, 512]))
    gu.det_init_(dec)
    f = [t.clone().requires_grad_(True) for t in feats]
    out = dec(f)
    disps = [out[("disp", i)] for i in range(4)]
    sum((d * u).sum() for d, u in zip(disps, up_disp)).backward()
    for i, d in enumerate(disps):
        res[f"disp{i}"] = np32(d)
        sd, dd = disp_to_depth(d.detach(), 0.1, 100.0)
        res[f"scaled_disp{i}"], res[f"depth{i}"] = np32(sd), np32(dd)
    for i, t in enumerate(f):
        res[f"grad_feat{i}"] = np32(t.grad)
    names, norms = [], []
    for n, p in dec.named_parameters():
        names.append(n)
        norms.append(float(p.grad.double().norm()))
        if n.endswith("bias") or p.numel() <= 4096:
            res[f"grad:{n}"] = np32(p.grad)
    res["dec_grad_names"], res["dec_grad_norms"] = np.array(names), np.array(norms, dtype=np.float64)
    pdec = PoseDecoder(np.array([64, 64, 128, 256, 512]), num_input_features=1, num_frames_to_predict_for=2)
    gu.det_init_(pdec)
    last = feats[-1].clone().requires_grad_(True)
    axisangle, translation = pdec([[None, None, None, None, last]])
    pose = torch.cat([axisangle, translation], -1)
    (pose * up_pose).sum().backward()
    res["axisangle"], res["translation"] = np32(axisangle), np32(translation)
    res["grad_pose_feat"] = np32(last.grad)
    names, norms = [], []
    for n, p in pdec.named_parameters():
        names.append(n)
        norms.append(float(p.grad.double().norm()))
        if n.endswith("bias") or p.numel() <= 4096:
            res[f"pgrad:{n}"] = np32(p.grad)
    res["pose_grad_names"], res["pose_grad_norms"] = np.array(names), np.array(norms, dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "decoders_resnet.npz"), **res)
    print(f"  decoders_resnet: disp0 sum={float(disps[0].double().sum()):.6f} "
          f"pose sum={float(pose.double().sum()):.6e}")


def gen_depth_metrics():
    g = torch.Generator().manual_seed(31)
    B, H, W = 2, 192, 640
    gt = 1.0 + 79.0 * torch.rand(B, 1, H, W, generator=g)
    gt[torch.rand(B, 1, H, W, generator=g) < 0.6] = 0.0   # sparse, like velodyne
    pred = gt.clamp(min=1.0) * (1.0 + 0.1 * torch.randn(B, 1, H, W, generator=g)) * 1.3
    pred = pred.clamp(0.5, 90.0)
    cfg = types.SimpleNamespace(min_depth=0.0, max_depth=80.0, crop="garg", scale_output="top-center")
    with_scale = compute_depth_metrics(cfg, gt, pred, use_gt_scale=True)
    no_scale = compute_depth_metrics(cfg, gt, pred, use_gt_scale=False)
    cfg2 = types.SimpleNamespace(min_depth=1e-3, max_depth=80.0, crop="", scale_output="top-center")
    no_crop = compute_depth_metrics(cfg2, gt, pred, use_gt_scale=True)
    # sigmoid conversions (docstring known answers + dense sweep)
    s = torch.linspace(0, 1, 101)
    np.savez_compressed(os.path.join(OUT, "depth_metrics.npz"), seed=np.int64(31),
                        with_scale=np32(with_scale), no_scale=np32(no_scale), no_crop=np32(no_crop),
                        sig=np32(s), depth_lin=np32(sigmoid_to_depth_linear(s, 0.05, 80.0)),
                        inv_lin=np32(sigmoid_to_inv_depth(s, 0.05, 80.0)),
                        depth_lin_05=np32(sigmoid_to_depth_linear(s, 0.5, 80.0)),
                        depth_lin_0=np32(sigmoid_to_depth_linear(s, 0.0, 80.0)))


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    os.makedirs(OUT, exist_ok=True)
    import contextlib
    import io
    which = sys.argv[1:] or ["geom", "ssim", "losses", "kitti", "metrics", "step", "fisheye"]
    for w in which:
        print(f"[gen] {w}")
        if w.startswith("losses:"):   # a subset of the loss cases: losses:name1,name2
            gen_losses(w.split(":", 1)[1].split(","))
            continue
        quiet = io.StringIO()
        with contextlib.redirect_stdout(quiet) if w == "metrics" else contextlib.nullcontext():
            {"geom": gen_geom, "ssim": gen_ssim, "losses": gen_losses, "kitti": gen_kitti_1img,
             "metrics": gen_depth_metrics, "step": gen_step_packnet, "fisheye": gen_fisheye,
             "step_san": gen_step_packnet_san, "decoders": gen_decoders}[w]()
    print("done")
