"""GPU parity of the HIP photometric path against the reference's golden fixtures and the CPU
oracle — every case runs through BOTH gradient paths: K12 (forward + eager backward in one sweep,
psfm_photometric_fwd_grad, the training default) and K1 forward / K2+K3 backward.

Tolerances (BASELINE.json north_star: 1e-4 rel fp32):
  * loss / metrics: 1e-4 relative;
  * dL/dsig: every pixel within 1e-3 * max|g|, except pixels that oracle.sensitive_pixels flags
    (bilinear kinks: a sampling coordinate within 1e-5 px of an integer, where grid_sample's
    derivative jumps; min-reprojection near-ties within 5e-5 and their SSIM window).  There two
    fp32 implementations legitimately differ — ATen-GPU vs ATen-CPU shows the same effect
    (tools/debug_grads.py).  The exclusion is bounded (golden_util.grad_check_bounded): a flagged
    pixel must match, within 1e-3 * max, the oracle or the oracle with the other legitimate
    outcome at the flagged places (the other min selection at near-ties, the other bilinear cell
    at kinks, or both: golden_util.oracle_alternatives), or else stay within 5e-2 * max; at most
    5 % of the pixels may be flagged; the counts are printed;
  * dL/dpose: every entry within 1e-3 * max|g| of the float64 oracle plus twice the flagged
    pixels' own contribution to that entry (golden_util.pose_check_bounded: the oracle re-run in
    float64 with the flagged pixels' warp gradients dropped gives that contribution), or plus the
    largest move of that entry among the oracle's own alternatives where that is more (a net
    contribution can cancel on an entry one flip moves); inputs with no flagged pixel get no slack
    at all (test_kink_free_*).  The worst error / allowance ratio is printed.
"""
import numpy as np
import pytest
import torch

import golden_util as gu

pytestmark = pytest.mark.gpu

LOSS_TOL, GRAD_TOL = 1e-4, 1e-3
CASES = ["default", "mindepth0", "no_automask", "reduce_mean", "rand_mask", "clip", "l1_only",
         "multires", "one_ctx", "wide_motion", "progressive_p03", "progressive_p06"]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import __graft_entry__
    __graft_entry__.build()
    return torch.device("cuda:0")


@pytest.fixture(params=["k12", "k1k2"], autouse=True)
def grad_path(request):
    from packnet_sfm_amd.losses import _hip_photometric as HP
    old = HP.FUSED_GRAD
    HP.FUSED_GRAD = request.param == "k12"
    yield request.param
    HP.FUSED_GRAD = old


def _T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _kw(z):
    return {k: eval(v) for k, v in zip(z["kwargs_keys"], z["kwargs_vals"])}


def run_hip_case(z, dev, mask_none=False):
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    kw = _kw(z)
    nctx = sum(1 for k in z if k.startswith("ctx"))
    S = kw["num_scales"]
    sigs = [_T(z[f"sig{i}"], dev).requires_grad_(True) for i in range(S)]
    vec = _T(z["vec"], dev).requires_grad_(True)
    loss_fn = MultiViewPhotometricLoss(**kw)
    out = loss_fn(_T(z["image"], dev), [_T(z[f"ctx{j}"], dev) for j in range(nctx)], sigs,
                  _T(z["K"], dev), _T(z["K"], dev), [Pose.from_vec(vec[:, j], "euler") for j in range(nctx)],
                  mask=None if mask_none else _T(z["mask"], dev), progress=float(z.get("progress", 0.0)))
    out["loss"].sum().backward()
    torch.cuda.synchronize()
    return out, sigs, vec


def _sensitive(z):
    """(sensitive maps, oracle dL/dsig alternatives, (fp64 oracle dL/dpose, flagged-pixel pose
    bound)) — or (None, None, None) for a multi-resolution case (checked without exclusions)."""
    from oracle import photometric_oracle as O
    kw = _kw(z)
    nctx = sum(1 for k in z if k.startswith("ctx"))
    T = torch.from_numpy
    sigs = [T(z[f"sig{i}"]) for i in range(kw["num_scales"])]
    if any(s.shape[-2:] != sigs[0].shape[-2:] for s in sigs):
        return None, None, None
    mats = [O.pose_vec_to_mat(T(z["vec"])[:, j]) for j in range(nctx)]
    image, ctx = T(z["image"]), [T(z[f"ctx{j}"]) for j in range(nctx)]
    sens, ties = O.sensitive_pixels(image, ctx, sigs, T(z["K"]), mats, kw["min_depth"], kw["max_depth"],
                                    kw["automask_loss"], kw["ssim_loss_weight"], return_ties=True)
    alt, alt_pose, bound = gu.oracle_alternatives(
                                 image, ctx, sigs, T(z["K"]), mats, T(z["mask"]),
                                 ties if kw["photometric_reduce_op"] == "min" else None,
                                 pose_vec=T(z["vec"]), sensitive=sens,
                                 num_scales_=kw["num_scales"], ssim_loss_weight=kw["ssim_loss_weight"],
                                 smooth_loss_weight=kw["smooth_loss_weight"], C1=kw["C1"], C2=kw["C2"],
                                 photometric_reduce_op=kw["photometric_reduce_op"], clip_loss=kw["clip_loss"],
                                 automask_loss=kw["automask_loss"], min_depth=kw["min_depth"],
                                 max_depth=kw["max_depth"], progressive_scaling=kw["progressive_scaling"],
                                 progress=float(z.get("progress", 0.0)))
    return [m.numpy() for m in sens], alt, (alt_pose[0], bound)


@pytest.mark.parametrize("case", CASES)
def test_loss_and_grads_match_reference_golden(dev, case):
    z = gu.load_golden(f"loss_{case}")
    out, sigs, vec = run_hip_case(z, dev)
    assert gu.rel_err(out["loss"].detach().cpu(), z["loss"]) < LOSS_TOL
    assert gu.rel_err(out["metrics"]["photometric_loss"].cpu(), z["photometric_loss"]) < LOSS_TOL
    assert gu.rel_err(out["metrics"]["smoothness_loss"].cpu(), z["smoothness_loss"]) < LOSS_TOL
    sens, alt, pose_ref = _sensitive(z)
    n_used = int(z.get("n_used", len(sigs)))
    for i, s in enumerate(sigs):
        if i >= n_used:   # ProgressiveScaling dropped this scale: no gradient, as in the reference
            assert s.grad is None and not z[f"grad_sig{i}"].any()
            continue
        ok, st = gu.grad_check_bounded(s.grad.cpu(), z[f"grad_sig{i}"], None if alt is None else alt[i],
                                       None if sens is None else sens[i], GRAD_TOL)
        print(f"{case} dL/dsig{i}: {st}")
        assert ok, f"dL/dsig{i}: {st}"
    if pose_ref is None:   # multi-resolution case: no exclusions, the reference golden at 1e-3
        assert gu.rel_err(vec.grad.cpu(), z["grad_vec"]) < GRAD_TOL
        return
    ok, st = gu.pose_check_bounded(vec.grad.cpu(), *pose_ref, tol=GRAD_TOL)
    print(f"{case} dL/dpose: {st}")
    assert ok, f"dL/dpose: {st}"


def _seeded_inputs(seed, B, H, W, nctx=2):
    g = torch.Generator().manual_seed(seed)
    image = gu.smooth_texture(g, B, 3, H, W)
    ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(nctx)]
    return image, ctx, gu.kitti_K(B, H, W), gu.pose_vecs(g, B, nctx), [gu.sigmoid_maps(g, B, H, W) for _ in range(4)]


# Kink-free seeds (golden_util.KINK_FREE_SEEDS): partial band (H < RB), one / two / three stripes —
# (1, 5, 130) is the only no-slack check of dL/dpose across the wave boundaries of a multi-stripe
# band.  A committed seed that stops being kink-free FAILS (tests/test_oracle_golden.py checks them
# on the CPU too): it is never skipped.
KINK_FREE_SEEDS = gu.KINK_FREE_SEEDS


@pytest.mark.parametrize("B,H,W", sorted(KINK_FREE_SEEDS))
def test_kink_free_inputs_match_oracle_tightly(dev, B, H, W):
    """Seeded inputs with NO kink / near-tie pixel: every gradient entry within 1e-3 of the oracle."""
    from oracle import photometric_oracle as O
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    seed = KINK_FREE_SEEDS[(B, H, W)]
    image, ctx, K, vec, sigs = gu.seeded_inputs(seed, B, H, W)
    mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(2)]
    sens = O.sensitive_pixels(image, ctx, sigs, K, mats, 0.5, 80.0)
    assert not any(bool(m.any()) for m in sens), f"committed seed {seed} is no longer kink-free"
    s_c = [s.clone().requires_grad_(True) for s in sigs]
    v_c = vec.clone().requires_grad_(True)
    ref = O.photometric_loss(image, ctx, s_c, K, K, [O.pose_vec_to_mat(v_c[:, j]) for j in range(2)], None)
    ref[0].sum().backward()
    s_d = [s.to(dev).requires_grad_(True) for s in sigs]
    v_d = vec.to(dev).requires_grad_(True)
    fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                  photometric_reduce_op="min", automask_loss=True, clip_loss=0.0,
                                  min_depth=0.5, max_depth=80.0)
    out = fn(image.to(dev), [c.to(dev) for c in ctx], s_d, K.to(dev), K.to(dev),
             [Pose.from_vec(v_d[:, j], "euler") for j in range(2)])
    out["loss"].sum().backward()
    assert gu.rel_err(out["loss"].detach().cpu(), ref[0].detach()) < LOSS_TOL
    for i in range(4):
        ok, msg = gu.grad_check(s_d[i].grad.cpu(), s_c[i].grad, None, GRAD_TOL)
        assert ok, f"seed {seed} dL/dsig{i}: {msg}"
    assert gu.rel_err(v_d.grad.cpu(), v_c.grad) < GRAD_TOL, f"seed {seed}"


def test_mask_none_equals_ones_mask(dev):
    z = gu.load_golden("loss_default")
    a, _, _ = run_hip_case(z, dev, mask_none=True)
    assert gu.rel_err(a["loss"].detach().cpu(), z["loss"]) < LOSS_TOL


def test_deterministic_bitwise(dev):
    z = gu.load_golden("loss_default")
    a, sa, va = run_hip_case(z, dev)
    b, sb, vb = run_hip_case(z, dev)
    assert torch.equal(a["loss"], b["loss"])
    assert all(torch.equal(x.grad, y.grad) for x, y in zip(sa, sb))
    assert torch.equal(va.grad, vb.grad)


def test_kitti_full_res_golden(dev):
    """B=1, 192x640 (BASELINE config shape): scalars, grad norms and sampled pixels."""
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    z = gu.load_golden("loss_kitti_1img")
    B, H, W = 1, 192, 640
    g = torch.Generator().manual_seed(int(z["seed"]))
    image = gu.smooth_texture(g, B, 3, H, W)
    ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
    K = gu.kitti_K(B, H, W)
    vec = gu.pose_vecs(g, B, 2)
    sigs = [gu.sigmoid_maps(g, B, H, W) for _ in range(4)]
    s_d = [s.to(dev).requires_grad_(True) for s in sigs]
    v_d = vec.to(dev).requires_grad_(True)
    fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                  photometric_reduce_op="min", automask_loss=True, clip_loss=0.0,
                                  min_depth=0.5, max_depth=80.0)
    out = fn(image.to(dev), [c.to(dev) for c in ctx], s_d, K.to(dev), K.to(dev),
             [Pose.from_vec(v_d[:, j], "euler") for j in range(2)], mask=torch.ones(B, 1, H, W, device=dev))
    out["loss"].sum().backward()
    assert gu.rel_err(out["loss"].detach().cpu(), z["loss"]) < LOSS_TOL
    assert gu.rel_err(out["metrics"]["smoothness_loss"].cpu(), z["smoothness_loss"]) < LOSS_TOL
    from oracle import photometric_oracle as O
    mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(2)]
    sens, ties = O.sensitive_pixels(image, ctx, sigs, K, mats, 0.5, 80.0, return_ties=True)
    s_c = [s.clone().requires_grad_(True) for s in sigs]
    ref = O.photometric_loss(image, ctx, s_c, K, K, mats, None)
    ref[0].sum().backward()
    alt, alt_pose, bound = gu.oracle_alternatives(image, ctx, sigs, K, mats, None, ties, pose_vec=vec,
                                                  sensitive=sens)
    # 983k warp evaluations: kinks and near-ties always exist at this size (ATen-GPU vs the CPU
    # golden itself differs by 2.8e-3 on this pose gradient, tools/debug_grads.py); the bound is
    # the flagged pixels' own share
    ok, st = gu.pose_check_bounded(v_d.grad.cpu(), alt_pose[0], bound, tol=GRAD_TOL)
    print(f"kitti dL/dpose: {st}")
    assert ok, f"dL/dpose: {st}"
    idx = torch.from_numpy(z["sample_idx"])
    for i in range(4):
        g_cpu = s_c[i].grad.reshape(-1)
        assert gu.rel_err(g_cpu[idx], z[f"grad_sig{i}_samples"]) < 1e-3   # oracle == reference here
        ok, st = gu.grad_check_bounded(s_d[i].grad.cpu(), s_c[i].grad, alt[i], sens[i], GRAD_TOL)
        print(f"kitti dL/dsig{i}: {st}")
        assert ok, f"dL/dsig{i}: {st}"


def test_view_synthesis_matches_reference(dev):
    from packnet_sfm_amd.geometry.camera import Camera
    from packnet_sfm_amd.geometry.camera_utils import view_synthesis
    from packnet_sfm_amd.geometry.pose import Pose
    z = gu.load_golden("geom_small")
    K = _T(z["K"], dev)
    depth = _T(z["depth"], dev).requires_grad_(True)
    vec = _T(z["vec"], dev).requires_grad_(True)
    warped = view_synthesis(_T(z["ref"], dev), depth, Camera(K=K, Tcw=Pose.from_vec(vec, "euler")), Camera(K=K))
    assert gu.rel_err(warped.detach().cpu(), z["warped"]) < 1e-4
    # gradient against the oracle's autograd
    from oracle import photometric_oracle as O
    d_c = torch.from_numpy(z["depth"]).requires_grad_(True)
    v_c = torch.from_numpy(z["vec"]).requires_grad_(True)
    ref = O.synthesize(torch.from_numpy(z["ref"]), d_c, torch.from_numpy(z["K"]), torch.from_numpy(z["K"]),
                       O.pose_vec_to_mat(v_c))
    wgt = torch.linspace(0.5, 1.5, ref.numel()).reshape(ref.shape)
    (ref * wgt).sum().backward()
    (warped * wgt.to(dev)).sum().backward()
    assert gu.rel_err(depth.grad.cpu(), d_c.grad) < GRAD_TOL
    assert gu.rel_err(vec.grad.cpu(), v_c.grad) < GRAD_TOL


def test_grad_scales_with_upstream_gradient(dev, grad_path):
    """K12 produces the gradient for dL/dloss = 1; the finish pass applies the real dL/dloss
    (one rounding at the end: tight).  K2/K3 fold dL/dloss into every pixel's chain, so there
    the check is the usual gradient tolerance."""
    z = gu.load_golden("loss_default")
    a, sa, va = run_hip_case(z, dev)
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    kw = _kw(z)
    sigs = [_T(z[f"sig{i}"], dev).requires_grad_(True) for i in range(kw["num_scales"])]
    vec = _T(z["vec"], dev).requires_grad_(True)
    out = MultiViewPhotometricLoss(**kw)(_T(z["image"], dev), [_T(z[f"ctx{j}"], dev) for j in range(2)], sigs,
                                         _T(z["K"], dev), _T(z["K"], dev),
                                         [Pose.from_vec(vec[:, j], "euler") for j in range(2)], mask=_T(z["mask"], dev))
    (2.5 * out["loss"]).sum().backward(retain_graph=True)
    def close(a, b):
        if grad_path == "k12":
            return torch.allclose(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max()))
        return gu.grad_check(a.cpu(), b.cpu(), None, GRAD_TOL)[0]
    for x, y in zip(sigs, sa):
        assert close(x.grad, 2.5 * y.grad)
    assert gu.rel_err(vec.grad.cpu(), 2.5 * va.grad.cpu()) < (1e-5 if grad_path == "k12" else GRAD_TOL)
    g1 = [x.grad.clone() for x in sigs]
    out["loss"].sum().backward()   # a second backward through the same graph adds 1x more
    for x, y, g in zip(sigs, sa, g1):
        assert close(x.grad, g + y.grad)


def test_no_grad_forward_matches(dev):
    """Under no_grad the forward-only K1 path runs; same loss as the training path."""
    z = gu.load_golden("loss_default")
    a, _, _ = run_hip_case(z, dev)
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    kw = _kw(z)
    with torch.no_grad():
        out = MultiViewPhotometricLoss(**kw)(
            _T(z["image"], dev), [_T(z[f"ctx{j}"], dev) for j in range(2)],
            [_T(z[f"sig{i}"], dev) for i in range(kw["num_scales"])], _T(z["K"], dev), _T(z["K"], dev),
            [Pose.from_vec(_T(z["vec"], dev)[:, j], "euler") for j in range(2)], mask=_T(z["mask"], dev))
    assert gu.rel_err(out["loss"].cpu(), z["loss"]) < LOSS_TOL
    assert gu.rel_err(out["loss"].cpu(), a["loss"].detach().cpu()) < 1e-5


@pytest.mark.parametrize("B,H,W", [(4, 192, 640), (6, 192, 640), (1, 384, 640), (4, 384, 640)])
def test_benchmarked_shapes_match_oracle(dev, B, H, W):
    """The shapes bench.py runs (BASELINE configs 2/4: B=4 192x640; config 3: B=6 192x640;
    config 5: B=1 x 4 cameras 384x640 -> one image and four): loss, every dL/dsig plane (bounded
    exclusion, golden_util.grad_check_bounded) and dL/dpose against the oracle, with a different
    principal point per image (DDAD cameras differ)."""
    from oracle import photometric_oracle as O
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    torch.set_num_threads(16)
    g = torch.Generator().manual_seed(4000 + B * 7 + H)
    image = gu.smooth_texture(g, B, 3, H, W)
    ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
    K = gu.kitti_K(B, H, W)
    K[:, 0, 2] += torch.linspace(-0.02, 0.02, B) * W
    vec = gu.pose_vecs(g, B, 2)
    sigs = [gu.sigmoid_maps(g, B, H, W) for _ in range(4)]
    mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(2)]
    s_c = [s.clone().requires_grad_(True) for s in sigs]
    v_c = vec.clone().requires_grad_(True)
    ref = O.photometric_loss(image, ctx, s_c, K, K, [O.pose_vec_to_mat(v_c[:, j]) for j in range(2)], None)
    ref[0].sum().backward()
    sens, ties = O.sensitive_pixels(image, ctx, sigs, K, mats, 0.5, 80.0, return_ties=True)
    alt, alt_pose, pose_bound = gu.oracle_alternatives(image, ctx, sigs, K, mats, None, ties, pose_vec=vec,
                                                       sensitive=sens)
    s_d = [s.to(dev).requires_grad_(True) for s in sigs]
    v_d = vec.to(dev).requires_grad_(True)
    fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                  photometric_reduce_op="min", automask_loss=True, clip_loss=0.0,
                                  min_depth=0.5, max_depth=80.0)
    out = fn(image.to(dev), [c.to(dev) for c in ctx], s_d, K.to(dev), K.to(dev),
             [Pose.from_vec(v_d[:, j], "euler") for j in range(2)])
    out["loss"].sum().backward()
    torch.cuda.synchronize()
    assert gu.rel_err(out["loss"].detach().cpu(), ref[0].detach()) < LOSS_TOL
    assert gu.rel_err(out["metrics"]["smoothness_loss"].cpu(), ref[2].detach()) < LOSS_TOL
    for i in range(4):
        ok, st = gu.grad_check_bounded(s_d[i].grad.cpu(), s_c[i].grad, alt[i], sens[i], GRAD_TOL)
        print(f"B={B} {H}x{W} dL/dsig{i}: {st}")
        assert ok, f"dL/dsig{i}: {st}"
    # the pose gradient sums ~10^6 warps, among them the flagged pixels: every entry within
    # 1e-3 * max|g| + 2 x the flagged pixels' own contribution to that entry (float64 oracle with
    # their warp gradients dropped, or the oracle alternatives' spread: golden_util.oracle_alternatives)
    # of the float64 oracle
    ok, st = gu.pose_check_bounded(v_d.grad.cpu(), alt_pose[0], pose_bound, tol=GRAD_TOL)
    print(f"B={B} {H}x{W} dL/dpose: {st}")
    assert ok, f"dL/dpose: {st}"


@pytest.mark.parametrize("B,H,W,clip", [(2, 32, 96, 0.0), (4, 192, 640, 0.0), (1, 64, 128, 0.5)])
def test_nearest_scales_fold_matches_materialized(dev, B, H, W, clip):
    """upsample_output's lazy NearestScales (the training default): the kernels read the depth
    net's stored maps through the 2^k nearest mapping (psfm_params.sig_shift) instead of 4
    materialised full-size copies.  Same values in the same order -> loss, metrics and dL/dpose
    bitwise equal to the materialised path; the stored-size dL/dsig = the block sums of the
    materialised full-size gradient (fp32 sums of 4^k terms in another order: 1e-6 * max|g|).
    Also the forward-only (no_grad, K1) path, bitwise."""
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    from packnet_sfm_amd.utils.image import NearestScales, upsample_nearest
    image, ctx, K, vec, _ = _seeded_inputs(11, B, H, W)
    g = torch.Generator().manual_seed(7)
    stored = [gu.sigmoid_maps(g, B, H >> k, W >> k) for k in range(4)]
    fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                  photometric_reduce_op="min", automask_loss=True, clip_loss=clip,
                                  min_depth=0.5, max_depth=80.0)
    args = (image.to(dev), [c.to(dev) for c in ctx])

    def run(lazy, grad=True):
        st = [c.to(dev).requires_grad_(grad) for c in stored]
        v = vec.to(dev).requires_grad_(grad)
        sig = NearestScales(st, (H, W)) if lazy else [upsample_nearest(s, 1 << k) for k, s in enumerate(st)]
        out = fn(*args, sig, K.to(dev), K.to(dev), [Pose.from_vec(v[:, j], "euler") for j in range(2)])
        if grad:
            out["loss"].sum().backward()
        torch.cuda.synchronize()
        return out, st, v

    a, sa, va = run(True)
    b, sb, vb = run(False)
    assert torch.equal(a["loss"], b["loss"])
    for k in ("photometric_loss", "smoothness_loss"):
        assert torch.equal(a["metrics"][k], b["metrics"][k])
    assert torch.equal(va.grad, vb.grad)
    for k in range(4):
        assert sa[k].grad.shape == stored[k].shape
        tol = 1e-6 * float(sb[k].grad.abs().max())
        err = float((sa[k].grad - sb[k].grad).abs().max())
        assert err <= tol, f"scale {k}: {err} > {tol}"
    with torch.no_grad():
        c, _, _ = run(True, grad=False)
        d, _, _ = run(False, grad=False)
    assert torch.equal(c["loss"], d["loss"])
