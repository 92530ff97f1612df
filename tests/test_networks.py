"""Networks (PyTorch-ROCm side of the step): parameter layout and numerics vs the reference.

PackNet01/PoseNet have the reference's parameter names; loading the golden's deterministic
weights (golden_util.det_init_) must reproduce the reference's inverse-depth outputs and, with
the oracle loss, the reference's SelfSupModel loss (tests/golden/step_packnet_tiny.npz).
ResNet encoders follow torchvision's layout (torchvision is absent here: parity unpinned for
the trunk, which is the standard architecture)."""
import numpy as np
import pytest
import torch

import golden_util as gu


def _batch(B=1, H=64, W=192):
    g = torch.Generator().manual_seed(77)
    rgb = gu.smooth_texture(g, B, 3, H, W)
    ctx = [gu.smooth_texture(g, B, 3, H, W) for _ in range(2)]
    return rgb, ctx, gu.kitti_K(B, H, W)


def _packnet_model():
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.networks.depth.PackNet01 import PackNet01
    from packnet_sfm_amd.networks.pose.PoseNet import PoseNet
    depth, pose = PackNet01(version="1A"), PoseNet(nb_ref_imgs=2)
    gu.det_init_(depth)
    gu.det_init_(pose)
    return depth, pose


def test_packnet_parameter_count_matches_survey():
    depth, pose = _packnet_model()
    n_depth = sum(p.numel() for p in depth.parameters())
    n_pose = sum(p.numel() for p in pose.parameters())
    assert abs(n_depth / 1e6 - 128.29) < 0.01
    assert abs(n_pose / 1e6 - 1.59) < 0.01


def test_resnet_san_parameter_layout():
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.networks.depth.ResNetSAN01 import ResNetSAN01
    net = ResNetSAN01(version="18A")
    names = dict(net.named_parameters())
    assert "encoder.encoder.layer4.1.bn2.weight" in names
    assert "decoder.decoder.0.conv.conv.weight" in names
    n = sum(p.numel() for p in net.parameters())
    assert abs(n / 1e6 - 14.33) < 0.02            # SURVEY.md §2.4 (ResNet18 depth)


def test_packnet_step_matches_reference_cpu():
    """PackNet01 + PoseNet forward (ours, CPU) + oracle loss == the reference SelfSupModel step."""
    from oracle import photometric_oracle as O
    z = gu.load_golden("step_packnet_tiny")
    depth, pose = _packnet_model()
    depth.train()
    pose.train()
    rgb, ctx, K = _batch()
    torch.set_num_threads(8)
    inv = depth(rgb)["inv_depths"]
    inv_up = [torch.nn.functional.interpolate(i, size=rgb.shape[-2:], mode="nearest") for i in inv]
    assert abs(float(inv_up[0].double().sum()) - float(z["inv0_sum"])) / float(z["inv0_sum"]) < 1e-4
    np.testing.assert_allclose(inv_up[0].reshape(-1)[::997].detach().numpy(), z["inv0_samples"], rtol=1e-4)
    vec = pose(rgb, ctx)
    mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(2)]
    np.testing.assert_allclose(torch.stack(mats, 1).detach().numpy(), z["pose_mats"], rtol=1e-4, atol=1e-6)
    loss, photo, smooth, _ = O.photometric_loss(rgb, ctx, inv_up, K, K, mats, torch.ones(1, 1, 64, 192))
    assert gu.rel_err(loss.detach(), z["loss"]) < 1e-4
    assert gu.rel_err(smooth.detach(), z["smoothness_loss"]) < 1e-4


@pytest.mark.gpu
def test_selfsup_step_on_gpu_matches_reference():
    """Full SelfSupModel step on the GPU (MIOpen nets + HIP loss) vs the reference golden."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.models.SelfSupModel import SelfSupModel
    z = gu.load_golden("step_packnet_tiny")
    dev = torch.device("cuda:0")
    depth, pose = _packnet_model()
    model = SelfSupModel(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001, photometric_reduce_op="min",
                         automask_loss=True, clip_loss=0.0, min_depth=0.5, max_depth=80.0,
                         upsample_depth_maps=True, rotation_mode="euler")
    model.add_depth_net(depth)
    model.add_pose_net(pose)
    model = model.to(dev).train()
    rgb, ctx, K = _batch()
    rgb, ctx, K = rgb.to(dev), [c.to(dev) for c in ctx], K.to(dev)
    batch = dict(rgb=rgb, rgb_context=ctx, rgb_original=rgb, rgb_context_original=ctx, intrinsics=K,
                 mask=torch.ones(1, 1, 64, 192, device=dev))
    out = model(batch, progress=0.0)
    out["loss"].sum().backward()
    assert gu.rel_err(out["loss"].detach().cpu(), z["loss"]) < 1e-4
    assert gu.rel_err(out["metrics"]["smoothness_loss"].cpu(), z["smoothness_loss"]) < 1e-4
    params = {f"depth_net.{n}": p for n, p in model.depth_net.named_parameters()}
    params.update({f"pose_net.{n}": p for n, p in model.pose_net.named_parameters()})
    for name, ref in zip(z["grad_names"], z["grad_norms"]):
        got = float(params[str(name)].grad.double().norm())
        assert abs(got - ref) / ref < 2e-2, (name, got, ref)


def _packnet_san_model():
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.networks.depth.PackNetSAN01 import PackNetSAN01
    from packnet_sfm_amd.networks.pose.PoseNet import PoseNet
    depth, pose = PackNetSAN01(version="1A", dropout=None), PoseNet(nb_ref_imgs=2)
    gu.det_init_(depth)
    gu.det_init_(pose)
    return depth, pose


def test_packnet_san_parameters_match_reference():
    """PackNetSAN01 RGB path: the reference's parameter names (checkpoint keys, minus the absent
    MinkowskiEncoder) and count (BASELINE configs 3 / 5)."""
    z = gu.load_golden("step_packnet_san_tiny")
    depth, _ = _packnet_san_model()
    assert [n for n, _ in depth.named_parameters()] == [str(n) for n in z["param_names"]]
    assert sum(p.numel() for p in depth.parameters()) == int(z["param_count"])


def test_packnet_san_step_matches_reference_cpu():
    """PackNetSAN01 + PoseNet forward (ours, CPU: the reference op chain) + oracle loss == the
    reference SelfSupModel step (tests/golden/step_packnet_san_tiny.npz)."""
    from oracle import photometric_oracle as O
    z = gu.load_golden("step_packnet_san_tiny")
    depth, pose = _packnet_san_model()
    depth.train()
    pose.train()
    g = torch.Generator().manual_seed(78)
    rgb = gu.smooth_texture(g, 1, 3, 64, 192)
    ctx = [gu.smooth_texture(g, 1, 3, 64, 192) for _ in range(2)]
    K = gu.kitti_K(1, 64, 192)
    torch.set_num_threads(8)
    inv = depth(rgb)["inv_depths"]
    assert [list(t.shape) for t in inv] == [[1, 1, 64 >> i, 192 >> i] for i in range(4)]
    inv_up = [torch.nn.functional.interpolate(i, size=(64, 192), mode="nearest") for i in inv]
    assert [list(t.shape) for t in inv_up] == z["inv_shapes"].tolist()   # SfmModel.upsample_output
    for t, ref in zip(inv_up, z["inv_sums"]):
        assert abs(float(t.double().sum()) - ref) / abs(ref) < 1e-4
    np.testing.assert_allclose(inv_up[0].reshape(-1)[::997].detach().numpy(), z["inv0_samples"], rtol=1e-4)
    vec = pose(rgb, ctx)
    mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(2)]
    np.testing.assert_allclose(torch.stack(mats, 1).detach().numpy(), z["pose_mats"], rtol=1e-4, atol=1e-6)
    loss, photo, smooth, _ = O.photometric_loss(rgb, ctx, inv_up, K, K, mats, torch.ones(1, 1, 64, 192))
    assert gu.rel_err(loss.detach(), z["loss"]) < 1e-4
    assert gu.rel_err(smooth.detach(), z["smoothness_loss"]) < 1e-4
    depth.eval()
    with torch.no_grad():
        ev = depth(rgb)["inv_depths"]
    assert len(ev) == int(z["eval_len"]) == 1
    assert abs(float(ev[0].double().sum()) - float(z["eval_inv0_sum"])) / abs(float(z["eval_inv0_sum"])) < 1e-4


@pytest.mark.gpu
def test_selfsup_packnet_san_step_on_gpu_matches_reference():
    """PackNetSAN01 (fused d=4 pack / unpack kernels) + PoseNet + HIP loss on the GPU vs the
    reference golden: loss, smoothness, and 16 parameter-gradient norms."""
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.models.SelfSupModel import SelfSupModel
    z = gu.load_golden("step_packnet_san_tiny")
    dev = torch.device("cuda:0")
    depth, pose = _packnet_san_model()
    model = SelfSupModel(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001, photometric_reduce_op="min",
                         automask_loss=True, clip_loss=0.0, min_depth=0.5, max_depth=80.0,
                         upsample_depth_maps=True, rotation_mode="euler")
    model.add_depth_net(depth)
    model.add_pose_net(pose)
    model = model.to(dev).train()
    g = torch.Generator().manual_seed(78)
    rgb = gu.smooth_texture(g, 1, 3, 64, 192).to(dev)
    ctx = [gu.smooth_texture(g, 1, 3, 64, 192).to(dev) for _ in range(2)]
    K = gu.kitti_K(1, 64, 192).to(dev)
    batch = dict(rgb=rgb, rgb_context=ctx, rgb_original=rgb, rgb_context_original=ctx, intrinsics=K,
                 mask=torch.ones(1, 1, 64, 192, device=dev))
    out = model(batch, progress=0.0)
    out["loss"].sum().backward()
    assert gu.rel_err(out["loss"].detach().cpu(), z["loss"]) < 1e-4
    assert gu.rel_err(out["metrics"]["smoothness_loss"].cpu(), z["smoothness_loss"]) < 1e-4
    params = {f"depth_net.{n}": p for n, p in model.depth_net.named_parameters()}
    params.update({f"pose_net.{n}": p for n, p in model.pose_net.named_parameters()})
    for name, ref in zip(z["grad_names"], z["grad_norms"]):
        got = float(params[str(name)].grad.double().norm())
        assert abs(got - ref) / ref < 2e-2, (name, got, ref)


@pytest.mark.parametrize("f,cl", [(2, False), (2, True), (4, True), (8, False)])
def test_upsample_nearest_equals_interpolate(f, cl):
    """utils.image.upsample_nearest (deterministic block-sum backward) == F.interpolate nearest,
    forward and backward, any memory format."""
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.utils.image import upsample_nearest, interpolate_scales
    g = torch.Generator().manual_seed(f)
    x = torch.randn(2, 3, 5, 7, generator=g, dtype=torch.float64)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    a, b = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya = upsample_nearest(a, f)
    yb = torch.nn.functional.interpolate(b, scale_factor=f, mode="nearest")
    assert torch.equal(ya, yb)
    gy = torch.randn(ya.shape, generator=g, dtype=torch.float64)
    ya.backward(gy)
    yb.backward(gy)
    torch.testing.assert_close(a.grad, b.grad, rtol=1e-12, atol=1e-12)
    ups = interpolate_scales([x, x[..., :3, :4]], shape=(5 * f, 7 * f), mode="nearest", align_corners=None)
    assert torch.equal(ups[0], yb)    # exact multiple -> the deterministic op
    assert ups[1].shape[-2:] == (5 * f, 7 * f)   # not a multiple -> F.interpolate


@pytest.mark.gpu
def test_config1_depthresnet_poseresnet_step_on_gpu_matches_cpu_oracle():
    """BASELINE config 1 (configs/overfit_kitti.yaml): SelfSupModel(DepthResNet 18pt + PoseResNet
    18pt), fp32, B=6, 192x640, min_depth 0 / max_depth 80.  The GPU step (MIOpen nets + HIP loss
    through the lazy upsample fold) vs the same weights on CPU with the oracle loss: loss 1e-4
    relative, every parameter-gradient norm 2e-2 (fp32 MIOpen vs CPU convolutions re-round the
    activations, which moves min-reprojection near-ties / bilinear kinks of the photometric
    gradient — the same tolerance as the reference-golden step tests)."""
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import __graft_entry__
    __graft_entry__.build()
    from oracle import photometric_oracle as O
    from packnet_sfm_amd.models.SelfSupModel import SelfSupModel
    from packnet_sfm_amd.networks.depth.DepthResNet import DepthResNet
    from packnet_sfm_amd.networks.pose.PoseResNet import PoseResNet
    torch.manual_seed(3)
    kw = dict(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001, photometric_reduce_op="min",
              automask_loss=True, clip_loss=0.0, min_depth=0.0, max_depth=80.0)
    model = SelfSupModel(**kw, upsample_depth_maps=True, rotation_mode="euler")
    model.add_depth_net(DepthResNet(version="18pt"))
    model.add_pose_net(PoseResNet(version="18pt"))
    model.train()
    B, H, W = 6, 192, 640
    rgb, ctx, K = _batch(B, H, W)
    # CPU: the same nets, upsample_output materialised, oracle loss (tests-only checker)
    inv = model.depth_net(rgb)["inv_depths"]
    inv = [torch.nn.functional.interpolate(i, size=(H, W), mode="nearest") for i in inv]
    vec = model.pose_net(rgb, ctx)
    ref = O.photometric_loss(rgb, ctx, inv, K, K, [O.pose_vec_to_mat(vec[:, j]) for j in range(2)], None,
                             num_scales_=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                             photometric_reduce_op="min", automask_loss=True, clip_loss=0.0,
                             min_depth=0.0, max_depth=80.0)[0]
    ref.sum().backward()
    ref_norms = {n: float(p.grad.double().norm()) for n, p in model.named_parameters() if p.grad is not None}
    model.zero_grad(set_to_none=True)
    dev = torch.device("cuda:0")
    model = model.to(dev)
    batch = dict(rgb=rgb.to(dev), rgb_context=[c.to(dev) for c in ctx], rgb_original=rgb.to(dev),
                 rgb_context_original=[c.to(dev) for c in ctx], intrinsics=K.to(dev))
    out = model(batch, progress=0.0)
    out["loss"].sum().backward()
    assert gu.rel_err(out["loss"].detach().cpu(), ref.detach()) < 1e-4
    got = {n: float(p.grad.double().norm()) for n, p in model.named_parameters() if p.grad is not None}
    assert set(got) == set(ref_norms)
    bad = {n: (got[n], r) for n, r in ref_norms.items() if abs(got[n] - r) > 2e-2 * r + 1e-12}
    assert not bad, bad


@pytest.mark.gpu
def test_ddad_packnet_san_four_camera_step_matches_oracle_on_its_outputs():
    """BASELINE config 5 per GPU (configs/train_packnet_san_ddad.yaml): one DDAD sample of 4
    cameras at 384x640 (5-D batch, folded into the batch by flatten_cameras == stack_batch,
    model_utils.py:68-94), PackNetSAN01 (d = 4 pack / unpack kernels) + PoseNet under bf16
    autocast, HIP loss.  The loss and both metrics equal the oracle evaluated on the step's own
    network outputs (sigmoid maps upsampled to full resolution, pose matrices, per-camera
    intrinsics) within 1e-4; the backward through both nets runs and leaves finite gradients
    in every parameter."""
    import __graft_entry__
    __graft_entry__.build()
    import bench
    from oracle import photometric_oracle as O
    from packnet_sfm_amd.datasets.synthetic import SyntheticSfmDataset
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = False
    args = bench.parse(["--config", "ddad-packnet-san"])
    torch.manual_seed(0)
    model = bench.to_channels_last(bench.build_model(args, dev))
    s = SyntheticSfmDataset(1, 384, 640, 2, cameras=4, seed=5)[0]
    assert s["rgb"].shape == (4, 3, 384, 640)
    batch = {"rgb": s["rgb"][None].to(dev), "rgb_context": [c[None].to(dev) for c in s["rgb_context"]],
             "intrinsics": s["intrinsics"][None].to(dev)}
    batch["rgb_original"], batch["rgb_context_original"] = batch["rgb"], batch["rgb_context"]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = model(batch, progress=0.0)
    out["loss"].sum().backward()
    torch.cuda.synchronize()
    inv = [out["inv_depths"][i].detach().float().cpu() for i in range(4)]
    assert all(tuple(t.shape) == (4, 1, 384, 640) for t in inv)
    mats = [p.mat.detach().float().cpu() for p in out["poses"]]
    rgb, ctx, K = s["rgb"], list(s["rgb_context"]), s["intrinsics"]
    torch.set_num_threads(16)
    ref = O.photometric_loss(rgb, ctx, inv, K, K, mats, None, num_scales_=4, ssim_loss_weight=0.85,
                             smooth_loss_weight=0.001, photometric_reduce_op="min", automask_loss=True,
                             clip_loss=0.0, min_depth=0.5, max_depth=200.0)
    print(f"4-camera 384x640 loss: HIP {float(out['loss']):.8f}, oracle {float(ref[0]):.8f}")
    assert gu.rel_err(out["loss"].detach().cpu(), ref[0].detach()) < 1e-4
    assert gu.rel_err(out["metrics"]["smoothness_loss"].cpu(), ref[2].detach()) < 1e-4
    assert gu.rel_err(out["metrics"]["photometric_loss"].cpu(), ref[0].detach()) < 1e-4   # the fork's alias
    # the LiDAR fusion weights of PackNetSAN01 (depth_net.weight / .bias) are unused on the RGB path
    missing = [n for n, p in model.named_parameters() if p.requires_grad and p.grad is None]
    assert missing == ["depth_net.weight", "depth_net.bias"], missing[:5]
    bad = [n for n, p in model.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
    assert not bad, bad[:5]


# -------------------------------------------------------------------------------------------------
# per-element network-gradient parity: the golden's own upstream gradients
# (dL/d inverse-depth outputs, dL/d pose vector: no min-reprojection flip can enter) fed into the
# build's nets; every element of the pinned layers' gradients (inverse-depth heads, the first pack /
# unpack Conv3d — the HIP pack3d kernels on the GPU — and the PoseNet head) vs the reference
def _net_grads_vs_golden(depth, pose, z, dev, seed, tol):
    g = torch.Generator().manual_seed(seed)
    rgb = gu.smooth_texture(g, 1, 3, 64, 192).to(dev)
    ctx = [gu.smooth_texture(g, 1, 3, 64, 192).to(dev) for _ in range(2)]
    depth, pose = depth.to(dev).train(), pose.to(dev).train()
    inv = depth(rgb)["inv_depths"]
    vec = pose(rgb, ctx)
    up = [torch.from_numpy(z[f"up_inv{i}"]).to(dev) for i in range(len(inv))]
    assert [tuple(a.shape) for a in inv] == [tuple(u.shape) for u in up]
    (sum((a * u).sum() for a, u in zip(inv, up)) + (vec * torch.from_numpy(z["up_vec"]).to(dev)).sum()).backward()
    params = {f"depth_net.{n}": p for n, p in depth.named_parameters()}
    params.update({f"pose_net.{n}": p for n, p in pose.named_parameters()})
    names = [str(n) for n in z["full_grad_names"]]
    assert any("conv3d" in n for n in names) and any("pose_pred" in n for n in names)
    errs = {}
    for n in names:
        errs[n] = gu.rel_err(params[n].grad.detach().cpu(), z[f"full_grad:{n}"])
    print("per-element gradient error / max:", {k: f"{v:.1e}" for k, v in errs.items()})
    bad = {k: v for k, v in errs.items() if v > tol}
    assert not bad, bad


def test_packnet_layer_gradients_match_reference_cpu():
    depth, pose = _packnet_model()
    torch.set_num_threads(8)
    _net_grads_vs_golden(depth, pose, gu.load_golden("step_packnet_tiny"), torch.device("cpu"), 77, 1e-4)


def test_packnet_san_layer_gradients_match_reference_cpu():
    depth, pose = _packnet_san_model()
    torch.set_num_threads(8)
    _net_grads_vs_golden(depth, pose, gu.load_golden("step_packnet_san_tiny"), torch.device("cpu"), 78, 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["packnet", "packnet_san"])
def test_packnet_layer_gradients_match_reference_gpu_fp32(which):
    """fp32 on the GPU: MIOpen convolutions + the HIP pack / unpack Conv3d kernels, 1e-3 * max per
    element of every pinned layer gradient."""
    import __graft_entry__
    __graft_entry__.build()
    torch.backends.cudnn.benchmark = False
    depth, pose = _packnet_model() if which == "packnet" else _packnet_san_model()
    z = gu.load_golden("step_packnet_tiny" if which == "packnet" else "step_packnet_san_tiny")
    _net_grads_vs_golden(depth, pose, z, torch.device("cuda:0"), 77 if which == "packnet" else 78, 1e-3)
