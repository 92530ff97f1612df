"""GPU parity of the pose / camera-record kernels (include/psfm_pose.h) against the reference's
golden `Pose.from_vec` (tests/golden/geom_small.npz, tools/gen_goldens.py) and the CPU oracle.

Tolerances (fp32 kernels vs float64 oracle):
  * matrices: 2e-6 absolute (sin / cos + one two-term sum per entry, |entries| <= 1 + |t|);
  * dL/dvec: 2e-5 relative to the largest component (a few fp32 roundings per term);
  * camera records: bit-identical to the same fp32 ATen ops on the device (IEEE division both).
"""
import numpy as np
import pytest
import torch

import golden_util as gu
from oracle import photometric_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import __graft_entry__
    __graft_entry__.build()
    return torch.device("cuda", 0)


def test_from_vec_matches_reference_golden(dev):
    from packnet_sfm_amd.geometry.pose import Pose
    z = gu.load_golden("geom_small")
    m = Pose.from_vec(torch.from_numpy(z["vec"]).to(dev), "euler").mat
    np.testing.assert_allclose(m.cpu().numpy(), z["pose_mat"], rtol=0, atol=2e-6)


@pytest.mark.parametrize("B,N", [(1, 1), (4, 2), (5, 3), (3, 8)])
def test_from_vecs_fwd_bwd_match_oracle(dev, B, N):
    from packnet_sfm_amd.geometry.pose import Pose
    g = torch.Generator().manual_seed(100 + 10 * B + N)
    vec = torch.randn(B, N, 6, generator=g)
    vec[..., 3:] = (torch.rand(B, N, 3, generator=g) * 2 - 1) * 3.1   # full angle range
    up = [torch.randn(B, 4, 4, generator=g) for _ in range(N)]
    vd = vec.to(dev).requires_grad_(True)
    poses = Pose.from_vecs(vd, "euler")
    sum(((p.mat * u.to(dev)).sum() for p, u in zip(poses, up))).backward()
    vr = vec.double().requires_grad_(True)
    ref = [O.pose_vec_to_mat(vr[:, j]) for j in range(N)]
    sum(((r * u.double()).sum() for r, u in zip(ref, up))).backward()
    for p, r in zip(poses, ref):
        np.testing.assert_allclose(p.mat.detach().cpu().double().numpy(), r.detach().numpy(), rtol=0, atol=2e-6)
    gv, gr = vd.grad.cpu().double(), vr.grad
    assert (gv - gr).abs().max().item() <= 2e-5 * gr.abs().max().item()


def test_unused_context_gets_zero_grad(dev):
    from packnet_sfm_amd.geometry.pose import Pose
    vd = torch.randn(3, 2, 6, device=dev).requires_grad_(True)
    p0, p1 = Pose.from_vecs(vd, "euler")
    (p1.mat * 2.0).sum().backward()
    assert torch.all(vd.grad[:, 0] == 0)
    assert torch.any(vd.grad[:, 1] != 0)


def test_from_vec_single_equals_batched(dev):
    from packnet_sfm_amd.geometry.pose import Pose
    vd = torch.randn(4, 2, 6, device=dev)
    both = Pose.from_vecs(vd, "euler")
    for j in range(2):
        assert torch.equal(Pose.from_vec(vd[:, j], "euler").mat, both[j].mat)


@pytest.mark.parametrize("scale", [1.0, 0.5, 0.25])
@pytest.mark.parametrize("t_rows", [3, 4])
def test_pinhole_cam_records_bitwise(dev, scale, t_rows):
    from packnet_sfm_amd import _hip
    B, N, S = 3, 2, 2
    K = gu.kitti_K(B, 192, 640).to(dev)
    refK = gu.kitti_K(B, 192, 640).to(dev) * 1.01
    T = torch.randn(N, B, t_rows, 4, device=dev)
    cam = torch.empty(S, N, B, _hip.CAMREC, device=dev)
    _hip.check(_hip.lib().psfm_pinhole_cam_records(_hip.ptr(K), _hip.ptr(refK), _hip.ptr(T), 4 * t_rows, B, N, S,
                                                   scale, _hip.ptr(cam), _hip.stream(dev)), "psfm_pinhole_cam_records")
    # the same fp32 ATen ops the loss used before (camera_utils.scale_intrinsics + pinhole_inverse)
    from packnet_sfm_amd.geometry.camera_utils import pinhole_inverse, scale_intrinsics
    Kt = scale_intrinsics(K.clone(), scale, scale) if scale != 1.0 else K
    Kr = scale_intrinsics(refK.clone(), scale, scale) if scale != 1.0 else refK
    want = torch.cat([pinhole_inverse(Kt).reshape(1, 1, B, 9).expand(S, N, B, 9),
                      Kr.reshape(1, 1, B, 9).expand(S, N, B, 9),
                      T[:, :, :3, :].reshape(1, N, B, 12).expand(S, N, B, 12),
                      torch.zeros(S, N, B, _hip.CAMREC - 30, device=dev)], -1)
    assert torch.equal(cam, want)


def test_loss_grad_through_full_pose_matrices(dev):
    """MultiViewPhotometricLoss now hands the loss the whole [4,4] matrices: the pose gradient
    (bottom row zero) must equal the one through the [3,4] slices."""
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses._hip_photometric import photometric_loss_hip
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    g = torch.Generator().manual_seed(7)
    B, H, W = 2, 32, 96
    image = gu.smooth_texture(g, B, 3, H, W).to(dev)
    ctx = [gu.smooth_texture(g, B, 3, H, W).to(dev) for _ in range(2)]
    K = gu.kitti_K(B, H, W).to(dev)
    vec = gu.pose_vecs(g, B, 2).to(dev)
    sigs = [gu.sigmoid_maps(g, B, H, W).to(dev) for _ in range(4)]
    loss_fn = MultiViewPhotometricLoss(num_scales=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001,
                                       photometric_reduce_op="min", automask_loss=True, min_depth=0.5,
                                       max_depth=80.0)
    v1 = vec.clone().requires_grad_(True)
    out = loss_fn(image, ctx, sigs, K, K, Pose.from_vecs(v1, "euler"))
    out["loss"].sum().backward()
    v2 = vec.clone().requires_grad_(True)
    poses = Pose.from_vecs(v2, "euler")
    T = torch.stack([p.mat[:, :3, :] for p in poses], 0)
    from packnet_sfm_amd import _hip
    cfg = dict(n=4, automask=True, reduce_op=_hip.REDUCE_MIN, ssim_w=0.85, C1=float(loss_fn.C1),
               C2=float(loss_fn.C2), min_depth=0.5, max_depth=80.0, clip=float(loss_fn.clip_loss), smooth_w=0.001)
    loss2, _, _ = photometric_loss_hip(image, ctx, sigs, K, K, T, None, cfg)
    loss2.sum().backward()
    assert torch.equal(out["loss"].detach(), loss2.detach())
    torch.testing.assert_close(v1.grad, v2.grad, rtol=1e-6, atol=1e-9)
