"""GPU parity of the depth-evaluation reduction (include/psfm_metrics.h, the Abs Rel gate;
reference packnet_sfm/utils/depth.py:258-447) against the reference's golden fixture and the CPU
oracle (oracle.depth_metrics, itself pinned to that fixture in test_oracle_golden.py).

Tolerance: 1e-5 relative on the 7-vector (fp64 sums vs the reference's fp32 means; the medians
are exact — radix select on the float bits)."""
import types

import numpy as np
import pytest
import torch

import golden_util as gu

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import __graft_entry__
    __graft_entry__.build()
    return torch.device("cuda:0")


def _cfg(min_depth=0.0, max_depth=80.0, crop="garg", scale_output="top-center"):
    return types.SimpleNamespace(min_depth=min_depth, max_depth=max_depth, crop=crop, scale_output=scale_output)


def _metrics_inputs():  # the generator of tools/gen_goldens.py:gen_depth_metrics
    g = torch.Generator().manual_seed(31)
    B, H, W = 2, 192, 640
    gt = 1.0 + 79.0 * torch.rand(B, 1, H, W, generator=g)
    gt[torch.rand(B, 1, H, W, generator=g) < 0.6] = 0.0
    pred = gt.clamp(min=1.0) * (1.0 + 0.1 * torch.randn(B, 1, H, W, generator=g)) * 1.3
    return gt, pred.clamp(0.5, 90.0)


def test_matches_reference_golden(dev):
    from packnet_sfm_amd.utils.depth import compute_depth_metrics
    z = gu.load_golden("depth_metrics")
    gt, pred = _metrics_inputs()
    gt, pred = gt.to(dev), pred.to(dev)
    assert gu.rel_err(compute_depth_metrics(_cfg(), gt, pred, True).cpu(), z["with_scale"]) < TOL
    assert gu.rel_err(compute_depth_metrics(_cfg(), gt, pred, False).cpu(), z["no_scale"]) < TOL
    assert gu.rel_err(compute_depth_metrics(_cfg(1e-3, crop=""), gt, pred, True).cpu(), z["no_crop"]) < TOL


@pytest.mark.parametrize("B,H,W,density,quant", [(3, 192, 640, 0.3, 0.0), (2, 375, 1242, 0.05, 0.0),
                                                 (2, 31, 57, 0.5, 0.5), (1, 8, 8, 1.0, 4.0)])
def test_matches_oracle(dev, B, H, W, density, quant):
    """random sparse gt (velodyne-like), ties when quantised, odd and even valid counts, and an
    image without any valid pixel (contributes 0, still divides by B)"""
    from oracle import photometric_oracle as O
    from packnet_sfm_amd.utils.depth import compute_depth_metrics
    g = torch.Generator().manual_seed(B * 1000 + H)
    gt = 0.5 + 85.0 * torch.rand(B, 1, H, W, generator=g)
    if quant > 0:
        gt = torch.round(gt / quant) * quant + quant   # many exact ties
    gt[torch.rand(B, 1, H, W, generator=g) > density] = 0.0
    if B > 1:
        gt[-1] = 0.0
    pred = (gt.clamp(min=1.0) * (1.0 + 0.2 * torch.randn(B, 1, H, W, generator=g)) * 0.7).clamp(0.3, 95.0)
    for crop in ("garg", ""):
        for scale in (True, False):
            ref = O.depth_metrics(gt, pred, 0.0, 80.0, crop, scale)
            got = compute_depth_metrics(_cfg(crop=crop), gt.to(dev), pred.to(dev), scale).cpu()
            assert gu.rel_err(got, ref) < TOL, (crop, scale, got, ref)


def test_resize_scale_output_and_determinism(dev):
    """pred at network resolution, bilinearly resized to the gt size ('resize', depth.py:450-483)"""
    from oracle import photometric_oracle as O
    from packnet_sfm_amd.utils.depth import compute_depth_metrics
    g = torch.Generator().manual_seed(7)
    gt = 1.0 + 70.0 * torch.rand(2, 1, 96, 320, generator=g)
    gt[torch.rand(2, 1, 96, 320, generator=g) < 0.7] = 0.0
    pred = 1.0 + 70.0 * torch.rand(2, 1, 48, 160, generator=g)
    up = torch.nn.functional.interpolate(pred, size=(96, 320), mode="bilinear", align_corners=True)
    ref = O.depth_metrics(gt, up, 0.0, 80.0, "garg", True)
    a = compute_depth_metrics(_cfg(scale_output="resize"), gt.to(dev), pred.to(dev), True)
    b = compute_depth_metrics(_cfg(scale_output="resize"), gt.to(dev), pred.to(dev), True)
    assert gu.rel_err(a.cpu(), ref) < 1e-4   # ATen-GPU vs ATen-CPU bilinear resample
    assert torch.equal(a, b)


def test_all_invalid_batch_is_zero(dev):
    from packnet_sfm_amd.utils.depth import compute_depth_metrics
    gt = torch.zeros(2, 1, 16, 16, device=dev)
    out = compute_depth_metrics(_cfg(), gt, torch.ones_like(gt), True)
    assert torch.equal(out.cpu(), torch.zeros(7))
    np.testing.assert_equal(out.shape, (7,))


def test_evaluate_depth_batch(dev):
    """ModelWrapper.evaluate_depth (model_wrapper.py:621-789): sigmoid -> depth variants, 6 metric
    vectors, each equal to the oracle on the same conversions."""
    from oracle import photometric_oracle as O
    from packnet_sfm_amd.models.evaluate import evaluate_depth
    g = torch.Generator().manual_seed(3)
    sig = torch.rand(2, 1, 64, 160, generator=g) * 0.3 + 0.02
    gt = 1.0 + 60.0 * torch.rand(2, 1, 64, 160, generator=g)
    gt[torch.rand(2, 1, 64, 160, generator=g) < 0.5] = 0.0

    class Stub(torch.nn.Module):
        def forward(self, batch):
            return {"inv_depths": [sig.to(dev)]}

    res = evaluate_depth(Stub(), {"rgb": None, "depth": gt[:, 0].to(dev)}, 0.5, 80.0)
    assert list(res["metrics"]) == ["depth", "depth_gt", "depth_lin", "depth_lin_gt", "depth_log", "depth_log_gt"]
    inv = 1 / 80.0 + (1 / 0.5 - 1 / 80.0) * sig
    depth = 1.0 / inv.clamp(min=1e-6)
    for scale, key in ((False, "depth"), (True, "depth_gt")):
        ref = O.depth_metrics(gt, depth, 0.5, 80.0, "garg", scale)
        assert gu.rel_err(res["metrics"][key].cpu(), ref) < 1e-4, key
    lin = O.sigmoid_to_depth(sig, 0.5, 80.0)
    assert gu.rel_err(res["metrics"]["depth_lin_gt"].cpu(), O.depth_metrics(gt, lin, 0.5, 80.0, "garg", True)) < 1e-4
