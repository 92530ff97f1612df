"""Depth helpers (packnet_sfm/utils/depth.py): `inv2depth` (:103-120), `depth2inv`,
`inv_depths_normalize` (:146-162), `calc_smoothness` (:165-198), `scale_depth` (:450-483)
and `compute_depth_metrics` (:258-447, the Abs Rel gate)."""
import torch

from .image import gradient_x, gradient_y, interpolate_image


def inv2depth(inv_depth):
    if isinstance(inv_depth, (list, tuple)):
        return [inv2depth(x) for x in inv_depth]
    return 1.0 / inv_depth.clamp(min=1e-6)


def depth2inv(depth):
    if isinstance(depth, (list, tuple)):
        return [depth2inv(x) for x in depth]
    inv = 1.0 / depth.clamp(min=1e-6)
    inv[depth <= 0.0] = 0.0
    return inv


def inv_depths_normalize(inv_depths):
    return [d / d.mean(2, True).mean(3, True).clamp(min=1e-6) for d in inv_depths]


def calc_smoothness(inv_depths, images, num_scales):
    norm = inv_depths_normalize(inv_depths)
    sx, sy = [], []
    for i in range(num_scales):
        wx = torch.exp(-gradient_x(images[i]).abs().mean(1, keepdim=True))
        wy = torch.exp(-gradient_y(images[i]).abs().mean(1, keepdim=True))
        sx.append(gradient_x(norm[i]) * wx)
        sy.append(gradient_y(norm[i]) * wy)
    return sx, sy


def scale_depth(pred, gt, scale_fn):
    if scale_fn == "resize":
        return interpolate_image(pred, gt.shape, mode="bilinear", align_corners=True)
    if scale_fn != "top-center":
        raise NotImplementedError("Depth scale function {} not implemented.".format(scale_fn))
    out = torch.zeros(gt.shape, dtype=pred.dtype, device=pred.device)
    top, left = gt.shape[2] - pred.shape[2], (gt.shape[3] - pred.shape[3]) // 2
    out[:, :, top:top + pred.shape[2], left:left + pred.shape[3]] = pred
    return out


def garg_crop_mask(H, W, device=None):
    m = torch.zeros(H, W, dtype=torch.bool, device=device)
    m[int(0.40810811 * H):int(0.99189189 * H), int(0.03594771 * W):int(0.96405229 * W)] = True
    return m


def compute_depth_metrics(config, gt, pred, use_gt_scale=True):
    """[abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3] averaged over the batch — utils/depth.py:258-447.

    `scale_depth` (ATen resample / uncrop) then ONE HIP reduction (csrc/psfm_metrics.hip,
    include/psfm_metrics.h): per image the valid mask, exact lower medians by radix select, median
    scaling and the seven metrics; batch average with images without valid pixels adding 0.
    ROCm tensors only (no CPU fallback; the CPU restatement is oracle.depth_metrics)."""
    from .. import _hip
    import ctypes
    pred = scale_depth(pred, gt, config.scale_output)
    gt32, pred32 = gt.float().contiguous(), pred.float().contiguous()
    _hip.require_device(gt32, pred32)
    B, _, H, W = gt.shape
    p = _hip.MetricsParams(B=B, H=H, W=W, min_depth=float(config.min_depth), max_depth=float(config.max_depth),
                           crop_garg=int(config.crop == "garg"), use_gt_scale=int(bool(use_gt_scale)))
    per = torch.empty(B, 8, device=gt.device, dtype=torch.float32)
    out = torch.empty(7, device=gt.device, dtype=torch.float32)
    _hip.check(_hip.lib().psfm_depth_metrics(ctypes.byref(p), _hip.ptr(gt32), _hip.ptr(pred32), _hip.ptr(per),
                                             _hip.ptr(out), _hip.stream(gt.device)), "psfm_depth_metrics")
    return out.to(gt.dtype)
