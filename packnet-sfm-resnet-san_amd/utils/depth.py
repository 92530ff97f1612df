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
    """[abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3] averaged over the batch.

    Batched on the device (one masked reduction per image, medians via torch.median on the
    valid pixels); same semantics as the reference's per-image loop.
    """
    B, _, H, W = gt.shape
    pred = scale_depth(pred, gt, config.scale_output)
    crop = garg_crop_mask(H, W, gt.device) if config.crop == "garg" else None
    acc = torch.zeros(7, dtype=torch.float64, device=gt.device)
    for g, p in zip(gt[:, 0], pred[:, 0]):
        valid = (g > config.min_depth) & (g < config.max_depth)
        if crop is not None:
            valid = valid & crop
        if not bool(valid.any()):
            continue
        g, p = g[valid], p[valid]
        if use_gt_scale:
            p = p * (torch.median(g) / torch.median(p))
        th = torch.max(g / p, p / g)
        d = g - p
        acc += torch.stack([(d.abs() / g).mean(), (d ** 2 / g).mean(), (d ** 2).mean().sqrt(),
                            ((g.log() - p.log()) ** 2).mean().sqrt(), (th < 1.25).float().mean(),
                            (th < 1.25 ** 2).float().mean(), (th < 1.25 ** 3).float().mean()]).double()
    return (acc / B).to(gt.dtype)
