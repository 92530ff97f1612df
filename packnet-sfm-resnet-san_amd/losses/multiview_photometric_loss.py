"""MultiViewPhotometricLoss — same constructor kwargs, `forward` signature and return dict as
packnet_sfm/losses/multiview_photometric_loss.py:58-410, computed by the fused HIP kernels
(losses/_hip_photometric.py -> include/psfm.h).

Semantics (pinned by tests/golden/, generated from the reference):
  * `inv_depths` are the depth net's SIGMOID outputs (fork semantics, :362-369): depth =
    sigmoid_to_depth_linear(s), inv = 1/(depth+1e-8), warp depth = 1/clamp(inv, 1e-6);
    smoothness acts on the sigmoid maps (:404-405);
  * pinhole intrinsics `K [B,3,3]` or the fork's FisheyeCamera (VADAS) dicts {k [B,7], s, div,
    ux, uy} (:131-195; the pose is applied to the reconstructed points as R X + t, which the fork
    cannot do on CPU / on [B,3,N]); `mask=None` means "no mask" (== all ones);
  * `metrics['photometric_loss']` aliases the loss value, as the reference's in-place
    `loss += smoothness` does (:296, :405).
"""
import torch

from .loss_base import LossBase, ProgressiveScaling
from ._hip_photometric import photometric_loss_hip
from .. import _hip
from ..utils.image import NearestScales


def SSIM(x, y, C1=1e-4, C2=9e-4, kernel_size=3, stride=1):
    """Reference SSIM map (:15-54) — kept for API parity / diagnostics (not on the hot path)."""
    import torch.nn.functional as F
    x, y = F.pad(x, (1, 1, 1, 1), mode="reflect"), F.pad(y, (1, 1, 1, 1), mode="reflect")
    pool = lambda t: F.avg_pool2d(t, kernel_size, stride)  # noqa: E731
    mx, my = pool(x), pool(y)
    sx, sy, sxy = pool(x * x) - mx * mx, pool(y * y) - my * my, pool(x * y) - mx * my
    return ((2 * mx * my + C1) * (2 * sxy + C2)) / ((mx * mx + my * my + C1) * (sx + sy + C2))


class MultiViewPhotometricLoss(LossBase):
    def __init__(self, num_scales=4, ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.1,
                 C1=1e-4, C2=9e-4, photometric_reduce_op="mean", disp_norm=True, clip_loss=0.5,
                 progressive_scaling=0.0, padding_mode="zeros", automask_loss=False,
                 min_depth=0.05, max_depth=80.0, **kwargs):
        super().__init__()
        self.n = num_scales
        self.ssim_loss_weight = ssim_loss_weight
        self.occ_reg_weight = occ_reg_weight
        self.smooth_loss_weight = smooth_loss_weight
        self.C1, self.C2 = C1, C2
        self.photometric_reduce_op = photometric_reduce_op
        self.disp_norm = disp_norm
        self.clip_loss = clip_loss
        self.padding_mode = padding_mode
        self.automask_loss = automask_loss
        self.min_depth, self.max_depth = min_depth, max_depth
        self.progressive_scaling = ProgressiveScaling(progressive_scaling, self.n)
        if self.automask_loss:
            assert self.photometric_reduce_op == "min", \
                "For automasking only the min photometric_reduce_op is supported."
        if photometric_reduce_op not in ("min", "mean"):
            raise NotImplementedError("Unknown photometric_reduce_op: {}".format(photometric_reduce_op))
        if padding_mode != "zeros":
            raise NotImplementedError("HIP photometric path implements padding_mode='zeros' (reference default)")

    @property
    def logs(self):
        return {"num_scales": self.n}

    def forward(self, image, context, inv_depths, intrinsics, ref_intrinsics, poses,
                return_logs=False, progress=0.0, mask=None):
        if isinstance(intrinsics, dict) != isinstance(ref_intrinsics, dict):
            raise ValueError("intrinsics and ref_intrinsics must be both pinhole K or both fisheye dicts")
        self.n = self.progressive_scaling(progress)
        if isinstance(inv_depths, NearestScales):   # stored maps + 2^k nearest mapping (no full-size copies)
            sigs = NearestScales([s.float() for s in inv_depths.stored[:self.n]], inv_depths.shape)
        else:
            sigs = [s.float() for s in inv_depths[:self.n]]  # nets may run under bf16 autocast
        # [N,B,4,4], differentiable: the whole matrices (the kernels read rows 0-2 and write a zero
        # bottom-row gradient), so autograd needs no slice / zero-fill per pose
        T = torch.stack([p.mat for p in poses], 0)
        cfg = dict(n=self.n, automask=bool(self.automask_loss),
                   reduce_op=_hip.REDUCE_MIN if self.photometric_reduce_op == "min" else _hip.REDUCE_MEAN,
                   ssim_w=float(self.ssim_loss_weight), C1=float(self.C1), C2=float(self.C2),
                   min_depth=float(self.min_depth), max_depth=float(self.max_depth),
                   clip=float(self.clip_loss), smooth_w=float(self.smooth_loss_weight))
        if mask is not None:
            mask = mask.float()
        with torch.autocast("cuda", enabled=False):   # the photometric path is fp32 end to end
            fl = (lambda k: {n: v.float() for n, v in k.items()}) if isinstance(intrinsics, dict) else \
                (lambda k: k.float())
            loss, photo, smooth = photometric_loss_hip(image.float(), [c.float() for c in context], sigs,
                                                       fl(intrinsics), fl(ref_intrinsics), T.float(), mask, cfg)
        self.add_metric("photometric_loss", photo)
        if self.smooth_loss_weight > 0.0:
            self.add_metric("smoothness_loss", smooth)
        return {"loss": loss, "metrics": self.metrics}
