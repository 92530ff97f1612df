"""SelfSupModel (packnet_sfm/models/SelfSupModel.py:8-121): SfmModel + MultiViewPhotometricLoss.

Differences from the fork, all documented in DESIGN.md §Semantics:
  * `forward` accepts the `masks=` keyword its caller passes (model_wrapper.py:299 — the fork's
    signature rejects it); the mask is `masks` if given, else batch['mask'];
  * cameras: a fisheye (VADAS) dict in batch['distortion_coeffs'] goes to the loss for both
    cameras, as the fork does (:108-117); otherwise the pinhole batch['intrinsics'] [B,3,3].
"""
import torch

from ..losses.multiview_photometric_loss import MultiViewPhotometricLoss
from .SfmModel import SfmModel
from .model_utils import merge_outputs
from ..datasets.synthetic import flatten_cameras


class SelfSupModel(SfmModel):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self._photometric_loss = MultiViewPhotometricLoss(**kwargs)

    @property
    def logs(self):
        return {**super().logs, **self._photometric_loss.logs}

    def self_supervised_loss(self, image, ref_images, inv_depths, poses, intrinsics, ref_intrinsics=None,
                             return_logs=False, progress=0.0, mask=None):
        return self._photometric_loss(image, ref_images, inv_depths, intrinsics,
                                      intrinsics if ref_intrinsics is None else ref_intrinsics, poses,
                                      return_logs=return_logs, progress=progress, mask=mask)

    def forward(self, batch, return_logs=False, progress=0.0, masks=None, **kwargs):
        if batch["rgb"].dim() == 5:   # multi-camera samples: cameras -> batch (SfmModel.forward)
            batch = flatten_cameras(batch)
        output = super().forward(batch, return_logs=return_logs)
        if not self.training:
            return output
        dc = batch.get("distortion_coeffs", None)
        K = dc if isinstance(dc, dict) else batch["intrinsics"]
        mask = masks if masks is not None else batch.get("mask", None)
        self_sup_output = self.self_supervised_loss(
            batch["rgb_original"], batch["rgb_context_original"], output["inv_depths"], output["poses"],
            K, return_logs=return_logs, progress=progress, mask=mask)
        return {"loss": self_sup_output["loss"], **merge_outputs(output, self_sup_output)}
