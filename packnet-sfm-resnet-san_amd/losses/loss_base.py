"""LossBase / ProgressiveScaling (packnet_sfm/losses/loss_base.py:10-81)."""
import numpy as np
import torch
import torch.nn as nn


class ProgressiveScaling:
    """After each `progressive_scaling` fraction of training, drop one scale — as documented.  As
    executed by the reference, never: it keeps the thresholds in an np.float32 array and tests
    `is_list(...)` (utils/types.py:21-23, isinstance(data, list)), which is False for an array,
    so __call__ always returns num_scales (loss_base.py:23-49; goldens loss_progressive_p03 /
    _p06).  `reference_quirk=False` applies the documented schedule instead."""

    def __init__(self, progressive_scaling, num_scales=4, reference_quirk=True):
        self.num_scales = num_scales
        self.reference_quirk = reference_quirk
        if progressive_scaling > 0.0:
            self.progressive_scaling = np.float32(
                [progressive_scaling * (i + 1) for i in range(num_scales - 1)] + [1.0])
        else:
            self.progressive_scaling = progressive_scaling

    def __call__(self, progress):
        if isinstance(self.progressive_scaling, np.ndarray) and not self.reference_quirk:
            return int(self.num_scales - np.searchsorted(self.progressive_scaling, progress))
        return self.num_scales


class LossBase(nn.Module):
    def __init__(self):
        super().__init__()
        self._logs = {}
        self._metrics = {}

    @property
    def logs(self):
        return self._logs

    @property
    def metrics(self):
        return self._metrics

    def add_metric(self, key, val):
        self._metrics[key] = val.detach() if hasattr(val, "detach") else torch.tensor(float(val))
