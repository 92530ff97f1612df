"""Per-sample mirror of packnet_sfm/datasets/transforms.py (train_transforms :21-50,
validation_transforms :52-77) over the batched GPU transform in augmentations.py.

A sample holds decoded uint8 HWC images on a ROCm device ('rgb' [h,w,3], 'rgb_context'
[[h,w,3], ...]) instead of PIL images; the result holds fp32 CHW tensors like the reference's
`to_tensor_sample` output.  For throughput call `train_transforms_batch` on a whole batch.
"""
import random
from functools import partial

from .augmentations import train_transforms_batch, validation_transforms_batch


def _batched(sample):
    b = {k: v for k, v in sample.items()}
    b["rgb"] = sample["rgb"][None]
    if "rgb_context" in sample:
        b["rgb_context"] = [c[None] for c in sample["rgb_context"]]
    if "intrinsics" in sample:
        b["intrinsics"] = sample["intrinsics"][None]
    return b


def _unbatched(out):
    res = {}
    for k, v in out.items():
        if isinstance(v, list) and k != "jitter_params":
            res[k] = [t[0] for t in v]
        elif k == "jitter_params":
            res[k] = None if v is None else v[0]
        elif hasattr(v, "dim") and k in ("rgb", "rgb_original", "intrinsics", "intrinsics_full"):
            res[k] = v[0]
        else:
            res[k] = v
    return res


def train_transforms(sample, image_shape, jittering, crop_train_borders, rng=random):
    """datasets/transforms.py:21-50 for one sample."""
    return _unbatched(train_transforms_batch(_batched(sample), image_shape, jittering, crop_train_borders, rng=rng))


def validation_transforms(sample, image_shape, crop_eval_borders):
    """datasets/transforms.py:52-77 for one sample."""
    return _unbatched(validation_transforms_batch(_batched(sample), image_shape, crop_eval_borders))


def get_transforms(mode, image_shape=(), jittering=(), crop_train_borders=(), crop_eval_borders=()):
    """datasets/transforms.py get_transforms: the per-sample transform for a split."""
    if mode == "train":
        return partial(train_transforms, image_shape=image_shape, jittering=jittering,
                       crop_train_borders=crop_train_borders)
    if mode in ("validation", "test"):
        return partial(validation_transforms, image_shape=image_shape, crop_eval_borders=crop_eval_borders)
    raise ValueError("Unknown mode {}".format(mode))
