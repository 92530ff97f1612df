"""Model output helpers (packnet_sfm/models/model_utils.py): `merge_outputs` (:33-65),
`stack_batch` (:68-94), `flip_batch_input` (:97-124), `flip_output` (:127-149),
`upsample_output` (:152-196)."""
import torch

from ..utils.image import NearestScales, flip_lr, interpolate_scales
from ..utils.misc import filter_dict


def flip(tensor, flip_fn):
    if not isinstance(tensor, list):
        return flip_fn(tensor)
    if not isinstance(tensor[0], list):
        return [flip_fn(v) for v in tensor]
    return [[flip_fn(v) for v in vs] for vs in tensor]


def merge_outputs(*outputs):
    ignore, combine = ["loss"], ["metrics"]
    merge = {key: {} for key in combine}
    for output in outputs:
        for key, val in output.items():
            if key in combine:
                for sk, sv in val.items():
                    assert sk not in merge[key], "Combining duplicated key {} to {}".format(sk, key)
                    merge[key][sk] = sv
            elif key not in ignore:
                assert key not in merge, "Adding duplicated key {}".format(key)
                merge[key] = val
    return merge


def stack_batch(batch):
    if len(batch["rgb"].shape) == 5:
        assert batch["rgb"].shape[0] == 1, "Only batch size 1 is supported for multi-cameras"
        for key in batch.keys():
            if isinstance(batch[key], list):
                if torch.is_tensor(batch[key][0]) or hasattr(batch[key][0], "shape"):
                    batch[key] = [sample[0] for sample in batch[key]]
            else:
                batch[key] = batch[key][0]
    return batch


def flip_batch_input(batch):
    for key in filter_dict(batch, ["rgb", "rgb_context", "input_depth", "input_depth_context"]):
        batch[key] = flip(batch[key], flip_lr)
    for key in filter_dict(batch, ["intrinsics"]):
        batch[key] = batch[key].clone()
        batch[key][:, 0, 2] = batch["rgb"].shape[3] - batch[key][:, 0, 2]
    return batch


def flip_output(output):
    for key in filter_dict(output, ["uncertainty", "logits_semantic", "ord_probability", "inv_depths",
                                    "inv_depths_context", "inv_depths1", "inv_depths2", "pred_depth",
                                    "pred_depth_context", "pred_depth1", "pred_depth2", "pred_inv_depth",
                                    "pred_inv_depth_context", "pred_inv_depth1", "pred_inv_depth2"]):
        output[key] = flip(output[key], flip_lr)
    return output


def upsample_output(output, mode="nearest", align_corners=None, lazy=False):
    """`lazy` (the training step, SfmModel.compute_depth_net): 'inv_depths' reaching full size by
    exact 2^k nearest factors become a NearestScales sequence — the loss reads the stored maps
    through the index mapping and nothing full-size is written (utils/image.py)."""
    for key in filter_dict(output, ["inv_depths", "uncertainty"]):
        v = output[key]
        if lazy and key == "inv_depths" and mode == "nearest" and NearestScales.exact(v, v[0].shape[-2:]):
            output[key] = NearestScales(v, v[0].shape[-2:])
            continue
        output[key] = interpolate_scales(v, mode=mode, align_corners=align_corners)
    for key in filter_dict(output, ["inv_depths_context"]):
        output[key] = [interpolate_scales(v, mode=mode, align_corners=align_corners) for v in output[key]]
    return output
