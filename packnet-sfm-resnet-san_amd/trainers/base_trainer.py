"""Trainer helpers (packnet_sfm/trainers/base_trainer.py): `sample_to_cuda` (:8-39) is the
host->device boundary of a batch."""
import torch


def sample_to_cuda(data, dtype=None, device=None, non_blocking=True):
    if isinstance(data, str):
        return data
    if isinstance(data, dict):
        return {k: sample_to_cuda(v, dtype, device, non_blocking) for k, v in data.items()}
    if isinstance(data, (list, tuple)):
        return [sample_to_cuda(v, dtype, device, non_blocking) for v in data]
    if torch.is_tensor(data):
        dev = device or torch.device("cuda", torch.cuda.current_device())
        t = data.to(dev, non_blocking=non_blocking)
        return t.to(dtype) if dtype is not None and t.is_floating_point() else t
    return data
