"""Metric reductions (packnet_sfm/utils/reduce.py: reduce_dict :9-29, all_reduce_metrics :31-80)
over real collectives (utils/horovod.py)."""
import torch

from .horovod import allreduce, world_size


def reduce_dict(data, to_item=False):
    for key, val in data.items():
        data[key] = allreduce(data[key], average=True)
        if to_item:
            data[key] = data[key].item()
    return data


def all_reduce_metrics(metrics_sum, counts):
    """Sum per-dataset-sample metric tensors [N,7] and their seen-counts [N] over ranks, then
    average (each rank fills only the samples its DistributedSampler gave it)."""
    metrics_sum = allreduce(metrics_sum, average=False)
    counts = allreduce(counts, average=False)
    seen = counts.clamp(min=1).unsqueeze(-1)
    return (metrics_sum / seen).mean(0)


def average_key(batch_list, key):
    values = torch.stack([b[key] for b in batch_list])
    return values.mean()
