"""Metric reductions of packnet_sfm/utils/reduce.py over real collectives (utils/horovod.py):
reduce_dict (:9-29), all_reduce_metrics (:31-80), collate_metrics (:84-113), create_dict
(:115-146), average_key / average_sub_key / average_loss_and_metrics (:150-220).

`all_reduce_metrics` keeps the reference's semantics — every dataset sample's metric vector is
placed at its index, summed over ranks together with how often each sample was seen, every
sample must have been seen (DistributedSampler pads the last ranks by repeating samples, so a
sample may be seen twice), and the per-sample average is averaged over the dataset — but sends
ONE all-reduce per dataset: [len(dataset), 1 + sum(dims)] float64 (seen counts beside every
metric), on the metrics' own device (RCCL for GPU tensors, gloo on CPU)."""
from collections import OrderedDict

import torch

from .horovod import reduce_value


def reduce_dict(data, to_item=False):
    for key, val in data.items():
        data[key] = reduce_value(data[key], average=True, name=key)
        if to_item:
            data[key] = data[key].item()
    return data


def all_reduce_metrics(output_data_batch, datasets, name="depth"):
    """output_data_batch: list (per dataset) of lists of per-batch dicts with 'idx' [b] and
    metric keys starting with `name` ([7] per batch, or [b, 7] per sample)."""
    if isinstance(output_data_batch[0], dict):
        output_data_batch = [output_data_batch]
    names = [k for k in output_data_batch[0][0].keys() if k.startswith(name)]
    dims = [output_data_batch[0][0][k].shape[-1] for k in names]
    all_metrics = []
    for output_batch, dataset in zip(output_data_batch, datasets):
        length = len(dataset)
        dev = output_batch[0][names[0]].device if names else torch.device("cpu")
        table = torch.zeros(length, 1 + sum(dims), dtype=torch.float64, device=dev)
        for out in output_batch:
            idx = torch.as_tensor(out["idx"], device=dev).reshape(-1).long()
            table[:, 0].index_add_(0, idx, torch.ones(idx.numel(), dtype=torch.float64, device=dev))
            col = 1
            for k, d in zip(names, dims):
                v = out[k].to(dev, torch.float64)
                # the reference assigns metrics[idx] = output[name] (a batch-level vector
                # broadcast to every sample of the batch)
                table[idx, col:col + d] = v.reshape(-1, d).expand(idx.numel(), d) if v.dim() == 1 else v
                col += d
        table = reduce_value(table, average=False, name="metrics")
        seen = table[:, 0]
        assert bool((seen > 0).all()), "Not all samples were seen during evaluation"
        metrics = OrderedDict()
        col = 1
        for k, d in zip(names, dims):
            metrics[k] = (table[:, col:col + d] / seen.view(-1, 1)).mean(0).float()
            col += d
        all_metrics.append(metrics)
    return all_metrics


def collate_metrics(output_data_batch, name="depth"):
    if isinstance(output_data_batch[0], dict):
        output_data_batch = [output_data_batch]
    metrics_data = []
    for output_batch in output_data_batch:
        metrics = OrderedDict()
        for key in output_batch[0]:
            if key.startswith(name):
                metrics[key] = torch.stack([o[key] for o in output_batch], 0).mean(0)
        metrics_data.append(metrics)
    return metrics_data


def create_dict(metrics_data, metrics_keys, metrics_modes, prefixes, name="depth"):
    """`prefixes[n]` replaces the reference's prepare_dataset_prefix(config, n)."""
    out = {}
    for n, metrics in enumerate(metrics_data):
        if metrics:
            for i, key in enumerate(metrics_keys):
                for mode in metrics_modes:
                    out["{}-{}{}".format(prefixes[n], key, mode)] = metrics["{}{}".format(name, mode)][i].item()
    return out


def average_key(batch_list, key):
    values = [b[key] for b in batch_list]
    return sum(values) / len(values)


def average_sub_key(batch_list, key, sub_key):
    values = [b[key][sub_key] for b in batch_list]
    return sum(values) / len(values)


def average_loss_and_metrics(batch_list, prefix):
    values = OrderedDict()
    values["{}-loss".format(prefix)] = average_key(batch_list, "loss")
    for sub_key in batch_list[0]["metrics"].keys():
        values["{}-{}".format(prefix, sub_key)] = average_sub_key(batch_list, "metrics", sub_key)
    return values
