"""Depth evaluation of a batch — ModelWrapper.evaluate_depth (models/model_wrapper.py:621-789,
single-head path) with every metric on the HIP reduction of utils/depth.compute_depth_metrics.

The depth net outputs sigmoids; the evaluated depth is sigmoid -> bounded inverse depth ->
depth (the training conversion, post_process_depth.py:13-66), beside the linear and log
sigmoid->depth variants, each with and without ground-truth median scaling."""
from collections import OrderedDict
import types

import torch

from ..utils.depth import compute_depth_metrics, inv2depth
from ..utils.post_process_depth import sigmoid_to_depth_linear, sigmoid_to_depth_log, sigmoid_to_inv_depth


def _to_b1hw(x, device):  # model_wrapper.py:697-721
    if x is None or not isinstance(x, torch.Tensor):
        return None
    x = x.to(device=device, dtype=torch.float32)
    if x.dim() == 0:
        return x.view(1, 1, 1, 1)
    if x.dim() == 2:
        return x.unsqueeze(0).unsqueeze(0)
    if x.dim() == 3:
        return x.unsqueeze(0)[:, :1] if x.size(0) in (1, 3) else x.unsqueeze(1)
    if x.dim() == 4:
        return x[:, :1] if x.size(1) != 1 else x
    return None


@torch.no_grad()
def evaluate_depth(model, batch, min_depth, max_depth, crop="garg", scale_output="top-center",
                   use_log_space=False, metrics_fn=None):
    """Returns {'metrics': OrderedDict(depth, depth_gt, depth_lin, depth_lin_gt, depth_log,
    depth_log_gt) of [7] tensors, 'inv_depth', 'depth', 'depth_linear', 'depth_log'}.
    `metrics_fn` defaults to the HIP `compute_depth_metrics` (tests inject the CPU oracle)."""
    metrics_fn = compute_depth_metrics if metrics_fn is None else metrics_fn
    out = model(batch)
    sig0 = out["inv_depths"][0].float()
    inv_depth = sigmoid_to_inv_depth(sig0, min_depth, max_depth, use_log_space=use_log_space)
    depth_pred = inv2depth(inv_depth)
    depth_lin = sigmoid_to_depth_linear(sig0, min_depth, max_depth)
    depth_log = sigmoid_to_depth_log(sig0, min_depth, max_depth)
    gt = _to_b1hw(batch.get("depth"), depth_pred.device)
    cfg = types.SimpleNamespace(min_depth=min_depth, max_depth=max_depth, crop=crop, scale_output=scale_output)
    metrics = OrderedDict()
    if gt is not None:
        for name, pred in (("depth", depth_pred), ("depth_lin", depth_lin), ("depth_log", depth_log)):
            metrics[name] = metrics_fn(cfg, gt, pred, use_gt_scale=False)
            metrics[name + "_gt"] = metrics_fn(cfg, gt, pred, use_gt_scale=True)
    return {"metrics": metrics, "inv_depth": inv_depth, "depth": depth_pred, "depth_linear": depth_lin,
            "depth_log": depth_log}


def validation_step(model, batch, batch_idx, min_depth, max_depth, **kw):
    """ModelWrapper.validation_step (model_wrapper.py:354-398) minus the image logging:
    {'idx': sample indices, **metrics}."""
    output = evaluate_depth(model, batch, min_depth, max_depth, **kw)
    return {"idx": batch.get("idx", batch_idx), **output["metrics"]}


@torch.no_grad()
def validate(model, dataloaders, datasets, min_depth, max_depth, **kw):
    """HorovodTrainer.validate + ModelWrapper.validation_epoch_end (horovod_trainer.py:325-340,
    model_wrapper.py:476-539): every rank evaluates its DistributedSampler partition of each
    dataset; `utils.reduce.all_reduce_metrics` sums the per-sample metric vectors over ranks
    (asserting every sample was seen) and averages them.  Returns one OrderedDict per dataset
    (keys depth, depth_gt, depth_lin, depth_lin_gt, depth_log, depth_log_gt -> [7])."""
    from ..utils.reduce import all_reduce_metrics
    model.eval()
    outputs = []
    for loader in dataloaders:
        outputs.append([validation_step(model, batch, i, min_depth, max_depth, **kw)
                        for i, batch in enumerate(loader)])
    return all_reduce_metrics(outputs, datasets, "depth")
