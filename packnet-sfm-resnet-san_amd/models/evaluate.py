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
                   use_log_space=False):
    """Returns {'metrics': OrderedDict(depth, depth_gt, depth_lin, depth_lin_gt, depth_log,
    depth_log_gt) of [7] tensors, 'inv_depth', 'depth', 'depth_linear', 'depth_log'}."""
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
            metrics[name] = compute_depth_metrics(cfg, gt, pred, use_gt_scale=False)
            metrics[name + "_gt"] = compute_depth_metrics(cfg, gt, pred, use_gt_scale=True)
    return {"metrics": metrics, "inv_depth": inv_depth, "depth": depth_pred, "depth_linear": depth_lin,
            "depth_log": depth_log}
