"""Sigmoid -> (inverse) depth conversions (packnet_sfm/utils/post_process_depth.py:13-108)."""
import math

import torch


def _inv_range(min_depth, max_depth):
    return 1.0 / max(max_depth, 1e-6), 1.0 / max(min_depth, 1e-6)


def sigmoid_to_inv_depth(sigmoid_output, min_depth=0.05, max_depth=80.0, use_log_space=False):
    lo, hi = _inv_range(min_depth, max_depth)
    if use_log_space:
        return torch.exp(math.log(lo) + (math.log(hi) - math.log(lo)) * sigmoid_output)
    return lo + (hi - lo) * sigmoid_output


def sigmoid_to_depth_linear(sigmoid_output, min_depth=0.05, max_depth=80.0):
    lo, hi = _inv_range(min_depth, max_depth)
    return 1.0 / (lo + (hi - lo) * sigmoid_output + 1e-8)


def sigmoid_to_depth_log(sigmoid_output, min_depth=0.05, max_depth=80.0):
    """post_process_depth.py:111-170: interpolation in log(inverse depth) space (the INT8
    post-processing variant the reference evaluates beside the linear one)."""
    lo, hi = _inv_range(min_depth, max_depth)
    log_lo = torch.log(torch.tensor(lo, device=sigmoid_output.device))
    log_hi = torch.log(torch.tensor(hi, device=sigmoid_output.device))
    inv = torch.exp(log_lo + (log_hi - log_lo) * sigmoid_output)
    return 1.0 / (inv + 1e-8)
