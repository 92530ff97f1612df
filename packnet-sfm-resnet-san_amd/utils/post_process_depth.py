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
