"""monodepth2-style decoder blocks as used by this fork (packnet_sfm/networks/layers/resnet/
layers.py:12-72): Conv3x3 with zero padding inside the conv, ConvBlock = Conv3x3 + ReLU."""
import torch.nn as nn
import torch.nn.functional as F

from ..fused import ACT_RELU, bias_act, conv_nobias
from ....utils.image import upsample_nearest


def disp_to_depth(disp, min_depth, max_depth):
    lo, hi = 1 / max_depth, 1 / min_depth
    scaled = lo + (hi - lo) * disp
    return scaled, 1 / scaled


class Conv3x3(nn.Module):
    def __init__(self, in_channels, out_channels, use_refl=False):
        super().__init__()
        self.pad = nn.ReflectionPad2d(1) if use_refl else None
        self.conv = nn.Conv2d(int(in_channels), int(out_channels), 3, padding=0 if use_refl else 1)

    def forward(self, x):
        return self.conv(self.pad(x) if self.pad is not None else x)


class ConvBlock(nn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = Conv3x3(in_channels, out_channels)
        self.nonlin = nn.ReLU(inplace=True)

    def forward(self, x, nout=1):
        # Conv3x3 without its bias + fused (bias + ReLU) epilogue with the bias-gradient reduction;
        # nout > 1: forked output for several consumers (fused._fork)
        c = self.conv
        x = c.pad(x) if c.pad is not None else x
        return bias_act(conv_nobias(c.conv, x), c.conv.bias, ACT_RELU, self, nout=nout)


def upsample(x):
    """F.interpolate(x, scale_factor=2, mode='nearest') with a deterministic backward."""
    return upsample_nearest(x, 2)
