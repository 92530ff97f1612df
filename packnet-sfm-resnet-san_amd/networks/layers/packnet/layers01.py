"""PackNet building blocks (packnet_sfm/networks/layers/packnet/layers01.py:10-286), PyTorch-ROCm
(MIOpen convolutions).  Parameter names match the reference so its checkpoints load as-is.

`packing` (space-to-depth) is a pure index permutation; on a ROCm device the pack / unpack
3-D convolutions run as one fused HIP kernel per direction (pack3d.py, include/psfm_pack3d.h).
"""
from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..fused import ACT_ELU, gn_act
from . import packconv
from .pack3d import conv3d_unpack, pack_conv3d


class Conv2D(nn.Module):
    """zero-pad(k//2) -> Conv2d -> GroupNorm(16) -> ELU.  The zero padding is the convolution's
    own (`padding=k//2`, identical arithmetic to ConstantPad2d + unpadded conv, layers01.py:34-39)
    instead of a padded copy of the input; `pad` is kept as the (parameter-free) module.  The conv
    bias, GroupNorm and ELU run as one fused pass each way on bf16 channels_last activations
    (fused.gn_act, include/psfm_netops.h) instead of autocast's fp32 GroupNorm round trip."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__()
        self.kernel_size = kernel_size
        self.conv_base = nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size, stride=stride)
        self.pad = nn.ConstantPad2d([kernel_size // 2] * 4, value=0)
        self.normalize = nn.GroupNorm(16, out_channels)
        self.activ = nn.ELU(inplace=True)

    def forward(self, x):
        c = self.conv_base
        return gn_act(F.conv2d(x, c.weight, None, c.stride, self.kernel_size // 2), c.bias, self.normalize,
                      act=ACT_ELU)


class ResidualConv(nn.Module):
    """Two Conv2D + 1x1 shortcut, GroupNorm + ELU after the sum."""

    def __init__(self, in_channels, out_channels, stride, dropout=None):
        super().__init__()
        self.conv1 = Conv2D(in_channels, out_channels, 3, stride)
        self.conv2 = Conv2D(out_channels, out_channels, 3, 1)
        shortcut = nn.Conv2d(in_channels, out_channels, kernel_size=1, stride=stride)
        self.conv3 = nn.Sequential(shortcut, nn.Dropout2d(dropout)) if dropout else shortcut
        self.normalize = nn.GroupNorm(16, out_channels)
        self.activ = nn.ELU(inplace=True)

    def forward(self, x):
        # GN(conv2(conv1(x)) + shortcut(x)) + ELU: the sum, shortcut bias, GroupNorm and ELU fused
        r = self.conv2(self.conv1(x))
        if isinstance(self.conv3, nn.Conv2d):
            c = self.conv3
            return gn_act(F.conv2d(x, c.weight, None, c.stride), c.bias, self.normalize, act=ACT_ELU, residual=r)
        return gn_act(self.conv3(x), None, self.normalize, act=ACT_ELU, residual=r)


def ResidualBlock(in_channels, out_channels, num_blocks, stride, dropout=None):
    blocks = [ResidualConv(in_channels, out_channels, stride, dropout=dropout)]
    blocks += [ResidualConv(out_channels, out_channels, 1, dropout=dropout) for _ in range(1, num_blocks)]
    return nn.Sequential(*blocks)


class InvDepth(nn.Module):
    """3x3 conv -> sigmoid / min_depth.  As in Conv2D, the zero padding is the convolution's own
    (`padding=1` == ConstantPad2d(1) + unpadded conv, layers01.py:66-78) instead of a padded copy of
    the input (and its slice backward): at the full-resolution head that copy is 47 MB each way."""

    def __init__(self, in_channels, out_channels=1, min_depth=0.5):
        super().__init__()
        self.min_depth = min_depth
        self.conv1 = nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=1)
        self.pad = nn.ConstantPad2d([1] * 4, value=0)
        self.activ = nn.Sigmoid()

    def forward(self, x):
        c = self.conv1
        return self.activ(F.conv2d(x, c.weight, c.bias, c.stride, 1)) / self.min_depth


def _channels_last_view(t):
    """t with channels_last strides: a view for a contiguous one-channel map (its bytes are the
    same in both layouts), otherwise the layout conversion."""
    if t.dim() == 4 and t.shape[1] == 1 and t.is_contiguous():
        _, _, h, w = t.shape
        return t.as_strided(t.shape, (h * w, 1, w, 1))
    return t.contiguous(memory_format=torch.channels_last)


def merge_cat(parts):
    """torch.cat(parts, 1) of a decoder stage (PackNet01.py / PackNetSAN01.py `_merge`).  Under
    autocast the reference's cat promotes the bf16 features and the fp32 disparity map to an fp32
    tensor that the next (autocast) convolution casts straight back to bf16, and the mixed layouts
    made it NCHW (two more full-size copies before the channels_last convolution).  Casting the
    parts to the autocast dtype first gives that convolution the identical bf16 input (the bf16
    parts round-trip exactly, the disparity is rounded once either way) and the same gradients, and
    with every part channels_last the cat is written in the layout the convolution reads."""
    if len(parts) == 1:
        return parts[0]
    x0 = parts[0]
    if (x0.is_cuda and x0.dim() == 4 and torch.is_autocast_enabled("cuda")
            and x0.dtype == torch.get_autocast_dtype("cuda")
            and x0.is_contiguous(memory_format=torch.channels_last)):
        return torch.cat([_channels_last_view(p.to(x0.dtype)) for p in parts], 1)
    return torch.cat(parts, 1)


def packing(x, r=2):
    """[B,C,H,W] -> [B,C*r*r,H/r,W/r]; channel index = c*r*r + dy*r + dx (inverse of PixelShuffle)."""
    b, c, h, w = x.shape
    x = x.contiguous().view(b, c, h // r, r, w // r, r)
    return x.permute(0, 1, 3, 5, 2, 4).reshape(b, c * r * r, h // r, w // r)


class PackLayerConv2d(nn.Module):
    def __init__(self, in_channels, kernel_size, r=2):
        super().__init__()
        self.conv = Conv2D(in_channels * (r ** 2), in_channels, kernel_size, 1)
        self.pack = partial(packing, r=r)

    def forward(self, x):
        return self.conv(self.pack(x))


class UnpackLayerConv2d(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, r=2):
        super().__init__()
        self.conv = Conv2D(in_channels, out_channels * (r ** 2), kernel_size, 1)
        self.unpack = nn.PixelShuffle(r)

    def forward(self, x):
        return self.unpack(self.conv(x))


def _conv3d_d(d):
    return nn.Conv3d(1, d, kernel_size=(3, 3, 3), stride=(1, 1, 1), padding=(1, 1, 1))


class PackLayerConv3d(nn.Module):
    """pack -> Conv3d(1->d) over (channel, y, x) -> fold d into channels -> Conv2D.

    On a ROCm device in bf16 (autocast or bf16 input) the whole chain up to the Conv2d runs as the
    composed (k+2) x (k+2) convolution over the packed channels (packconv.py,
    include/psfm_packconv.h): the d*4C-channel packed volume is never written; the Conv2d bias,
    GroupNorm and ELU follow in the fused psfm_gn_act as before."""

    def __init__(self, in_channels, kernel_size, r=2, d=8):
        super().__init__()
        self.conv = Conv2D(in_channels * (r ** 2) * d, in_channels, kernel_size, 1)
        self.pack = partial(packing, r=r)
        self.conv3d = _conv3d_d(d)
        self.r = r
        self.in_channels = in_channels

    def _composed(self, x):
        c3 = self.conv3d
        return (self.r == 2 and x.is_cuda and x.dim() == 4 and x.shape[1] == self.in_channels
                and (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16
                     or not torch.is_autocast_enabled("cuda") and x.dtype == torch.bfloat16)
                and c3.in_channels == 1 and tuple(c3.kernel_size) == (3, 3, 3) and tuple(c3.padding) == (1, 1, 1)
                and tuple(c3.stride) == (1, 1, 1) and self.conv.conv_base.stride == (1, 1)
                and packconv.supported(x, self.in_channels, self.conv.kernel_size, c3.out_channels)
                and packconv.beneficial(x, self.in_channels))

    def forward(self, x):
        if self._composed(x):
            c = self.conv
            y = packconv.pack_conv2d(x, self.conv3d, c.conv_base, c.kernel_size)
            return gn_act(y, c.conv_base.bias, c.normalize, act=ACT_ELU)
        return self.conv(pack_conv3d(x, self.conv3d, self.r, self.pack))


class UnpackLayerConv3d(nn.Module):
    """Conv2D -> Conv3d(1->d) -> fold -> PixelShuffle."""

    def __init__(self, in_channels, out_channels, kernel_size, r=2, d=8):
        super().__init__()
        self.conv = Conv2D(in_channels, out_channels * (r ** 2) // d, kernel_size, 1)
        self.unpack = nn.PixelShuffle(r)
        self.conv3d = _conv3d_d(d)
        self.r = r

    def forward(self, x):
        return conv3d_unpack(self.conv(x), self.conv3d, self.r, self.unpack)
