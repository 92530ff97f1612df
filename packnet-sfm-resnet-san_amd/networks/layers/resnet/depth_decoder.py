"""DepthDecoder (packnet_sfm/networks/layers/resnet/depth_decoder.py:16-64): 5 up-stages with
skips, sigmoid disparity heads at scales 0..3.  State-dict layout (`decoder.<k>...`) as in the
reference's OrderedDict -> ModuleList construction."""
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn

from ..fused import ACT_SIGMOID, bias_act, conv_block_up_cat, conv_nobias
from .layers import Conv3x3, ConvBlock


class DepthDecoder(nn.Module):
    def __init__(self, num_ch_enc, scales=range(4), num_output_channels=1, use_skips=True):
        super().__init__()
        self.num_output_channels = num_output_channels
        self.use_skips = use_skips
        self.upsample_mode = "nearest"
        self.scales = scales
        self.num_ch_enc = num_ch_enc
        self.num_ch_dec = np.array([16, 32, 64, 128, 256])
        self.convs = OrderedDict()
        for i in range(4, -1, -1):
            cin = self.num_ch_enc[-1] if i == 4 else self.num_ch_dec[i + 1]
            self.convs[("upconv", i, 0)] = ConvBlock(cin, self.num_ch_dec[i])
            cin = self.num_ch_dec[i] + (self.num_ch_enc[i - 1] if (use_skips and i > 0) else 0)
            self.convs[("upconv", i, 1)] = ConvBlock(cin, self.num_ch_dec[i])
        for s in self.scales:
            self.convs[("dispconv", s)] = Conv3x3(self.num_ch_dec[s], self.num_output_channels)
        self.decoder = nn.ModuleList(list(self.convs.values()))
        self.sigmoid = nn.Sigmoid()

    def forward(self, input_features):
        out = {}
        x = input_features[-1]
        for i in range(4, -1, -1):
            # cat([upsample(upconv_i0(x)), skip]) with upconv_i0's bias + ReLU folded in: one fused
            # op each way after the convolution (fused.conv_block_up_cat)
            skip = input_features[i - 1] if (self.use_skips and i > 0) else None
            # upconv_i1's output feeds the next up-stage and, at a head scale > 0, the disparity head:
            # forked (fused._fork), so the bias + ReLU backward sums the two gradients itself
            fork = i in self.scales and i > 0
            x = self.convs[("upconv", i, 1)](conv_block_up_cat(self.convs[("upconv", i, 0)], x, skip),
                                             nout=2 if fork else 1)
            x, xh = x if fork else (x, x)
            if i in self.scales:
                head = self.convs[("dispconv", i)]  # Conv3x3 + sigmoid, fused epilogue (fp32 maps)
                xin = head.pad(xh) if head.pad is not None else xh
                out[("disp", i)] = bias_act(conv_nobias(head.conv, xin), head.conv.bias, ACT_SIGMOID, head)
        # not kept on the module (the reference stores self.outputs): a reference held between steps
        # keeps the previous step's autograd graph alive, and with it its AccumulateGrad nodes
        return out
