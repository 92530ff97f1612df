"""DepthResNet (packnet_sfm/networks/depth/DepthResNet.py:12-54): ResNet encoder + DepthDecoder,
disparity scaled to inverse depth in [1/100, 1/0.1]."""
from functools import partial

import torch.nn as nn

from ..layers.resnet.depth_decoder import DepthDecoder
from ..layers.resnet.layers import disp_to_depth
from ..layers.resnet.resnet_encoder import ResnetEncoder


class DepthResNet(nn.Module):
    def __init__(self, version=None, **kwargs):
        super().__init__()
        assert version is not None, "DispResNet needs a version"
        num_layers, pretrained = int(version[:2]), version[2:] == "pt"
        assert num_layers in [18, 34, 50], "ResNet version {} not available".format(num_layers)
        self.encoder = ResnetEncoder(num_layers=num_layers, pretrained=pretrained)
        self.decoder = DepthDecoder(num_ch_enc=self.encoder.num_ch_enc)
        self.scale_inv_depth = partial(disp_to_depth, min_depth=0.1, max_depth=100.0)

    def forward(self, rgb):
        x = self.decoder(self.encoder(rgb))
        inv = [self.scale_inv_depth(x[("disp", i)])[0] for i in range(4)]
        return {"inv_depths": inv if self.training else inv[0]}
