"""PackNet01 (packnet_sfm/networks/depth/PackNet01.py:8-185): 3D packing encoder / unpacking
decoder with inverse-depth heads at 4 scales.  Versions '1A' (skip concatenation) and '1B'
(skip addition).  Module names follow the reference (checkpoint compatible)."""
import torch
import torch.nn as nn

from ...utils.image import UpsampleNearest
from ..layers.packnet.layers01 import (Conv2D, InvDepth, PackLayerConv3d, ResidualBlock,
                                       UnpackLayerConv3d, merge_cat)


class PackNet01(nn.Module):
    def __init__(self, dropout=None, version=None, **kwargs):
        super().__init__()
        self.version = version[1:]
        ni, no = 64, 1
        n1, n2, n3, n4, n5 = 64, 64, 128, 256, 512
        num_blocks = [2, 2, 3, 3]
        pack_k, unpack_k, iconv_k = [5, 3, 3, 3, 3], [3] * 5, [3] * 5
        if self.version == "A":      # concatenation of skips
            ins = {1: n1 + ni + no, 2: n2 + n1 + no, 3: n3 + n2 + no, 4: n4 + n3, 5: n5 + n4}
            outs = {1: n1, 2: n2, 3: n3, 4: n4, 5: n5}
        elif self.version == "B":    # addition of skips
            ins = {1: n1 + no, 2: n2 + no, 3: n3 // 2 + no, 4: n4 // 2, 5: n5 // 2}
            outs = {1: n1, 2: n2, 3: n3 // 2, 4: n4 // 2, 5: n5 // 2}
        else:
            raise ValueError("Unknown PackNet version {}".format(version))

        self.pre_calc = Conv2D(3, ni, 5, 1)
        # construction order matters only for RNG-drawn init; kept as in the reference
        self.pack1 = PackLayerConv3d(n1, pack_k[0])
        self.pack2 = PackLayerConv3d(n2, pack_k[1])
        self.pack3 = PackLayerConv3d(n3, pack_k[2])
        self.pack4 = PackLayerConv3d(n4, pack_k[3])
        self.pack5 = PackLayerConv3d(n5, pack_k[4])
        self.conv1 = Conv2D(ni, n1, 7, 1)
        self.conv2 = ResidualBlock(n1, n2, num_blocks[0], 1, dropout=dropout)
        self.conv3 = ResidualBlock(n2, n3, num_blocks[1], 1, dropout=dropout)
        self.conv4 = ResidualBlock(n3, n4, num_blocks[2], 1, dropout=dropout)
        self.conv5 = ResidualBlock(n4, n5, num_blocks[3], 1, dropout=dropout)
        self.unpack5 = UnpackLayerConv3d(n5, outs[5], unpack_k[0])
        self.unpack4 = UnpackLayerConv3d(n5, outs[4], unpack_k[1])
        self.unpack3 = UnpackLayerConv3d(n4, outs[3], unpack_k[2])
        self.unpack2 = UnpackLayerConv3d(n3, outs[2], unpack_k[3])
        self.unpack1 = UnpackLayerConv3d(n2, outs[1], unpack_k[4])
        self.iconv5 = Conv2D(ins[5], n5, iconv_k[0], 1)
        self.iconv4 = Conv2D(ins[4], n4, iconv_k[1], 1)
        self.iconv3 = Conv2D(ins[3], n3, iconv_k[2], 1)
        self.iconv2 = Conv2D(ins[2], n2, iconv_k[3], 1)
        self.iconv1 = Conv2D(ins[1], n1, iconv_k[4], 1)
        self.unpack_disps = nn.PixelShuffle(2)
        self.unpack_disp4 = UpsampleNearest(2)
        self.unpack_disp3 = UpsampleNearest(2)
        self.unpack_disp2 = UpsampleNearest(2)
        self.disp4_layer = InvDepth(n4, out_channels=no)
        self.disp3_layer = InvDepth(n3, out_channels=no)
        self.disp2_layer = InvDepth(n2, out_channels=no)
        self.disp1_layer = InvDepth(n1, out_channels=no)
        self.init_weights()

    def init_weights(self):
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Conv3d)):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    m.bias.data.zero_()

    def _merge(self, unpacked, skip, disp=None):
        if self.version == "A":
            parts = [unpacked, skip]
        else:
            parts = [unpacked + skip]
        if disp is not None:
            parts.append(disp)
        return merge_cat(parts)

    def forward(self, rgb):
        x = self.pre_calc(rgb)
        x1 = self.conv1(x)
        x1p = self.pack1(x1)
        x2p = self.pack2(self.conv2(x1p))
        x3p = self.pack3(self.conv3(x2p))
        x4p = self.pack4(self.conv4(x3p))
        x5p = self.pack5(self.conv5(x4p))

        iconv5 = self.iconv5(self._merge(self.unpack5(x5p), x4p))
        iconv4 = self.iconv4(self._merge(self.unpack4(iconv5), x3p))
        disp4 = self.disp4_layer(iconv4)
        iconv3 = self.iconv3(self._merge(self.unpack3(iconv4), x2p, self.unpack_disp4(disp4)))
        disp3 = self.disp3_layer(iconv3)
        iconv2 = self.iconv2(self._merge(self.unpack2(iconv3), x1p, self.unpack_disp3(disp3)))
        disp2 = self.disp2_layer(iconv2)
        iconv1 = self.iconv1(self._merge(self.unpack1(iconv2), x, self.unpack_disp2(disp2)))
        disp1 = self.disp1_layer(iconv1)
        if self.training:
            return {"inv_depths": [disp1, disp2, disp3, disp4]}
        return {"inv_depths": disp1}
