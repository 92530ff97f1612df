"""PackNetSAN01 (packnet_sfm/networks/depth/PackNetSAN01.py:11-235) — the depth net of BASELINE
configs 3 and 5 (configs/train_packnet_san_kitti.yaml:19-21, train_packnet_san_ddad.yaml:19-22):
a PackNet encoder / decoder with ni = n1 = 32 and 4 three-dimensional features per packing layer
(num_3d_feat = 4, :165-170), inverse-depth heads at 4 scales.

RGB path only.  The SAN branch (`input_depth`) runs a MinkowskiEngine sparse encoder on LiDAR
(`self.mconvs`, :175, :190-203) — MinkowskiEngine is not in this image and that branch is off the
self-supervised photometric path (OUT OF SCOPE), so `input_depth` raises.  The
fusion parameters `weight` / `bias` [5] are kept (unused on the RGB path, as in the reference:
they get no gradient) so parameter names and counts match; a reference checkpoint loads with
`load_state_dict(strict=False)` minus its `mconvs.*` entries.

Module names follow the reference (`encoder.*`, `decoder.*`).  The pack / unpack 3-D
convolutions run on the fused HIP kernels (layers01.PackLayerConv3d / UnpackLayerConv3d, d = 4).
"""
import torch
import torch.nn as nn

from ...utils.image import UpsampleNearest
from ..layers.packnet.layers01 import (Conv2D, InvDepth, PackLayerConv3d, ResidualBlock,
                                       UnpackLayerConv3d, merge_cat)


class Encoder(nn.Module):
    """PackNetSAN01.py:11-50."""

    def __init__(self, version, in_channels, ni, n1, n2, n3, n4, n5, pack_kernel, num_blocks, num_3d_feat,
                 dropout):
        super().__init__()
        self.version = version
        self.pre_calc = Conv2D(in_channels, ni, 5, 1)
        self.pack1 = PackLayerConv3d(n1, pack_kernel[0], d=num_3d_feat)
        self.pack2 = PackLayerConv3d(n2, pack_kernel[1], d=num_3d_feat)
        self.pack3 = PackLayerConv3d(n3, pack_kernel[2], d=num_3d_feat)
        self.pack4 = PackLayerConv3d(n4, pack_kernel[3], d=num_3d_feat)
        self.pack5 = PackLayerConv3d(n5, pack_kernel[4], d=num_3d_feat)
        self.conv1 = Conv2D(ni, n1, 7, 1)
        self.conv2 = ResidualBlock(n1, n2, num_blocks[0], 1, dropout=dropout)
        self.conv3 = ResidualBlock(n2, n3, num_blocks[1], 1, dropout=dropout)
        self.conv4 = ResidualBlock(n3, n4, num_blocks[2], 1, dropout=dropout)
        self.conv5 = ResidualBlock(n4, n5, num_blocks[3], 1, dropout=dropout)

    def forward(self, rgb):
        x = self.pre_calc(rgb)
        x1p = self.pack1(self.conv1(x))
        x2p = self.pack2(self.conv2(x1p))
        x3p = self.pack3(self.conv3(x2p))
        x4p = self.pack4(self.conv4(x3p))
        x5p = self.pack5(self.conv5(x4p))
        return x5p, [x, x1p, x2p, x3p, x4p]


class Decoder(nn.Module):
    """PackNetSAN01.py:53-140.  Version 'A' concatenates the skips, 'B' adds them."""

    def __init__(self, version, out_channels, ni, n1, n2, n3, n4, n5, unpack_kernel, iconv_kernel, num_3d_feat):
        super().__init__()
        self.version = version
        n1i, n2i, n3i = n1 + ni + out_channels, n2 + n1 + out_channels, n3 + n2 + out_channels
        n4i, n5i = n4 + n3, n5 + n4
        self.unpack5 = UnpackLayerConv3d(n5, n5, unpack_kernel[0], d=num_3d_feat)
        self.unpack4 = UnpackLayerConv3d(n5, n4, unpack_kernel[1], d=num_3d_feat)
        self.unpack3 = UnpackLayerConv3d(n4, n3, unpack_kernel[2], d=num_3d_feat)
        self.unpack2 = UnpackLayerConv3d(n3, n2, unpack_kernel[3], d=num_3d_feat)
        self.unpack1 = UnpackLayerConv3d(n2, n1, unpack_kernel[4], d=num_3d_feat)
        self.iconv5 = Conv2D(n5i, n5, iconv_kernel[0], 1)
        self.iconv4 = Conv2D(n4i, n4, iconv_kernel[1], 1)
        self.iconv3 = Conv2D(n3i, n3, iconv_kernel[2], 1)
        self.iconv2 = Conv2D(n2i, n2, iconv_kernel[3], 1)
        self.iconv1 = Conv2D(n1i, n1, iconv_kernel[4], 1)
        self.unpack_disps = nn.PixelShuffle(2)
        self.unpack_disp4 = UpsampleNearest(2)
        self.unpack_disp3 = UpsampleNearest(2)
        self.unpack_disp2 = UpsampleNearest(2)
        self.disp4_layer = InvDepth(n4, out_channels=out_channels)
        self.disp3_layer = InvDepth(n3, out_channels=out_channels)
        self.disp2_layer = InvDepth(n2, out_channels=out_channels)
        self.disp1_layer = InvDepth(n1, out_channels=out_channels)

    def _merge(self, unpacked, skip, disp=None):
        if self.version == "A":
            parts = [unpacked, skip]
        else:
            parts = [unpacked + skip]
        if disp is not None:
            parts.append(disp)
        return merge_cat(parts)

    def forward(self, x5p, skips):
        skip1, skip2, skip3, skip4, skip5 = skips
        iconv5 = self.iconv5(self._merge(self.unpack5(x5p), skip5))
        iconv4 = self.iconv4(self._merge(self.unpack4(iconv5), skip4))
        inv_depth4 = self.disp4_layer(iconv4)
        iconv3 = self.iconv3(self._merge(self.unpack3(iconv4), skip3, self.unpack_disp4(inv_depth4)))
        inv_depth3 = self.disp3_layer(iconv3)
        iconv2 = self.iconv2(self._merge(self.unpack2(iconv3), skip2, self.unpack_disp3(inv_depth3)))
        inv_depth2 = self.disp2_layer(iconv2)
        iconv1 = self.iconv1(self._merge(self.unpack1(iconv2), skip1, self.unpack_disp2(inv_depth2)))
        inv_depth1 = self.disp1_layer(iconv1)
        if self.training:
            return [inv_depth1, inv_depth2, inv_depth3, inv_depth4]
        return [inv_depth1]


class PackNetSAN01(nn.Module):
    """PackNetSAN01.py:143-235 (RGB path)."""

    def __init__(self, dropout=None, version=None, **kwargs):
        super().__init__()
        self.version = version[1:]
        in_channels, out_channels = 3, 1
        ni, n1, n2, n3, n4, n5 = 32, 32, 64, 128, 256, 512
        num_blocks = [2, 2, 3, 3]
        pack_kernel, unpack_kernel, iconv_kernel = [5, 3, 3, 3, 3], [3] * 5, [3] * 5
        num_3d_feat = 4
        self.encoder = Encoder(self.version, in_channels, ni, n1, n2, n3, n4, n5, pack_kernel, num_blocks,
                               num_3d_feat, dropout)
        self.decoder = Decoder(self.version, out_channels, ni, n1, n2, n3, n4, n5, unpack_kernel, iconv_kernel,
                               num_3d_feat)
        self.mconvs = None   # MinkowskiEncoder (SAN LiDAR branch): out of scope, see module docstring
        self.weight = nn.Parameter(torch.ones(5), requires_grad=True)
        self.bias = nn.Parameter(torch.zeros(5), requires_grad=True)
        self.init_weights()

    def init_weights(self):
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Conv3d)):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    m.bias.data.zero_()

    def run_network(self, rgb, input_depth=None):
        if input_depth is not None:
            raise NotImplementedError("PackNetSAN01 LiDAR (SAN) branch needs MinkowskiEngine: out of scope "
                                      "(SURVEY.md §2); the self-supervised step uses the RGB path")
        x5p, skips = self.encoder(rgb)
        return self.decoder(x5p, skips), skips + [x5p]

    def forward(self, rgb, input_depth=None, **kwargs):
        inv_depths, _ = self.run_network(rgb, input_depth)
        return {"inv_depths": inv_depths}
