"""ResNetSAN01 (packnet_sfm/networks/depth/ResNetSAN01.py:13-355), RGB path.

ResNet encoder + DepthDecoder returning SIGMOID maps at 4 scales in training (the fork's
"sigmoid outputs, post-processed later" contract, :285-305) and 1 scale in eval.  The sparse
LiDAR branch (MinkowskiEngine encoder + FiLM fusion) is out of scope (needs
`input_depth` and a C++/CUDA sparse-conv library): passing `input_depth` raises.
The learnable fusion `weight`/`bias` parameters exist for checkpoint compatibility.
"""
import torch
import torch.nn as nn

from ..layers.resnet.depth_decoder import DepthDecoder
from ..layers.resnet.resnet_encoder import ResnetEncoder


class ResNetSAN01(nn.Module):
    def __init__(self, dropout=None, version=None, use_film=False, film_scales=[0], use_enhanced_lidar=False,
                 use_dual_head=False, min_depth=0.5, max_depth=80.0, **kwargs):
        super().__init__()
        if max_depth <= 0:
            max_depth = 80.0
        if min_depth <= 0:
            min_depth = 0.5
        if max_depth <= min_depth:
            max_depth = min_depth + 1.0
        self.min_depth, self.max_depth = float(min_depth), float(max_depth)
        if use_film or use_dual_head:
            raise NotImplementedError("ResNetSAN01 LiDAR/FiLM and dual-head variants are out of scope "
                                      "(SURVEY.md §2.1)")
        self.use_dual_head = self.is_dual_head = False
        num_layers = int(version[:2]) if version else 18
        self.variant = (version[2:] or "A") if version else "A"
        self.encoder = ResnetEncoder(num_layers=num_layers, pretrained=True)
        self.decoder = DepthDecoder(num_ch_enc=self.encoder.num_ch_enc)
        self.use_film, self.film_scales, self.use_enhanced_lidar = use_film, film_scales, use_enhanced_lidar
        self.mconvs = None
        self.weight = nn.Parameter(torch.ones(5) * 0.5, requires_grad=True)
        self.bias = nn.Parameter(torch.zeros(5), requires_grad=True)
        self.init_weights()

    def init_weights(self):
        """Xavier for everything but the encoder (kept at its own init, as the reference)."""
        for name, m in self.named_modules():
            if name.startswith("encoder"):
                continue
            if isinstance(m, (nn.Conv2d, nn.Conv3d)):
                nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    m.bias.data.zero_()

    def run_network(self, rgb, input_depth=None):
        if input_depth is not None:
            raise NotImplementedError("sparse LiDAR input (SAN branch) is out of scope")
        skips = self.encoder(rgb)
        out = self.decoder(skips)
        n = 4 if self.training else 1
        return [out[("disp", i)] for i in range(n)], skips

    def forward(self, rgb, input_depth=None, **kwargs):
        sig, _ = self.run_network(rgb, input_depth)
        return {"inv_depths": sig}
