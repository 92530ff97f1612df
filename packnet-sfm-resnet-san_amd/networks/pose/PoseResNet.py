"""PoseResNet (packnet_sfm/networks/pose/PoseResNet.py:11-47): 6-channel ResNet encoder per
(target, context) pair + PoseDecoder -> [B,N,6] = (translation, axis-angle)."""
import torch
import torch.nn as nn

from ..layers.resnet.pose_decoder import PoseDecoder
from ..layers.resnet.resnet_encoder import ResnetEncoder


class PoseResNet(nn.Module):
    def __init__(self, version=None, **kwargs):
        super().__init__()
        assert version is not None, "PoseResNet needs a version"
        num_layers, pretrained = int(version[:2]), version[2:] == "pt"
        assert num_layers in [18, 34, 50], "ResNet version {} not available".format(num_layers)
        self.encoder = ResnetEncoder(num_layers=num_layers, pretrained=pretrained, num_input_images=2)
        self.decoder = PoseDecoder(self.encoder.num_ch_enc, num_input_features=1, num_frames_to_predict_for=2)

    def forward(self, target_image, ref_imgs):
        outs = []
        for ref in ref_imgs:
            axisangle, translation = self.decoder([self.encoder(torch.cat([target_image, ref], 1))])
            outs.append(torch.cat([translation[:, 0], axisangle[:, 0]], 2))
        return torch.cat(outs, 1)
