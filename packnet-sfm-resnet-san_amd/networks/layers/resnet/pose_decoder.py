"""PoseDecoder (packnet_sfm/networks/layers/resnet/pose_decoder.py:13-53)."""
from collections import OrderedDict

import torch
import torch.nn as nn


class PoseDecoder(nn.Module):
    def __init__(self, num_ch_enc, num_input_features, num_frames_to_predict_for=None, stride=1):
        super().__init__()
        self.num_ch_enc = num_ch_enc
        self.num_input_features = num_input_features
        self.num_frames_to_predict_for = (num_input_features - 1 if num_frames_to_predict_for is None
                                          else num_frames_to_predict_for)
        self.convs = OrderedDict()
        self.convs["squeeze"] = nn.Conv2d(self.num_ch_enc[-1], 256, 1)
        self.convs[("pose", 0)] = nn.Conv2d(num_input_features * 256, 256, 3, stride, 1)
        self.convs[("pose", 1)] = nn.Conv2d(256, 256, 3, stride, 1)
        self.convs[("pose", 2)] = nn.Conv2d(256, 6 * self.num_frames_to_predict_for, 1)
        self.relu = nn.ReLU()
        self.net = nn.ModuleList(list(self.convs.values()))

    def forward(self, input_features):
        x = torch.cat([self.relu(self.convs["squeeze"](f[-1])) for f in input_features], 1)
        for i in range(3):
            x = self.convs[("pose", i)](x)
            if i != 2:
                x = self.relu(x)
        x = 0.01 * x.mean(3).mean(2).view(-1, self.num_frames_to_predict_for, 1, 6)
        return x[..., :3], x[..., 3:]
