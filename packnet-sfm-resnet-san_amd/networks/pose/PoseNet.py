"""PoseNet (packnet_sfm/networks/pose/PoseNet.py:38-84): 7 stride-2 conv+GroupNorm+ReLU
blocks over [target, contexts] stacked on channels, 1x1 head, spatial mean, x0.01 -> [B,N,6]."""
import torch
import torch.nn as nn

from ..layers.fused import cat_input, conv_nobias, gn_act


def conv_gn(in_planes, out_planes, kernel_size=3):
    return nn.Sequential(
        nn.Conv2d(in_planes, out_planes, kernel_size=kernel_size, padding=(kernel_size - 1) // 2, stride=2),
        nn.GroupNorm(16, out_planes),
        nn.ReLU(inplace=True))


class PoseNet(nn.Module):
    def __init__(self, nb_ref_imgs=2, rotation_mode="euler", **kwargs):
        super().__init__()
        self.nb_ref_imgs = nb_ref_imgs
        self.rotation_mode = rotation_mode
        ch = [16, 32, 64, 128, 256, 256, 256]
        ks = [7, 5, 3, 3, 3, 3, 3]
        ins = [3 * (1 + nb_ref_imgs)] + ch[:-1]
        for i in range(7):
            setattr(self, f"conv{i + 1}", conv_gn(ins[i], ch[i], kernel_size=ks[i]))
        self.pose_pred = nn.Conv2d(ch[-1], 6 * nb_ref_imgs, kernel_size=1, padding=0)
        self.init_weights()

    def init_weights(self):
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
                nn.init.xavier_uniform_(m.weight.data)
                if m.bias is not None:
                    m.bias.data.zero_()

    def forward(self, image, context):
        assert len(context) == self.nb_ref_imgs
        x = cat_input([image, *context])   # under bf16 autocast: the bf16 concatenation in one pass
        for i in range(7):  # conv -> (bias + GroupNorm + ReLU) fused epilogue (fused.py)
            conv, gn, _ = getattr(self, f"conv{i + 1}")
            x = gn_act(conv_nobias(conv, x), conv.bias, gn, relu=True)
        pose = self.pose_pred(x).mean(3).mean(2)
        return 0.01 * pose.view(pose.size(0), self.nb_ref_imgs, 6)
