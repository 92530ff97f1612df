"""ResNet encoder (packnet_sfm/networks/layers/resnet/resnet_encoder.py:16-98).

The reference builds it from torchvision (`models.resnet18/34/50/...` plus an ImageNet
download).  torchvision is not part of this stack, so the ResNet trunk is defined here with
torchvision's module/parameter names (`conv1`, `bn1`, `layerK.i.{conv1,bn1,conv2,bn2,[conv3,bn3],
downsample.0/1}`) — torchvision / reference checkpoints load into it unchanged.  No pretrained
download (offline); `pretrained=True` only changes nothing but is accepted for API parity.
"""
import numpy as np
import torch
import torch.nn as nn

from ..fused import bn_act, bn_relu_maxpool, normalize_input


def conv3x3(i, o, stride=1):
    return nn.Conv2d(i, o, kernel_size=3, stride=stride, padding=1, bias=False)


def conv1x1(i, o, stride=1):
    return nn.Conv2d(i, o, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample

    def forward(self, x, x_idt=None, nout=1):
        """conv -> BN -> ReLU, conv -> BN -> +identity -> ReLU as fused BN epilogues (fused.py).
        x_idt: the identity / downsample input — x's values as the producer's other forked view, so
        that both gradients reach the producer's backward (fused._fork); nout: forked outputs."""
        x_idt = x if x_idt is None else x_idt
        idt = x_idt if self.downsample is None else bn_act(self.downsample[0](x_idt), self.downsample[1], relu=False)
        out = bn_act(self.conv1(x), self.bn1, relu=True)
        return bn_act(self.conv2(out), self.bn2, relu=True, residual=idt, nout=nout)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = conv1x1(inplanes, planes)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = conv3x3(planes, planes, stride)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = conv1x1(planes, planes * 4)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x, x_idt=None, nout=1):
        x_idt = x if x_idt is None else x_idt
        idt = x_idt if self.downsample is None else bn_act(self.downsample[0](x_idt), self.downsample[1], relu=False)
        out = bn_act(self.conv1(x), self.bn1, relu=True)
        out = bn_act(self.conv2(out), self.bn2, relu=True)
        return bn_act(self.conv3(out), self.bn3, relu=True, residual=idt, nout=nout)


RESNET_SPECS = {18: (BasicBlock, [2, 2, 2, 2]), 34: (BasicBlock, [3, 4, 6, 3]),
                50: (Bottleneck, [3, 4, 6, 3]), 101: (Bottleneck, [3, 4, 23, 3]),
                152: (Bottleneck, [3, 8, 36, 3])}


class ResNet(nn.Module):
    """torchvision-layout ResNet trunk (no fc head is used by the encoder)."""

    def __init__(self, block, layers, num_input_images=1):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3 * num_input_images, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        down = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            down = nn.Sequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                 nn.BatchNorm2d(planes * block.expansion))
        mods = [block(self.inplanes, planes, stride, down)]
        self.inplanes = planes * block.expansion
        mods += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)


def resnet_multiimage_input(num_layers, pretrained=False, num_input_images=1):
    block, layers = RESNET_SPECS[num_layers]
    return ResNet(block, layers, num_input_images=num_input_images)


class ResnetEncoder(nn.Module):
    """Multi-scale features [relu(bn1), layer1..4] of a ResNet on (x-0.45)/0.225."""

    def __init__(self, num_layers, pretrained, num_input_images=1):
        super().__init__()
        if num_layers not in RESNET_SPECS:
            raise ValueError("{} is not a valid number of resnet layers".format(num_layers))
        self.num_ch_enc = np.array([64, 64, 128, 256, 512])
        self.encoder = resnet_multiimage_input(num_layers, pretrained, num_input_images)
        if num_layers > 34:
            self.num_ch_enc[1:] *= 4

    def forward(self, input_image):
        """[relu(bn1(conv1)), layer1..4] as the reference (resnet_encoder.py:89-98).  Every tensor with
        several consumers is produced forked (fused._fork): the stem output (maxpool, decoder skip), a
        block output inside a layer (next block's conv1 and identity) and a layer output (next layer's
        conv1 and downsample, decoder skip) — their gradients are summed by the producer's backward
        kernel, not by autograd's bf16 add kernels.  The stem's ReLU + max-pool is one HIP pass each way
        (fused.bn_relu_maxpool), its pooled output forked for layer1's first block (conv1, identity)."""
        e = self.encoder
        skip, *h = bn_relu_maxpool(e.conv1(normalize_input(input_image, 0.45, 0.225)), e.bn1, e.maxpool, nout=2)
        feats = [skip]
        layers = (e.layer1, e.layer2, e.layer3, e.layer4)
        for li, layer in enumerate(layers):
            blocks = list(layer)
            for bi, blk in enumerate(blocks):
                last = bi == len(blocks) - 1
                nout = (3 if li < len(layers) - 1 else 1) if last else 2
                outs = blk(h[0], h[1], nout=nout)
                outs = outs if isinstance(outs, tuple) else (outs,)
                h = outs[:2] if len(outs) > 1 else None
                if last:
                    feats.append(outs[-1])
        # not kept on the module (the reference stores self.features): a reference held between
        # steps keeps the previous step's encoder graph alive, and with it the AccumulateGrad nodes
        # of every encoder parameter — the next step (or HIP-graph capture) on another stream then
        # reuses nodes bound to the old stream (tools/diag_accgrad_nodes.py)
        return feats
