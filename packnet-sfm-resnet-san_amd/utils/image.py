"""Image helpers with the reference API (packnet_sfm/utils/image.py:85-282):
`gradient_x/y`, `interpolate_image`, `interpolate_scales`, `match_scales`, `meshgrid`,
`image_grid`, `flip_lr`."""
from functools import lru_cache

import torch
import torch.nn.functional as funct


def flip_lr(image):
    assert image.dim() == 4, "You need to provide a [B,C,H,W] image to flip"
    return torch.flip(image, [3])


def gradient_x(image):
    return image[:, :, :, :-1] - image[:, :, :, 1:]


def gradient_y(image):
    return image[:, :, :-1, :] - image[:, :, 1:, :]


def same_shape(a, b):
    return tuple(a[-2:]) == tuple(b[-2:])


def interpolate_image(image, shape, mode="bilinear", align_corners=True):
    shape = tuple(shape[-2:])
    if same_shape(image.shape, shape):
        return image
    return funct.interpolate(image, size=shape, mode=mode, align_corners=align_corners)


def interpolate_scales(images, shape=None, mode="bilinear", align_corners=False):
    shape = tuple((images[0].shape if shape is None else shape)[-2:])
    return [funct.interpolate(im, shape, mode=mode, align_corners=align_corners) for im in images]


def match_scales(image, targets, num_scales, mode="bilinear", align_corners=True):
    return [image if same_shape(image.shape, targets[i].shape)
            else interpolate_image(image, targets[i].shape, mode=mode, align_corners=align_corners)
            for i in range(num_scales)]


@lru_cache(maxsize=None)
def meshgrid(B, H, W, dtype, device, normalized=False):
    if normalized:
        xs = torch.linspace(-1, 1, W, device=device, dtype=dtype)
        ys = torch.linspace(-1, 1, H, device=device, dtype=dtype)
    else:
        xs = torch.linspace(0, W - 1, W, device=device, dtype=dtype)
        ys = torch.linspace(0, H - 1, H, device=device, dtype=dtype)
    ys, xs = torch.meshgrid([ys, xs], indexing="ij")
    return xs.repeat([B, 1, 1]), ys.repeat([B, 1, 1])


@lru_cache(maxsize=None)
def image_grid(B, H, W, dtype, device, normalized=False):
    xs, ys = meshgrid(B, H, W, dtype, device, normalized=normalized)
    return torch.stack([xs, ys, torch.ones_like(xs)], dim=1)
