"""Image helpers with the reference API (packnet_sfm/utils/image.py:85-282):
`gradient_x/y`, `interpolate_image`, `interpolate_scales`, `match_scales`, `meshgrid`,
`image_grid`, `flip_lr`."""
from collections.abc import Sequence
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


class _UpsampleNearest(torch.autograd.Function):
    """Nearest upsampling by an integer factor f — the same values as F.interpolate(mode='nearest')
    for an exact multiple — with a deterministic backward: each f x f block of the gradient is
    summed by a reshape + sum reduction (fp32 accumulation, fixed order).  ATen's
    upsample_nearest2d_backward accumulates with atomics; in bf16 every add rounds, which made the
    bf16 training step's gradients differ by ~5 % between identical runs (tools/diag_cycles.py)."""

    @staticmethod
    def forward(ctx, x, f):
        ctx.f = f
        return funct.interpolate(x, scale_factor=f, mode="nearest")

    @staticmethod
    def backward(ctx, g):
        f = ctx.f
        B, C, H, W = g.shape
        return g.reshape(B, C, H // f, f, W // f, f).sum((3, 5)), None


def upsample_nearest(x, factor=2):
    """x [B,C,H,W] -> [B,C,fH,fW] nearest, deterministic backward (see _UpsampleNearest)."""
    return x if factor == 1 else _UpsampleNearest.apply(x, int(factor))


class UpsampleNearest(torch.nn.Module):
    """nn.Upsample(scale_factor=f, mode='nearest') with the deterministic backward (no parameters:
    state dicts unchanged)."""

    def __init__(self, scale_factor=2):
        super().__init__()
        self.scale_factor = int(scale_factor)

    def forward(self, x):
        return upsample_nearest(x, self.scale_factor)


class NearestScales(Sequence):
    """Inverse-depth scales nearest-upsampled to one size (`upsample_output(mode='nearest')`,
    models/model_utils.py:152-196) WITHOUT materialising the upsampled maps.

    The photometric loss reads the stored maps through the 2^k index mapping
    (psfm_params.sig_shift, include/psfm.h) and returns their gradient at the stored size, so
    the training step never writes the 4 full-resolution copies nor runs their backward
    reductions.  Indexing / iterating yields the upsampled tensors (differentiable, deterministic
    backward), so callers that read `output['inv_depths'][i]` see the reference's values."""

    def __init__(self, stored, shape):
        self.stored = list(stored)
        self.shape = tuple(shape[-2:])
        self.shifts = []
        for t in self.stored:
            f = self.shape[0] // t.shape[-2]
            k = f.bit_length() - 1
            if f != (1 << k) or t.shape[-2] * f != self.shape[0] or t.shape[-1] * f != self.shape[1]:
                raise ValueError(f"NearestScales: {tuple(t.shape[-2:])} -> {self.shape} is not a 2^k upsampling")
            self.shifts.append(k)

    @staticmethod
    def exact(images, shape):
        """True when every image reaches `shape` by an exact power-of-two factor."""
        for t in images:
            f = shape[0] // t.shape[-2]
            if f < 1 or f & (f - 1) or t.shape[-2] * f != shape[0] or t.shape[-1] * f != shape[1]:
                return False
        return True

    def __len__(self):
        return len(self.stored)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return NearestScales(self.stored[i], self.shape)
        return upsample_nearest(self.stored[i], 1 << self.shifts[i])

    def materialize(self):
        return [self[i] for i in range(len(self))]


def interpolate_scales(images, shape=None, mode="bilinear", align_corners=False):
    shape = tuple((images[0].shape if shape is None else shape)[-2:])
    out = []
    for im in images:
        h, w = im.shape[-2:]
        f = shape[0] // h
        if mode == "nearest" and f * h == shape[0] and f * w == shape[1]:
            out.append(upsample_nearest(im, f))   # exact integer factor: deterministic backward
        else:
            out.append(funct.interpolate(im, shape, mode=mode, align_corners=align_corners))
    return out


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
