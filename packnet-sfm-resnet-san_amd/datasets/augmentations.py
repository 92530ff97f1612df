"""Training-sample transforms on the GPU — the host data path of packnet_sfm/datasets
(SURVEY §8f row 2), batched.

The reference runs, per sample on CPU DataLoader workers, `train_transforms`
(datasets/transforms.py:21-50): `crop_sample` -> `resize_sample` (LANCZOS) ->
`duplicate_sample` -> `colorjitter_sample` -> `to_tensor_sample` on PIL images.  Here the
decoded uint8 images of a whole batch go to the device once (3 B/px) and one C-ABI call
(`psfm_train_augment`, include/psfm_augment.h) produces `rgb` / `rgb_original` (and the
context lists) as fp32 [B,3,H,W], bit-identical to Pillow's arithmetic.  The random draws stay
here, in Python's `random` and in the reference's order, so a seeded run reproduces the
reference's jitter factors sample by sample.

No CPU fallback: tensors must be on a ROCm device and the HIP library must be built.
"""
import ctypes
import random

import torch

from .. import _hip
from ..utils.misc import parse_crop_borders

JIT_BRIGHTNESS, JIT_CONTRAST, JIT_SATURATION, JIT_HUE = 0, 1, 2, 3


# ---------------------------------------------------------------------------------------------------------------------
# random draws (host, per sample)
# ---------------------------------------------------------------------------------------------------------------------
def random_color_jitter_params(parameters, prob=1.0, rng=random):
    """The fixed parameters of one sample's colour jitter, drawn exactly as
    colorjitter_sample + random_color_jitter_transform draw them (datasets/augmentations.py:
    295 prob test, :346-364 one uniform per op in the order brightness, contrast, saturation,
    hue, :368 shuffle of the four ops, :299-304 the optional colour-matrix diagonal).

    Returns a dict {apply, order, factors, hue_factor, hue_shift, matrix}.
    """
    out = dict(apply=False, order=[0, 1, 2, 3], factors=[1.0, 1.0, 1.0], hue_factor=0.0, hue_shift=0,
               matrix=None)
    if not rng.random() < prob:
        return out
    b, c, s, h = parameters[:4]
    bf = rng.uniform(max(0, 1 - b), 1 + b)
    cf = rng.uniform(max(0, 1 - c), 1 + c)
    sf = rng.uniform(max(0, 1 - s), 1 + s)
    hf = rng.uniform(-h, h)
    order = [JIT_BRIGHTNESS, JIT_CONTRAST, JIT_SATURATION, JIT_HUE]
    rng.shuffle(order)
    matrix = None
    if len(parameters) > 4 and parameters[4] > 0:
        m = parameters[4]
        matrix = [rng.uniform(1. - m, 1 + m) for _ in range(3)]
    # torchvision adjust_hue: np_h += np.array(hue_factor * 255).astype(np.uint8) (wraps mod 256)
    out.update(apply=True, order=order, factors=[bf, cf, sf], hue_factor=hf, hue_shift=int(hf * 255) & 255,
               matrix=matrix)
    return out


def jitter_record(params):
    """psfm_jitter from random_color_jitter_params (factors rounded to float32 like Image.blend)."""
    j = _hip.Jitter()
    j.apply = 1 if params["apply"] else 0
    for i in range(4):
        j.order[i] = params["order"][i]
    for i in range(3):
        j.factor[i] = params["factors"][i]
    j.hue_shift = params["hue_shift"]
    j.use_matrix = 0 if params["matrix"] is None else 1
    for i in range(3):
        j.matrix[i] = 0.0 if params["matrix"] is None else params["matrix"][i]
    return j


# ---------------------------------------------------------------------------------------------------------------------
# the batched transform
# ---------------------------------------------------------------------------------------------------------------------
class _Plans:
    """Device resample plans / workspaces, cached per geometry (one upload per image size)."""

    def __init__(self):
        self.plans, self.ws = {}, {}
        self.ring, self.ring_pos = [], 0

    def upload(self, raw, device):
        """Jitter records -> device without a host sync: a ring of pinned staging buffers, each
        reused only after its previous asynchronous copy has completed (event)."""
        n = len(raw)
        if not self.ring or self.ring[0][0].numel() < n:
            self.ring = [(torch.empty(max(n, 4096), dtype=torch.uint8).pin_memory(), None) for _ in range(8)]
        host, ev = self.ring[self.ring_pos]
        if ev is not None:
            ev.synchronize()
        host[:n].copy_(torch.frombuffer(raw, dtype=torch.uint8))
        dev = torch.empty(n, dtype=torch.uint8, device=device)
        dev.copy_(host[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        self.ring[self.ring_pos] = (host, ev)
        self.ring_pos = (self.ring_pos + 1) % len(self.ring)
        return dev

    def get(self, p, device):
        key = (p.crop_r - p.crop_l, p.crop_b - p.crop_t, p.out_h, p.out_w, device)
        if key not in self.plans:
            L = _hip.lib()
            n = L.psfm_augment_plan(ctypes.byref(p), None)
            if n < 0:
                _hip.check(int(n), "psfm_augment_plan")
            host = torch.empty(int(n), dtype=torch.int32)
            _hip.check(0 if L.psfm_augment_plan(ctypes.byref(p), ctypes.c_void_p(host.data_ptr())) == n else -1,
                       "psfm_augment_plan")
            self.plans[key] = host.to(device)
        nbytes = int(_hip.lib().psfm_augment_ws_bytes(ctypes.byref(p)))
        wkey = (device, nbytes)
        if wkey not in self.ws:
            self.ws = {wkey: torch.empty(nbytes, dtype=torch.uint8, device=device)}
        return self.plans[key], self.ws[wkey]


_PLANS = _Plans()


def augment_images(images, n_samples, box, shape, jitter_params=None):
    """Crop `box` -> LANCZOS resize to `shape` -> ToTensor (+ colour jitter) of a stack of images.

    images: uint8 [n_img, h, w, 3] on a ROCm device (HWC RGB, as PIL decodes), n_img a multiple
        of n_samples; image i belongs to sample i % n_samples.
    box: (left, top, right, bottom) PIL crop box; shape: (H, W) output size.
    jitter_params: list of n_samples random_color_jitter_params dicts, or None (no jitter).
    Returns (original fp32 [n_img,3,H,W], jittered fp32 [n_img,3,H,W] or None).
    """
    if not (images.is_cuda and images.dtype == torch.uint8 and images.dim() == 4 and images.shape[-1] == 3):
        raise RuntimeError("augment_images needs a uint8 [n, h, w, 3] tensor on a ROCm (HIP) device; "
                           f"got {images.dtype} {tuple(images.shape)} on {images.device}")
    images = images.contiguous()
    n_img, h, w, _ = images.shape
    H, W = shape
    p = _hip.AugmentParams(n_samples=n_samples, n_img=n_img, src_h=h, src_w=w, src_stride=h * w * 3,
                           crop_l=box[0], crop_t=box[1], crop_r=box[2], crop_b=box[3], out_h=H, out_w=W)
    plan, ws = _PLANS.get(p, images.device)
    orig = torch.empty((n_img, 3, H, W), dtype=torch.float32, device=images.device)
    rgb, jit = None, None
    if jitter_params is not None:
        if len(jitter_params) != n_samples:
            raise ValueError("one jitter record per sample")
        recs = (_hip.Jitter * n_samples)(*[jitter_record(j) for j in jitter_params])
        jit = _PLANS.upload(bytearray(recs), images.device)
        rgb = torch.empty_like(orig)
    rc = _hip.lib().psfm_train_augment(ctypes.byref(p), _hip.ptr(images), _hip.ptr(plan), _hip.ptr(jit), _hip.ptr(ws),
                                       _hip.ptr(orig), _hip.ptr(rgb), _hip.stream(images.device))
    _hip.check(rc, "psfm_train_augment")
    return orig, rgb


def crop_intrinsics(intrinsics, borders):
    """datasets/augmentations.py:392-410: principal point shifted by the crop (float32)."""
    K = intrinsics.clone()
    K[..., 0, 2] -= borders[0]
    K[..., 1, 2] -= borders[1]
    return K


def resize_intrinsics(intrinsics, orig_hw, shape):
    """datasets/augmentations.py:108-131: fx, cx *= W/w; fy, cy *= H/h (float32 products)."""
    K = intrinsics.clone()
    sw, sh = shape[1] / orig_hw[1], shape[0] / orig_hw[0]
    K[..., 0, 0] *= sw
    K[..., 1, 1] *= sh
    K[..., 0, 2] *= sw
    K[..., 1, 2] *= sh
    return K


def train_transforms_batch(batch, image_shape=(), jittering=(), crop_train_borders=(), prob=1.0, rng=random):
    """Batched datasets/transforms.py:21-50 train_transforms.

    batch: {'rgb': uint8 [B,h,w,3], 'rgb_context': [uint8 [B,h,w,3], ...], 'intrinsics':
    [B,3,3] float32, ...} with the images on a ROCm device.  Returns the collated sample the
    reference's DataLoader would produce: 'rgb', 'rgb_original' fp32 [B,3,H,W],
    'rgb_context', 'rgb_context_original' lists, 'intrinsics' (cropped, resized) and, when
    cropped, 'intrinsics_full'.  Jitter draws happen per sample in sample order from `rng`.
    """
    rgb = batch["rgb"]
    B, h, w, _ = rgb.shape
    ctx = list(batch.get("rgb_context", []))
    box = parse_crop_borders(crop_train_borders, (h, w))
    ch, cw = box[3] - box[1], box[2] - box[0]
    shape = tuple(image_shape) if len(image_shape) > 0 else (ch, cw)
    jit = None
    if len(jittering) > 0:
        jit = [random_color_jitter_params(jittering, prob, rng) for _ in range(B)]
    images = torch.cat([rgb] + ctx, 0) if ctx else rgb
    orig, jittered = augment_images(images, B, box, shape, jit)
    if jittered is None:
        jittered = orig.clone()   # duplicate_sample: rgb and rgb_original are separate copies
    out = {k: v for k, v in batch.items() if k not in ("rgb", "rgb_context")}
    out["rgb"], out["rgb_original"] = jittered[:B], orig[:B]
    out["rgb_context"] = [jittered[(i + 1) * B:(i + 2) * B] for i in range(len(ctx))]
    out["rgb_context_original"] = [orig[(i + 1) * B:(i + 2) * B] for i in range(len(ctx))]
    if "intrinsics" in batch:
        K = batch["intrinsics"].float()
        if len(crop_train_borders) > 0:
            out["intrinsics_full"] = K.clone()
            K = crop_intrinsics(K, box)
        if len(image_shape) > 0:
            K = resize_intrinsics(K, (ch, cw), shape)
        out["intrinsics"] = K
    out["jitter_params"] = jit
    return out


def validation_transforms_batch(batch, image_shape=(), crop_eval_borders=()):
    """Batched datasets/transforms.py:52-77 validation_transforms: crop -> resize of 'rgb' only
    (contexts are cropped, not resized, as in the reference) -> ToTensor."""
    rgb = batch["rgb"]
    B, h, w, _ = rgb.shape
    box = parse_crop_borders(crop_eval_borders, (h, w))
    ch, cw = box[3] - box[1], box[2] - box[0]
    out = {k: v for k, v in batch.items() if k not in ("rgb", "rgb_context")}
    shape = tuple(image_shape) if len(image_shape) > 0 else (ch, cw)
    out["rgb"] = augment_images(rgb, B, box, shape)[0]
    if "rgb_context" in batch:
        out["rgb_context"] = [augment_images(c, B, box, (ch, cw))[0] for c in batch["rgb_context"]]
    if "intrinsics" in batch and len(crop_eval_borders) > 0:
        out["intrinsics_full"] = batch["intrinsics"].float().clone()
        out["intrinsics"] = crop_intrinsics(batch["intrinsics"].float(), box)
    return out
