#!/usr/bin/env python3
"""Golden fixtures for the training-sample transform, from Pillow itself.

The reference's transform chain (datasets/transforms.py:21-50 -> datasets/augmentations.py) calls
torchvision's PIL functional API, which is absent from this image; its arithmetic is Pillow's
(present here, PIL.__version__ recorded in the fixture).  This script makes exactly the Pillow
calls torchvision's PIL backend makes:
  Resize(LANCZOS)      -> Image.resize((W, H), Image.LANCZOS)
  adjust_brightness    -> ImageEnhance.Brightness(img).enhance(f)
  adjust_contrast      -> ImageEnhance.Contrast(img).enhance(f)
  adjust_saturation    -> ImageEnhance.Color(img).enhance(f)
  adjust_hue           -> img.convert('HSV') split, np_h += np.array(f * 255).astype(np.uint8),
                          Image.merge('HSV', ...).convert('RGB')
  colour matrix        -> img.convert('RGB', matrix)               (augmentations.py:300-317)
  crop                 -> img.crop(box)                             (augmentations.py:373-389)
and the crop boxes come from the reference's own `parse_crop_borders` (utils/misc.py:77-146,
imported from /root/reference with the same module stubs as tools/gen_goldens.py).
The jitter draws follow colorjitter_sample / random_color_jitter_transform's order
(augmentations.py:295-304, :346-368) with `random.seed(k)`.

Outputs tests/golden/augment_pil.npz.   Usage: python tools/gen_augment_goldens.py
"""
import hashlib
import os
import random
import sys
import types

import numpy as np
import PIL
from PIL import Image, ImageEnhance

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden", "augment_pil.npz")


def reference_parse_crop_borders():
    for name in ("yacs", "yacs.config"):
        m = types.ModuleType(name)
        sys.modules[name] = m
    sys.modules["yacs.config"].CfgNode = type("CfgNode", (dict,), {})
    sys.modules["yacs"].config = sys.modules["yacs.config"]
    sys.path.insert(0, "/root/reference")
    sys.dont_write_bytecode = True
    from packnet_sfm.utils.misc import parse_crop_borders
    return parse_crop_borders


def smooth_image(rng, h, w):
    """Smooth texture + noise (compresses well, exercises every code path)."""
    base = rng.random((h // 8 + 2, w // 8 + 2, 3))
    ys, xs = np.linspace(0, base.shape[0] - 1.001, h), np.linspace(0, base.shape[1] - 1.001, w)
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[:, None, None], (xs - x0)[None, :, None]
    b = base
    img = (b[y0][:, x0] * (1 - fy) * (1 - fx) + b[y0 + 1][:, x0] * fy * (1 - fx) +
           b[y0][:, x0 + 1] * (1 - fy) * fx + b[y0 + 1][:, x0 + 1] * fy * fx)
    img = img * 255 + rng.normal(0, 6, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def draw_jitter(parameters, prob, rng):
    """colorjitter_sample + random_color_jitter_transform draw order (augmentations.py:295-368)."""
    if not rng.random() < prob:
        return None
    b, c, s, h = parameters[:4]
    f = [rng.uniform(max(0, 1 - b), 1 + b), rng.uniform(max(0, 1 - c), 1 + c),
         rng.uniform(max(0, 1 - s), 1 + s), rng.uniform(-h, h)]
    order = [0, 1, 2, 3]
    rng.shuffle(order)
    m = None
    if len(parameters) > 4 and parameters[4] > 0:
        m = [rng.uniform(1. - parameters[4], 1 + parameters[4]) for _ in range(3)]
    return f, order, m


def pil_hue(img, hue_factor):
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    np_h += np.array(hue_factor * 255).astype(np.uint8)
    return Image.merge("HSV", (Image.fromarray(np_h, "L"), s, v)).convert("RGB")


def pil_jitter(img, draw):
    if draw is None:
        return img
    f, order, m = draw
    for o in order:
        if o == 0:
            img = ImageEnhance.Brightness(img).enhance(f[0])
        elif o == 1:
            img = ImageEnhance.Contrast(img).enhance(f[1])
        elif o == 2:
            img = ImageEnhance.Color(img).enhance(f[2])
        else:
            img = pil_hue(img, f[3])
    if m is not None:
        img = img.convert("RGB", (m[0], 0, 0, 0, 0, m[1], 0, 0, 0, 0, m[2], 0))
    return img


def sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def main():
    parse_crop_borders = reference_parse_crop_borders()
    rng = np.random.default_rng(20261016)
    z = {"pil_version": np.array(PIL.__version__)}

    # 1. resize cases (crop box, output size), incl. up / down / one-axis / identity / out-of-image crops
    cases = [((37, 53), (0, 0, 53, 37), (16, 24)), ((24, 80), (0, 0, 80, 24), (48, 160)),
             ((60, 200), (0, 0, 200, 60), (60, 100)), ((61, 40), (0, 0, 40, 61), (30, 40)),
             ((30, 45), (0, 0, 45, 30), (30, 45)), ((50, 90), (-7, 5, 80, 58), (20, 33)),
             ((75, 248), (3, 5, 246, 70), (19, 64)), ((9, 300), (0, 0, 300, 9), (7, 13))]
    for i, (hw, box, out) in enumerate(cases):
        img = smooth_image(rng, *hw) if i % 2 else rng.integers(0, 256, hw + (3,), dtype=np.uint8)
        pil = Image.fromarray(img).crop(box)
        res = pil.resize((out[1], out[0]), Image.LANCZOS) if pil.size != (out[1], out[0]) else pil
        z[f"resize{i}_in"], z[f"resize{i}_box"], z[f"resize{i}_out"] = img, np.array(box), np.array(res)
    z["n_resize"] = np.array(len(cases))

    # 2. KITTI-size resize (input regenerated from the seed in the test; pinned by its sha256)
    kin = np.random.default_rng(7).integers(0, 256, (375, 1242, 3), dtype=np.uint8)
    kout = np.array(Image.fromarray(kin).resize((640, 192), Image.LANCZOS))
    z["kitti_in_sha"], z["kitti_out_sha"], z["kitti_out_rows"] = sha(kin), sha(kout), kout[[0, 1, 95, 190, 191]]

    # 3. jitter cases on one image: seeded draws in the reference order
    jimg = smooth_image(rng, 40, 64)
    z["jitter_img"] = jimg
    params = [(0.2, 0.2, 0.2, 0.05), (0.5, 0.9, 1.5, 0.5), (0.2, 0.2, 0.2, 0.05, 0.1), (0.0, 0.0, 0.0, 0.0),
              (1.2, 1.2, 1.2, 0.3, 0.3)]
    k = 0
    for pi, par in enumerate(params):
        for seed in range(4):
            r = random.Random(1000 * pi + seed)
            d = draw_jitter(par, 1.0 if seed else 0.5, r)
            z[f"jit{k}_params"] = np.array(par + (0.0,) * (5 - len(par)), np.float64)
            z[f"jit{k}_seed"], z[f"jit{k}_prob"] = np.array(1000 * pi + seed), np.array(1.0 if seed else 0.5)
            z[f"jit{k}_apply"] = np.array(d is not None)
            if d is not None:
                z[f"jit{k}_f"], z[f"jit{k}_order"] = np.array(d[0]), np.array(d[1])
                z[f"jit{k}_m"] = np.array(d[2] if d[2] is not None else [np.nan] * 3)
            z[f"jit{k}_out"] = np.array(pil_jitter(Image.fromarray(jimg), d))
            k += 1
    z["n_jit"] = np.array(k)

    # 4. exhaustive hue: every RGB colour through adjust_hue (sha256 of Pillow's result)
    allc = np.arange(1 << 24, dtype=np.uint32)
    every = np.stack([(allc >> 16) & 255, (allc >> 8) & 255, allc & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
    for f in (0.0, 7 / 255, -12.75 / 255):
        z[f"hue_all_{int(np.array(f * 255).astype(np.uint8))}"] = sha(np.array(pil_hue(Image.fromarray(every), f)))

    # 5. crop specs through the reference's parse_crop_borders
    specs = [((-352, 0, 0.5, 1216), (375, 1242)), ((-352, 0, 0.5, 1216), (370, 1224)), ((), (375, 1242)),
             ((10, 100, 20, 300), (375, 1242)), ((-100, -10, -300, -20), (375, 1242)), ((0.5, 100, 0.5, 300), (200, 640)),
             ((20, 30), (375, 1242)), ((-20, -30), (375, 1242)), ((100.0, 0.5), (375, 1242))]
    z["n_crop"] = np.array(len(specs))
    for i, (b, shp) in enumerate(specs):
        z[f"crop{i}_spec"] = np.array([float(v) for v in b] + [np.nan] * (4 - len(b)))
        z[f"crop{i}_isint"] = np.array([isinstance(v, int) for v in b] + [False] * (4 - len(b)))
        z[f"crop{i}_len"], z[f"crop{i}_shape"] = np.array(len(b)), np.array(shp)
        z[f"crop{i}_box"] = np.array(parse_crop_borders(b, shp))

    # 6. one full training sample: 3 images, tiny-config-style crop, resize, jitter (seeded)
    simgs = [smooth_image(rng, 75, 248) for _ in range(3)]
    box = parse_crop_borders((-70, 0, 0.5, 240), (75, 248))
    r = random.Random(42)
    d = draw_jitter((0.2, 0.2, 0.2, 0.05), 1.0, r)
    orig, jit = [], []
    for im in simgs:
        p = Image.fromarray(im).crop(box).resize((80, 24), Image.LANCZOS)
        orig.append(np.array(p))
        jit.append(np.array(pil_jitter(p, d)))
    z["sample_in"], z["sample_box"] = np.stack(simgs), np.array(box)
    z["sample_orig"], z["sample_rgb"] = np.stack(orig), np.stack(jit)
    z["sample_seed"] = np.array(42)

    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    np.savez_compressed(OUT, **z)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
