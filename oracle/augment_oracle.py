"""ORACLE — test infrastructure only (never imported by the product path).

ctypes wrapper of `oracle/augment_oracle.c`, the plain-C restatement of the reference's
host data path (packnet_sfm/datasets/transforms.py:21-50 train_transforms: crop -> LANCZOS
resize -> duplicate -> colour jitter -> ToTensor).  Only `tests/` and the CPU-baseline leg of
`tools/augment_bench.py` may use it, and only as the checker / the CPU baseline.  Pinned to
Pillow itself by tests/golden/augment_*.npz (tools/gen_augment_goldens.py).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "augment_oracle.c")
LIB = os.path.join(HERE, "_build", "libaugment_oracle.so")


class Jitter(ctypes.Structure):
    """oracle_jitter (= psfm_jitter, include/psfm_augment.h)."""
    _fields_ = [("apply", ctypes.c_int), ("order", ctypes.c_int * 4), ("factor", ctypes.c_float * 3),
                ("hue_shift", ctypes.c_int), ("use_matrix", ctypes.c_int), ("matrix", ctypes.c_float * 3)]


def build(force=False):
    """gcc the restatement (no FMA contraction: Pillow's x86-64 wheels do plain mul + add)."""
    if force or not os.path.exists(LIB) or os.path.getmtime(SRC) > os.path.getmtime(LIB):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-shared", SRC, "-o", LIB + ".tmp", "-lm"],
                       check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(build())
        u8p, V = ctypes.c_void_p, ctypes.c_void_p
        L.oracle_resample_plan.argtypes = [ctypes.c_int, ctypes.c_int, V, V]
        L.oracle_resample_plan.restype = ctypes.c_int
        L.oracle_resize_lanczos.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int, ctypes.c_int]
        L.oracle_color_jitter.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Jitter)]
        L.oracle_to_tensor.argtypes = [u8p, ctypes.c_int, ctypes.c_int, V]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def resample_plan(in_size, out_size):
    """(ksize, bounds [out,2] int32, coeffs [out,ksize] int32) — Pillow precompute_coeffs."""
    L = lib()
    k = L.oracle_resample_plan(in_size, out_size, None, None)
    b = np.zeros((out_size, 2), np.int32)
    c = np.zeros((out_size, k), np.int32)
    L.oracle_resample_plan(in_size, out_size, _ptr(b), _ptr(c))
    return k, b, c


def crop(img, box):
    """PIL Image.crop(box): box (left, top, right, bottom), zero fill outside the image."""
    l, t, r, b = box
    h, w = img.shape[:2]
    out = np.zeros((b - t, r - l, 3), np.uint8)
    sy0, sy1, sx0, sx1 = max(t, 0), min(b, h), max(l, 0), min(r, w)
    if sy1 > sy0 and sx1 > sx0:
        out[sy0 - t:sy1 - t, sx0 - l:sx1 - l] = img[sy0:sy1, sx0:sx1]
    return out


def resize(img, H, W):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.empty((H, W, 3), np.uint8)
    lib().oracle_resize_lanczos(_ptr(img), img.shape[0], img.shape[1], _ptr(out), H, W)
    return out


def make_jitter(apply=1, order=(0, 1, 2, 3), factors=(1.0, 1.0, 1.0), hue_shift=0, matrix=None):
    j = Jitter()
    j.apply = int(apply)
    for i in range(4):
        j.order[i] = int(order[i])
    for i in range(3):
        j.factor[i] = float(factors[i])
    j.hue_shift = int(hue_shift) & 255
    j.use_matrix = 0 if matrix is None else 1
    for i in range(3):
        j.matrix[i] = 0.0 if matrix is None else float(matrix[i])
    return j


def color_jitter(img, jitter):
    out = np.ascontiguousarray(img, np.uint8).copy()
    lib().oracle_color_jitter(_ptr(out), out.shape[0], out.shape[1], ctypes.byref(jitter))
    return out


def to_tensor(img):
    img = np.ascontiguousarray(img, np.uint8)
    out = np.empty((3,) + img.shape[:2], np.float32)
    lib().oracle_to_tensor(_ptr(img), img.shape[0], img.shape[1], _ptr(out))
    return out


def train_transform(images, box, shape, jitter):
    """One sample: images = [rgb, ctx...] HWC uint8 -> (rgb_original list, rgb list) CHW fp32."""
    orig, jit = [], []
    for im in images:
        c = crop(im, box) if box is not None else im
        r = resize(c, *shape) if shape is not None else np.ascontiguousarray(c)
        orig.append(to_tensor(r))
        jit.append(to_tensor(color_jitter(r, jitter)))
    return orig, jit
