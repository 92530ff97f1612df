"""fp32 emulation of K12's pinhole sampling positions against float64, over random KITTI-shaped points
(u, v on the 640x192 grid, depth log-uniform in [0.5, 80], the test poses of tests/golden_util):
  ref    the reference chain: x_n = K^-1 [u, v, 1], X = d x_n, c = R X + t, p = K_ref c
  A      p = d (A x) + m, A = K_ref R K^-1 (rounded once)
  E      p = d (E x) + (d x + m), E = A - I (rounded once; the round-6 kernel, fused.h PairProj)
Prints the max / 99.9th percentile / mean |ix - ix64| over in-image projections (fma emulated in float64).
  python tools/emu_projection_error.py"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import golden_util as gu  # noqa: E402
from oracle import photometric_oracle as O  # noqa: E402

f = np.float32


def fma(a, b, c):
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(f)


def run(seed, B=1, H=192, W=640, N=1000000):
    K = gu.kitti_K(B, H, W)[0].double().numpy()
    g = torch.Generator().manual_seed(seed)
    T = np.asarray(O.pose_vec_to_mat(gu.pose_vecs(g, B, 2)[:, 0])[0], dtype=np.float64)
    Ki = np.linalg.inv(K)
    rng = np.random.default_rng(seed)
    u = rng.integers(0, W, N).astype(np.float64)
    v = rng.integers(0, H, N).astype(np.float64)
    d = np.exp(rng.uniform(np.log(0.5), np.log(80), N))
    X = d * (Ki @ np.stack([u, v, np.ones_like(u)]))
    p = K @ (T[:3, :3] @ X + T[:3, 3:4])
    ex, ey = p[0] / p[2], p[1] / p[2]
    ok = (p[2] > 0.1) & (ex > -1) & (ex < W) & (ey > -1) & (ey < H)
    uu, vv, dd = u.astype(f), v.astype(f), d.astype(f)

    def err(pp):
        ix, iy = (pp[0] / pp[2]).astype(f), (pp[1] / pp[2]).astype(f)
        e = np.concatenate([np.abs(ix - ex)[ok], np.abs(iy - ey)[ok]])
        return f"max {e.max():.2e}  p99.9 {np.percentile(e, 99.9):.2e}  mean {e.mean():.2e}"
    K32, Ki32, T32 = K.astype(f), Ki.astype(f), T.astype(f)
    xn = [fma(Ki32[k, 1], vv, Ki32[k, 0] * uu) + Ki32[k, 2] for k in range(3)]
    Xo = [x * dd for x in xn]
    co = [((T32[r, 0] * Xo[0] + T32[r, 1] * Xo[1]) + T32[r, 2] * Xo[2]) + T32[r, 3] for r in range(3)]
    po = [(K32[r, 0] * co[0] + K32[r, 1] * co[1]) + K32[r, 2] * co[2] for r in range(3)]
    A64, m64 = K @ T[:3, :3] @ Ki, K @ T[:3, 3]
    A, m = A64.astype(f), m64.astype(f)
    pa = [fma(fma(A[k, 1], vv, fma(A[k, 0], uu, A[k, 2])), dd, m[k]) for k in range(3)]
    E = (A64 - np.eye(3)).astype(f)
    e = [fma(E[k, 1], vv, fma(E[k, 0], uu, E[k, 2])) for k in range(3)]
    base = [uu, vv, np.ones_like(uu)]
    pe = [fma(dd, e[k], fma(dd, base[k], m[k])) for k in range(3)]
    print(f"seed {seed}: ref {err(po)} | A {err(pa)} | E {err(pe)}")


if __name__ == "__main__":
    for s in (3, 5, 7):
        run(s)
