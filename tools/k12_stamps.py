"""Per-wave analysis of a K12 stamp dump (bench.py with PSFM_STAMP_DUMP=path.npy: [waves][2] int64
start / end on the 100 MHz clock, index = linear workgroup id L).  Maps L to the work item the way
psfm_sweep.h work_item() does (XCD = L % 8, contiguous w ranges per XCD; w -> (b, s, unit)) and
prints the duration distribution by XCD, scale, image, band and stripe.

  python tools/k12_stamps.py stamps.npy B S H W RB"""
import sys

import numpy as np

st = np.load(sys.argv[1])
B, S, H, W, RB = map(int, sys.argv[2:7])
OW = 60
nst = (W + OW - 1) // OW
nb = (H + RB - 1) // RB
units = nst * nb
T = units * B * S
assert st.shape[0] <= T, (st.shape, T)
L = np.arange(st.shape[0])
xcd, i = L & 7, L >> 3
q, r = T >> 3, T & 7
w = np.where(xcd < r, xcd * (q + 1) + i, r * (q + 1) + (xcd - r) * q + i)
bs, unit = w // units, w % units
b, s = bs // S, bs % S
band, stripe = unit // nst, unit % nst
t0 = st[:, 0].min()
start = (st[:, 0] - t0) * 0.01
dur = (st[:, 1] - st[:, 0]) * 0.01
end = start + dur
print(f"waves {len(st)}  span {end.max():.2f} us  wave mean {dur.mean():.2f} median {np.median(dur):.2f} "
      f"max {dur.max():.2f}  start spread max {start.max():.2f} us")
for name, key in (("xcd", xcd), ("scale", s), ("image", b), ("band", band), ("stripe", stripe)):
    parts = []
    for k in np.unique(key):
        m = key == k
        parts.append(f"{k}:{dur[m].mean():.1f}/{dur[m].max():.1f}")
    print(f"{name:7s} mean/max dur  " + "  ".join(parts))
print("slowest 12 waves (L xcd b s band stripe start dur):")
for j in np.argsort(-end)[:12]:
    print(f"  {j:5d} {xcd[j]} {b[j]} {s[j]} {band[j]:3d} {stripe[j]:3d} {start[j]:7.2f} {dur[j]:7.2f}")
hist, edges = np.histogram(dur, bins=12)
print("duration histogram:", " ".join(f"{e:.0f}:{h}" for e, h in zip(edges, hist)))
