#!/bin/bash
# DDAD-shaped K12 (B=4 images of 384x640) HBM fetch with smooth vs i.i.d.-noisy sigmoid maps: is the
# 6x fetch of the ddad-packnet-san bench the kernel's gather locality or the random-init network's
# per-pixel-noise depth?  One FETCH_SIZE pass each (rocprofv3 --pmc, K12 only), + timing.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for v in smooth noisy; do
  f=""; [ $v = noisy ] && f="--noisy"
  for H in 192 384; do
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k12_fwd_grad --output-format csv -d "$OUT/p_${v}_$H" -o run \
      -- python3 "$ROOT/tools/kbench.py" --paths k12 --B 4 --H $H --iters 3 $f > "$OUT/p_${v}_$H.log" 2>&1; rc=$?
    echo "[pmc $v H=$H] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p_${v}_$H.log"; exit $rc; }
    python3 - "$OUT/p_${v}_$H" $H $v <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
v = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == "FETCH_SIZE"]
H = int(sys.argv[2]); alg = H * 640 * 120 * 4
fb = sorted(v)[len(v) // 2] * 2 * 1024 if v else float("nan")
print(f"{sys.argv[3]} H={H}: K12 read bytes per launch (2*1024*FETCH_SIZE, median of {len(v)}) {fb/1e6:.1f} MB = {fb/alg:.2f}x the 120 B/px algorithmic bytes")
PY
    rm -rf "$OUT/p_${v}_$H"
  done
done
exit 0
