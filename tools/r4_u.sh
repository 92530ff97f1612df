#!/bin/bash
# K12 border-side split: photometric parity, kbench A/B (old vs new library, interleaved), bench in-step.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_hip_photometric.py -m gpu -q -x --timeout 250 --timeout-method thread -rfE \
  > "$OUT/photometric_tests.log" 2>&1; rc=$?
echo "[photometric tests] rc=$rc"; tail -2 "$OUT/photometric_tests.log"
[ $rc -ne 0 ] && exit $rc
for B in 4 6; do
  timeout -k 10 200 python -u tools/kbench.py --paths k12 --B $B --iters 20 --reps 3 \
    --lib build/variants/k12_before_border.so --lib build/variants/k12_border_split.so > "$OUT/kbench_b$B.log" 2>&1; rc=$?
  echo "[kbench B=$B] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/kbench_b$B.log"; exit $rc; }
  grep -o '^[^ ]*/k12_[a-z_]*\.so.*"K12_photometric_fwd_grad": [0-9.]*' "$OUT/kbench_b$B.log" | sed 's/{.*"K12/K12/' 
done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.err"; exit $rc; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['dominant_us_per_launch'], r.get('isolated_us_per_launch'), r['in_step'])"
