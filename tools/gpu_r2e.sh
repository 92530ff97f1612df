#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2e
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u tools/diag_cycles.py > "$OUT/diag_cycles.log" 2>&1; rc=$?
echo "[diag_cycles] rc=$rc"; grep spread "$OUT/diag_cycles.log"; crash $rc && exit $rc
for det in none cudnn all; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --deterministic $det > "$OUT/bench_$det.json" 2> "$OUT/bench_$det.err"; rc=$?
  echo "[bench det=$det] rc=$rc $(python3 -c "import json,sys; d=json.load(open('$OUT/bench_$det.json')); print(d['value'], d['ms_per_step'])" 2>/dev/null)"; crash $rc && exit $rc
done
timeout -k 10 700 python -u -m pytest tests/test_hip_photometric.py -k "golden or benchmarked" -v -rs --timeout 300 --timeout-method thread -s > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/gpu_tests.log" | tail -12; crash $rc && exit $rc
exit 0
