#!/bin/bash
# fold of upsample_output into K12 + decoder upcat: GPU tests, then bench A/B of the net epilogues
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2k; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread \
  -k "nearest_scales or upcat or networks or trainer or fused_adam or kitti_full or benchmarked" > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -8
[ $rc -ne 0 ] && exit $rc
for v in none bias gn bias,gn all; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --fused-nets $v > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"; rc=$?
  echo "[bench $v] rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['kernels_us_per_step'])" "$OUT/bench_$v.json" 2>/dev/null)"
  case $rc in 0) ;; *) tail -5 "$OUT/bench_$v.err"; exit $rc;; esac
done
