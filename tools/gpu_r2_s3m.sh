#!/bin/bash
# horizontal LANCZOS pass with one LDS word per pixel and tap-major coefficients: bit-exact augment
# tests, then augment micro-benchmark A/B (separate processes, interleaved)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3m; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_augment.py tests/test_augment_oracle.py -x -q --timeout 240 --timeout-method thread > "$OUT/augment_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -1 "$OUT/augment_tests.log"; [ $rc -ne 0 ] && exit $rc
V=build/variants
for i in 1 2; do for v in augold augnew; do
  timeout -k 10 120 python -u tools/augment_bench.py --lib $V/$v.so --no-cpu-baseline > "$OUT/bench_${v}_$i.json" 2> "$OUT/bench_${v}_$i.err"; rc=$?
  echo "[$v $i] rc=$rc $(grep -o '"us_per_call": [0-9.]*' "$OUT/bench_${v}_$i.json")"; [ $rc -ne 0 ] && exit $rc
done; done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/tools/augment_bench.py" --no-cpu-baseline) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"; [ $rc -ne 0 ] && exit $rc
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
grep -i "resize\|jitter" "$OUT/kernel_stats.csv" | cut -c1-160
rm -rf "$OUT/prof"
