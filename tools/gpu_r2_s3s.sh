#!/bin/bash
# round-end style check of the current tree: whole GPU suite, smoke, default bench (+ CPU baseline),
# rocprofv3 kernel stats + trace summary of the same bench command
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3s; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 100); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -6
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "[smoke] rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cut -c1-200 "$OUT/bench.json"; [ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --steps 6 --warmup 5 --no-cpu-baseline) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"; [ $rc -ne 0 ] && exit $rc
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
python3 tools/summarize_trace.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" "$OUT/step_summary.txt" && head -3 "$OUT/step_summary.txt"
rm -rf "$OUT/prof"
