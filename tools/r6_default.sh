#!/bin/bash
# The driver's default bench line (N = 1, defaults: config, steps, warmup, CPU baseline) + a rocprofv3
# kernel-trace --stats run of the same command.  usage: tools/r6_default.sh TAG
set -u
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 500 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
cat "$OUT/bench_default.json"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --no-cpu-baseline) > "$OUT/prof.log" 2>&1 || exit $?
python3 "$ROOT/tools/summarize_trace.py" "$OUT/prof/run_kernel_trace.csv" "$OUT/step_summary_default.txt" > /dev/null
rm -f "$OUT/prof/run_kernel_trace.csv"
head -8 "$OUT/step_summary_default.txt" | cut -c1-140
