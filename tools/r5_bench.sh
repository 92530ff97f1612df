#!/bin/bash
# Bench lines for a list of configs (+ rocprof kernel-trace step summary for each), heartbeat under
# gpurun_out/<TAG>.  usage: tools/r5_bench.sh TAG [--prof] config [config ...]
set -u
TAG=$1; shift
PROF=0
if [ "${1:-}" = "--prof" ]; then PROF=1; shift; fi
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
(for i in $(seq 1 100); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
for cfg in "$@"; do
  timeout -k 10 400 python -u bench.py --config "$cfg" --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err"; rc=$?
  [ $rc -ne 0 ] && { echo "[bench $cfg] rc=$rc"; tail -5 "$OUT/bench_$cfg.err"; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'))"
  if [ $PROF = 1 ]; then
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv \
       -- python3 "$ROOT/bench.py" --config "$cfg" --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing) > "$OUT/prof_$cfg.log" 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "[prof $cfg] rc=$rc"; tail -5 "$OUT/prof_$cfg.log"; exit $rc; }
    python3 "$ROOT/tools/summarize_trace.py" "$OUT/prof_$cfg/run_kernel_trace.csv" "$OUT/step_summary_$cfg.txt" > /dev/null
    rm -f "$OUT/prof_$cfg/run_kernel_trace.csv"
    head -30 "$OUT/step_summary_$cfg.txt" | cut -c1-150
  fi
done
