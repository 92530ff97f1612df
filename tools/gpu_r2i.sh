#!/bin/bash
# round-2 measurement: default bench line (N=1), rocprofv3 kernel-trace/stats of the same command,
# PMC passes (traffic, VALU) stamped for this config
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2i
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
cd "$ROOT"
timeout -k 10 500 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cat "$OUT/bench.json"; grep -v amdgpu.ids "$OUT/bench.err" | tail -3
[ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline "$@") > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"; grep -E '^\{' "$OUT/prof.log" | tail -1 > "$OUT/prof_bench.json"
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_trace.py "$OUT/prof/run_kernel_trace.csv" "$OUT/step_summary.txt" && head -30 "$OUT/step_summary.txt" | cut -c1-150
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
rm -f "$OUT/prof/run_kernel_trace.csv"
bash tools/gpu_pmc_bench.sh "$@"; rc=$?
echo "[pmc] rc=$rc"
# keep only the summaries (gpurun copies back at most 64 MiB)
rm -rf "$OUT/prof" "$ROOT"/gpurun_out/pmc/p[0-9]*
du -sh "$ROOT/gpurun_out"
exit 0
