#!/bin/bash
# evidence refresh: PMC traffic / SQ passes of the default bench config (tools/gpu_pmc_bench.sh),
# then a rocprof step summary of the PackNet01 B=6 config
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3t; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 120); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
bash tools/gpu_pmc_bench.sh > "$OUT/pmc.log" 2>&1; rc=$?
echo "[pmc] rc=$rc"; tail -3 "$OUT/pmc.log"; [ $rc -ne 0 ] && exit $rc
cp "$ROOT"/gpurun_out/pmc/*.json "$OUT/" && rm -rf "$ROOT"/gpurun_out/pmc   # raw passes exceed the copy-back cap
(cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --config kitti-packnet --steps 8 --warmup 4 --no-cpu-baseline --no-kernel-timing) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof packnet] rc=$rc"; [ $rc -ne 0 ] && exit $rc
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_packnet01.csv" \;
python3 tools/summarize_trace.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" "$OUT/step_summary_packnet01.txt" && head -3 "$OUT/step_summary_packnet01.txt"
rm -rf "$OUT/prof"
