#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2p; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 python -u tools/diag_graph_alive.py > "$OUT/diag.log" 2>&1; rc=$?
echo "[diag] rc=$rc"; grep -v amdgpu.ids "$OUT/diag.log" | tail -40
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 60); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --config kitti-packnet --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_trace.py "$OUT/prof/run_kernel_trace.csv" "$OUT/step_summary_packnet01.txt" && head -45 "$OUT/step_summary_packnet01.txt" | cut -c1-150
rm -rf "$OUT/prof"
