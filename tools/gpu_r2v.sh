#!/bin/bash
# glue census of one eager step (call sites of fills / copies / elementwise ops) + a kernel-trace
# timeline of one graph-replayed step (idle gaps, stream overlap)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2v; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 60); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 300 python -u tools/diag_glue_ops.py --out "$OUT/glue_ops.txt" > "$OUT/glue.log" 2>&1; rc=$?
echo "[glue] rc=$rc"; tail -3 "$OUT/glue.log"
case $rc in 124|134|137|139) exit $rc;; esac
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --steps 6 --warmup 5 --no-cpu-baseline) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_trace.py "$OUT/prof/run_kernel_trace.csv" "$OUT/step_timeline.txt" && tail -1 "$OUT/step_timeline.txt"
rm -rf "$OUT/prof"
