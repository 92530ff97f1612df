#!/bin/bash
# GN per-launch durations in the PackNet01 step, resident vs two-pass (rocprofv3 kernel trace, MIOpen
# heuristics instead of find to keep the run short), then the capture-crash bisection.
#   tools/r4_gn2.sh <tag>
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
for path in resident twopass; do
  if [ $path = twopass ]; then export PSFM_GN_PATH=twopass; else unset PSFM_GN_PATH; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_$path" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --config kitti-packnet --steps 6 --warmup 3 --no-cpu-baseline --no-kernel-timing \
     --no-miopen-find) > "$OUT/prof_$path.log" 2>&1; rc=$?
  echo "[prof $path] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/prof_$path.log"; exit $rc; }
  TR=$(find "$OUT/prof_$path" -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_grep.py "$TR" "k_gn" "$OUT/gn_$path.csv" --last-steps 2
  python3 tools/trace_grep.py "$TR" "." "$OUT/all_$path.csv" --last-steps 2
  rm -rf "$OUT/prof_$path"
done
unset PSFM_GN_PATH
i=0
for flags in "--keep" "" "--live-grad" "--live-grad --side-warmup --no-bench" "--live-grad --side-warmup --no-bench --cpu-model"; do
  i=$((i+1))
  timeout -k 10 200 python -u tools/diag_gn_capture.py $flags > "$OUT/cap_$i.log" 2>&1; rc=$?
  echo "[capture $i: $flags] rc=$rc"; grep -v amdgpu.ids "$OUT/cap_$i.log" | tail -4
  [ $rc -ne 0 ] && exit $rc
done
exit 0
