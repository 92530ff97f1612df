#!/bin/bash
# PackNet01 + PoseNet training-step bench (BASELINE configs[2] shapes: B=6, 192x640) + rocprof summary.
# MIOpen compiles the bf16 Conv3d kernels on a cold box (~6 min): the kernel cache is kept in
# $MIOPEN_CUSTOM_CACHE_DIR (build/miopen_cache if the tree carries one, else gpurun_out/).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/packnet; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -d "$ROOT/build/miopen_cache" ]; then export MIOPEN_CUSTOM_CACHE_DIR=$ROOT/build/miopen_cache
else export MIOPEN_CUSTOM_CACHE_DIR=$ROOT/gpurun_out/miopen_cache; fi
mkdir -p "$MIOPEN_CUSTOM_CACHE_DIR"
(for i in $(seq 1 60); do date >> "$OUT/heartbeat.txt"; sleep 20; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
(cd "$ROOT" && timeout -k 10 700 python bench.py --depth-net PackNet01 --batch 6 --steps 20 --warmup 5 --no-cpu-baseline --no-miopen-find) \
  > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cat "$OUT/bench.json"; grep -v amdgpu.ids "$OUT/bench.err" | tail -8
case $rc in 0) ;; *) exit $rc;; esac
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --depth-net PackNet01 --batch 6 --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-miopen-find) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"
python3 "$ROOT/tools/summarize_trace.py" "$OUT/prof/run_kernel_trace.csv" "$OUT/step_summary.txt" && head -45 "$OUT/step_summary.txt" | cut -c1-160
rm -f "$OUT/prof/run_kernel_trace.csv"
du -sh "$MIOPEN_CUSTOM_CACHE_DIR"
