#!/bin/bash
# pose algebra on HIP + pose net enqueued after the depth net: new pose tests, the photometric /
# trainer / network GPU tests, default bench, and a kernel-trace timeline of one graph step
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2z; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_pose.py tests/test_hip_photometric.py tests/test_trainer_gpu.py tests/test_fused_adam.py \
  tests/test_fisheye.py tests/test_networks.py -m gpu -x -v -rs --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -6
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cut -c1-300 "$OUT/bench.json"
[ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --steps 6 --warmup 5 --no-cpu-baseline) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_trace.py "$OUT/prof/run_kernel_trace.csv" "$OUT/step_timeline.txt" && tail -1 "$OUT/step_timeline.txt"
rm -rf "$OUT/prof"
