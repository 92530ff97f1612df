#!/bin/bash
# comm='overlap' on RCCL at world size 1 (tests + forced-comm bench), graph-vs-eager bf16 diagnosis,
# the rest of the trainer tests, smoke, default bench + CPU baseline, gloo N=2 launch rehearsal,
# rocprof kernel stats of the default bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3b; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
step() { name=$1; shift; echo "[$name] start $(date +%T)"; "$@"; rc=$?; echo "[$name] rc=$rc"; return $rc; }
step comm_tests timeout -k 10 300 python -u -m pytest tests/test_comm_gpu.py -m gpu -x -v -s -rs --timeout 240 --timeout-method thread > "$OUT/comm_tests.log" 2>&1
rc=$?; tail -4 "$OUT/comm_tests.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
step diag timeout -k 10 300 python -u tools/diag_graph_vs_eager.py > "$OUT/diag_graph_vs_eager.log" 2>&1 || exit $?
head -8 "$OUT/diag_graph_vs_eager.log"
step trainer_tests timeout -k 10 400 python -u -m pytest tests/test_trainer_gpu.py -m gpu -v -rs --timeout 240 --timeout-method thread > "$OUT/trainer_tests.log" 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed" "$OUT/trainer_tests.log" | tail -6; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -3 "$OUT/smoke.log"
step bench timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cut -c1-300 "$OUT/bench.json"
step bench_forcecomm timeout -k 10 400 python bench.py --force-comm --no-cpu-baseline > "$OUT/bench_forcecomm.json" 2> "$OUT/bench_forcecomm.err" || exit $?
cut -c1-300 "$OUT/bench_forcecomm.json"
step bench_g2_gloo timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_g2_gloo.json" 2> "$OUT/bench_g2_gloo.err" || exit $?
cut -c1-300 "$OUT/bench_g2_gloo.json"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --steps 6 --warmup 5 --no-cpu-baseline) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"
[ $rc -ne 0 ] && exit $rc
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
python3 tools/summarize_trace.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" "$OUT/step_timeline.txt" && head -3 "$OUT/step_timeline.txt"
rm -rf "$OUT/prof"
