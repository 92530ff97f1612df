#!/bin/bash
# round-2 final measurement: full GPU suite + smoke, default bench line, rocprof summary of the same
# command, PMC passes stamped for the default config (K12 traffic / VALU of the current kernel)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2u; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 90); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -4
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "[smoke] rc=$rc"; tail -2 "$OUT/smoke.log" | cut -c1-200
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cut -c1-400 "$OUT/bench.json"; grep -c AccumulateGrad "$OUT/bench.err"
[ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_trace.py "$OUT/prof/run_kernel_trace.csv" "$OUT/step_summary.txt" && head -3 "$OUT/step_summary.txt"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
grep k12_fwd_grad "$OUT/kernel_stats.csv" | cut -c1-160
rm -rf "$OUT/prof"
bash tools/gpu_pmc_bench.sh; rc=$?
echo "[pmc] rc=$rc"
rm -rf "$ROOT"/gpurun_out/pmc/p[0-9]*
