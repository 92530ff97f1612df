#!/bin/bash
# GPU box: augment parity tests, micro-bench, rocprof kernel stats (each step time-limited;
# stops at the first crash-like exit).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/augment; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_augment.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
echo "[augment tests] rc=$rc"; tail -3 "$OUT/tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/augment_bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[augment bench] rc=$rc"; cat "$OUT/bench.json"
[ $rc -ne 0 ] && exit $rc
rm -rf "$OUT/prof"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$ROOT/tools/augment_bench.py" --no-cpu-baseline --iters 50) > "$OUT/prof.log" 2>&1; rc=$?
echo "[augment prof] rc=$rc"
[ $rc -ne 0 ] && exit $rc
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/prof" -name "*kernel_trace.csv" -delete
head -12 "$OUT/kernel_stats.csv"
exit 0
