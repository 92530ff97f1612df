#!/bin/bash
# GPU-box driver: tests, bench, rocprof kernel trace.  Stops at the first crash-like exit
# (abort/segfault/timeout: 124, 134, 137, 139) so nothing else runs on a faulted GPU.
# usage: tools/gpu_run.sh [tests] [bench] [prof] [pmc]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 500 python -u -m pytest "$ROOT/tests" -m gpu -x -v -rs --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
      echo "[tests] rc=$rc"; tail -3 "$OUT/gpu_tests.log"; crash $rc && exit $rc ;;
    smoke)
      (cd "$ROOT" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()") > "$OUT/smoke.log" 2>&1; rc=$?
      echo "[smoke] rc=$rc"; tail -2 "$OUT/smoke.log"; crash $rc && exit $rc ;;
    bench)
      (cd "$ROOT" && timeout -k 10 600 python bench.py) > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
      echo "[bench] rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; crash $rc && exit $rc ;;
    prof)
      rm -rf "$OUT/prof"
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
         -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing) > "$OUT/prof.log" 2>&1; rc=$?
      echo "[prof] rc=$rc"; crash $rc && exit $rc
      python3 "$ROOT/tools/summarize_trace.py" "$OUT/prof/run_kernel_trace.csv" "$OUT/prof/step_summary.txt"
      rm -f "$OUT/prof/run_kernel_trace.csv" ;;
    pmc)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        rm -rf "$OUT/pmc_$ctr"
        (cd /tmp && timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_$ctr" -o run \
           -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 --no-cpu-baseline --no-kernel-timing) > "$OUT/pmc_$ctr.log" 2>&1; rc=$?
        echo "[pmc $ctr] rc=$rc"; tail -2 "$OUT/pmc_$ctr.log"; crash $rc && exit $rc
      done ;;
    kpmc)
      for ctr in FETCH_SIZE WRITE_SIZE; do
        rm -rf "$OUT/kpmc_$ctr"
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/kpmc_$ctr" -o run \
           -- python3 "$ROOT/tools/kbench.py" --iters 3 --paths k12) > "$OUT/kpmc_$ctr.log" 2>&1; rc=$?
        echo "[kpmc $ctr] rc=$rc"; tail -2 "$OUT/kpmc_$ctr.log"; crash $rc && exit $rc
      done
      python3 "$ROOT/tools/pmc_traffic.py" "$OUT/kpmc_FETCH_SIZE" "$OUT/kpmc_WRITE_SIZE" "$OUT/pmc_traffic.json" 4 > /dev/null; echo "[kpmc] agg rc=$?" ;;
    kbench)
      (cd "$ROOT" && timeout -k 10 300 python tools/kbench.py --iters 30) > "$OUT/kbench.log" 2>&1; rc=$?
      echo "[kbench] rc=$rc"; tail -3 "$OUT/kbench.log"; crash $rc && exit $rc ;;
  esac
done
exit 0
