#!/bin/bash
# round-2 session B, call 1: full GPU test suite + smoke on a fresh box
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2h
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread --durations=25 > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -15; crash $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "[smoke] rc=$rc"; tail -8 "$OUT/smoke.log"
exit 0
