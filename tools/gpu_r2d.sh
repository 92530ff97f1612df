#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2d
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u tools/diag_cycles.py > "$OUT/diag_cycles.log" 2>&1; rc=$?
echo "[diag_cycles] rc=$rc"; grep spread "$OUT/diag_cycles.log"; crash $rc && exit $rc
timeout -k 10 300 python -u tools/diag_accgrad.py > "$OUT/diag_accgrad.log" 2>&1; rc=$?
echo "[diag_accgrad] rc=$rc"; grep diag "$OUT/diag_accgrad.log"; crash $rc && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread -s > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/gpu_tests.log" | tail -12; crash $rc && exit $rc
exit 0
