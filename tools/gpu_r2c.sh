#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2c
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u tools/diag_accgrad.py > "$OUT/diag_accgrad.log" 2>&1; rc=$?
echo "[diag_accgrad] rc=$rc"; grep diag "$OUT/diag_accgrad.log"; crash $rc && exit $rc
timeout -k 10 300 python -u tools/diag_conv_det.py > "$OUT/diag_conv.log" 2>&1; rc=$?
echo "[diag_conv] rc=$rc"; grep det= "$OUT/diag_conv.log"; crash $rc && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_pack3d.py tests/test_trainer_gpu.py -x -q --timeout 200 --timeout-method thread > "$OUT/p3d_tests.log" 2>&1; rc=$?
echo "[p3d tests] rc=$rc"; tail -5 "$OUT/p3d_tests.log"; crash $rc && exit $rc
timeout -k 10 300 python -u tools/p3d_bench.py --iters 10 > "$OUT/p3d_bench.log" 2>&1; rc=$?
echo "[p3d bench] rc=$rc"; tail -3 "$OUT/p3d_bench.log"
exit 0
