#!/bin/bash
# round-2 GPU session A: tests, diagnostics, bench (N=1 sampler path), N=2 gloo rehearsal
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2a
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -4 "$OUT/gpu_tests.log"; crash $rc && exit $rc
timeout -k 10 200 python -u tools/diag_accgrad.py > "$OUT/diag_accgrad.log" 2>&1; rc=$?
echo "[diag_accgrad] rc=$rc"; tail -5 "$OUT/diag_accgrad.log"; crash $rc && exit $rc
timeout -k 10 120 python -u tools/diag_rccl_capture.py > "$OUT/diag_rccl.log" 2>&1; rc=$?
echo "[diag_rccl] rc=$rc"; tail -3 "$OUT/diag_rccl.log"; crash $rc && exit $rc
timeout -k 10 400 python bench.py --steps 30 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"; crash $rc && exit $rc
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_g2.json" 2> "$OUT/bench_g2.err"; rc=$?
echo "[bench gloo x2] rc=$rc"; cat "$OUT/bench_g2.json"; tail -5 "$OUT/bench_g2.err"
exit 0
