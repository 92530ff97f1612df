#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2f
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_trainer_gpu.py tests/test_hip_photometric.py -v -rs --timeout 300 --timeout-method thread -s > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|passed|failed|median relative" "$OUT/gpu_tests.log" | tail -12; crash $rc && exit $rc
timeout -k 10 300 python -u tools/p3d_bench.py --iters 10 --net packnet-san > "$OUT/p3d_bench_san.log" 2>&1; rc=$?
echo "[p3d bench san] rc=$rc"; tail -1 "$OUT/p3d_bench_san.log"
exit 0
