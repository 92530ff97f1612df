#!/bin/bash
# round-2 GPU session B: full GPU tests, gradient diagnostics, PackNetSAN01 bench (config 3)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2b
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -d "$ROOT/build/miopen_cache" ]; then export MIOPEN_CUSTOM_CACHE_DIR=$ROOT/build/miopen_cache
else export MIOPEN_CUSTOM_CACHE_DIR=$ROOT/gpurun_out/miopen_cache; fi
mkdir -p "$MIOPEN_CUSTOM_CACHE_DIR"
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread -s > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/gpu_tests.log" | tail -8; crash $rc && exit $rc
timeout -k 10 200 python -u tools/diag_wgrad.py > "$OUT/diag_wgrad.log" 2>&1; rc=$?
echo "[diag_wgrad] rc=$rc"; tail -30 "$OUT/diag_wgrad.log"; crash $rc && exit $rc
timeout -k 10 200 python -u tools/diag_accgrad.py > "$OUT/diag_accgrad.log" 2>&1; rc=$?
echo "[diag_accgrad] rc=$rc"; tail -3 "$OUT/diag_accgrad.log"; crash $rc && exit $rc
timeout -k 10 600 python bench.py --config kitti-packnet-san --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_pns.json" 2> "$OUT/bench_pns.err"; rc=$?
echo "[bench packnet-san] rc=$rc"; cat "$OUT/bench_pns.json"; grep -v amdgpu.ids "$OUT/bench_pns.err" | tail -5
du -sh "$MIOPEN_CUSTOM_CACHE_DIR"
exit 0
