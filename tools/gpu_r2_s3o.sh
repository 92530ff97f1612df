#!/bin/bash
# (1) whole GPU suite + smoke + default bench on the current tree (pack3d r = 2 shift path);
# (2) op-level attribution of the PackNet01 B=6 step (which ops launch the big copies)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3o; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 120); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -6
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "[smoke] rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cut -c1-200 "$OUT/bench.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/op_profile.py --depth-net PackNet01 --batch 6 --steps 2 --out "$OUT/op_profile_packnet01.txt" > "$OUT/op_profile.log" 2>&1; rc=$?
echo "[op_profile] rc=$rc"; tail -2 "$OUT/op_profile.log"
