#!/bin/bash
# photometric small kernels with batched loads (finalize / pose reduce / sigmoid sums): kbench A/B
# against HEAD (interleaved), then the whole GPU suite (incl. the capture-fallback test), smoke,
# default bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3g; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
V=build/variants
timeout -k 10 300 python -u tools/kbench.py --paths k12 --lib $V/phold.so --lib $V/phnew.so --lib $V/phold.so --lib $V/phnew.so > "$OUT/kbench_ab.log" 2>&1; rc=$?
echo "[kbench] rc=$rc"; grep k12 "$OUT/kbench_ab.log" | cut -c1-220
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/gpu_tests.log" | tail -8
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "[smoke] rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cut -c1-200 "$OUT/bench.json"
