#!/bin/bash
# K12 with the K0 candidates prefetched one step ahead: kbench A/B against HEAD (interleaved),
# photometric / fisheye / ABI parity, default bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3c; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
V=build/variants
timeout -k 10 300 python -u tools/kbench.py --paths k12 --lib $V/k12old.so --lib $V/k12pre.so --lib $V/k12old.so --lib $V/k12pre.so > "$OUT/kbench_ab.log" 2>&1; rc=$?
echo "[kbench] rc=$rc"; grep k12 "$OUT/kbench_ab.log" | cut -c1-200
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_hip_photometric.py tests/test_fisheye.py tests/test_abi.py -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/parity.log" 2>&1; rc=$?
echo "[parity] rc=$rc"; tail -2 "$OUT/parity.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cut -c1-200 "$OUT/bench.json"; grep -o '"dominant_us_per_launch": [0-9.]*' "$OUT/bench.json"
