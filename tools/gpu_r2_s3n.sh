#!/bin/bash
# comm='bucketed' (eager bucket all-reduces behind events recorded by the backward graph): world-1
# RCCL tests incl. the ordering test, then the forced-comm bench at N=1: split vs bucketed
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3n; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_comm_gpu.py tests/test_trainer_gpu.py -m gpu -x -v -s --timeout 240 --timeout-method thread > "$OUT/comm_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; grep -E "PASSED|FAILED|passed|failed" "$OUT/comm_tests.log" | tail -8; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for c in split bucketed; do
  timeout -k 10 300 python bench.py --force-comm --comm $c --no-cpu-baseline --no-kernel-timing > "$OUT/bench_${c}_$i.json" 2> "$OUT/bench_${c}_$i.err"; rc=$?
  echo "[bench $c $i] rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/bench_${c}_$i.json")"; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
