#!/bin/bash
# PackNet decoder merge written channels_last in the autocast dtype: pack3d + network tests, then
# the three PackNet bench presets
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3q; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 120); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_pack3d.py tests/test_networks.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -1 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
for cfg in kitti-packnet-san ddad-packnet-san kitti-packnet; do
  timeout -k 10 700 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err"; rc=$?
  echo "[bench $cfg] rc=$rc $(grep -o '"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' "$OUT/bench_$cfg.json")"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
