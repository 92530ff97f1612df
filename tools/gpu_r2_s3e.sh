#!/bin/bash
# single-launch cooperative BatchNorm(+residual)(+ReLU): netops parity (coop + tree forms, graph
# replays), A/B bench (MIOpen BN default vs fused coop BN, interleaved), kernel trace of the coop run
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3e; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_netops.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/netops_tests.log" 2>&1; rc=$?
echo "[netops] rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/netops_tests.log" | tail -4
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for f in bias,gn bias,gn,bn; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-timing --fused-nets $f > "$OUT/bench_${f//,/_}_$i.json" 2> "$OUT/bench_${f//,/_}_$i.err"; rc=$?
    echo "[bench $f $i] rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/bench_${f//,/_}_$i.json")"
    [ $rc -ne 0 ] && exit $rc
  done
done
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --steps 6 --warmup 5 --no-cpu-baseline --no-kernel-timing --fused-nets bias,gn,bn) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/summarize_trace.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" "$OUT/step_summary_coop_bn.txt" && head -3 "$OUT/step_summary_coop_bn.txt" && grep -i "bn_\|BatchNorm" "$OUT/step_summary_coop_bn.txt" | head -8
rm -rf "$OUT/prof"
