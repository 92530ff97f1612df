#!/bin/bash
# Round-3 GPU batch: pack3d tests + kernel A/B (VALU dW | MFMA dW | pipelined MFMA dW), the netops
# micro-benchmark under rocprofv3 (fused and reference chains), then PackNet bench lines.
#   tools/r3_batch.sh <tag> [bench configs...]
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
if [ "${TESTS:-}" != "" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v -s --timeout 300 --timeout-method thread -rfE > "$OUT/tests.log" 2>&1; rc=$?
  echo "[tests] rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/tests.log" | tail -5
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
if [ "${P3D:-1}" = 1 ]; then
  for net in packnet packnet-san; do
    timeout -k 10 300 python -u tools/p3d_bench.py --net $net --lib build/libpsfm_valu_dw.so --lib build/variants/mfma_nopipe.so \
      --lib packnet-sfm-resnet-san_amd/libpsfm_hip.so > "$OUT/p3d_$net.log" 2>&1; rc=$?
    echo "[p3d $net] rc=$rc"; grep total "$OUT/p3d_$net.log" | cut -c1-60; [ $rc -ne 0 ] && exit $rc
  done
fi
if [ "${NETOPS:-1}" = 1 ]; then
  for mode in fused ref; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/np_$mode" -o run --output-format csv \
       -- python3 "$ROOT/tools/netops_bench.py" --mode $mode --iters 20) > "$OUT/netops_$mode.log" 2>&1; rc=$?
    echo "[netops $mode] rc=$rc"; [ $rc -ne 0 ] && exit $rc
    find "$OUT/np_$mode" -name '*kernel_stats.csv' -exec cp {} "$OUT/netops_${mode}_kernel_stats.csv" \;
    rm -rf "$OUT/np_$mode"
  done
fi
for cfg in "$@"; do
  timeout -k 10 900 python -u bench.py --config $cfg --no-cpu-baseline > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err"; rc=$?
  echo "[bench $cfg] rc=$rc"; cut -c1-200 "$OUT/bench_$cfg.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_$cfg.err"; exit $rc; }
done
