#!/bin/bash
# pack3d address maps with the r = 2 dW software pipeline: parity + p3d micro-benchmark A/B (interleaved)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3l; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_pack3d.py -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pack3d_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -1 "$OUT/pack3d_tests.log"; [ $rc -ne 0 ] && exit $rc
V=build/variants
for net in packnet packnet-san; do
  timeout -k 10 300 python -u tools/p3d_bench.py --net $net --lib $V/dwold.so --lib $V/dwnew.so --lib $V/dwold.so --lib $V/dwnew.so > "$OUT/p3d_ab_$net.log" 2>&1; rc=$?
  echo "[p3d $net] rc=$rc"; grep total "$OUT/p3d_ab_$net.log" | sed 's/.*\(dwold\|dwnew\).*total_fwd_bwdx_bwdw_us": \(.*\)}/\1 \2/'
  [ $rc -ne 0 ] && exit $rc
done
exit 0
