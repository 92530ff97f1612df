#!/bin/bash
# pack3d channels_last dx, k-pair form: parity (test_pack3d) and p3d micro-benchmark A/B against
# the one-k form (P3D_DX_PAIRS=0), PackNet01 (d=8) and PackNetSAN01 (d=4), interleaved
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3h; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_pack3d.py -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pack3d_tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -2 "$OUT/pack3d_tests.log"; [ $rc -ne 0 ] && exit $rc
V=build/variants
for net in packnet packnet-san; do
  timeout -k 10 300 python -u tools/p3d_bench.py --net $net --lib $V/p3dx0.so --lib $V/p3dx1.so --lib $V/p3dx2.so --lib $V/p3dx0.so --lib $V/p3dx1.so --lib $V/p3dx2.so > "$OUT/p3d_ab_$net.log" 2>&1; rc=$?
  echo "[p3d $net] rc=$rc"; grep total "$OUT/p3d_ab_$net.log" | sed 's/.*\(p3dx[012]\).*total_fwd_bwdx_bwdw_us": \(.*\)}/\1 \2/'
  [ $rc -ne 0 ] && exit $rc
done
exit 0
