#!/bin/bash
# pack3d: parity (incl. both dx forms), microbench A/B of the dx forms, then the r4_l GN / DDAD runs.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
PSFM_P3D_DX=mfma timeout -k 10 500 python -u -m pytest tests/test_pack3d.py -m gpu -q -x --timeout 400 --timeout-method thread -rfE \
  -k "real_layer or matches_reference_chain or fused_op" -s > "$OUT/p3d_tests_mfma.log" 2>&1; rc=$?
echo "[p3d tests mfma default] rc=$rc"; tail -3 "$OUT/p3d_tests_mfma.log"; grep "^mode" "$OUT/p3d_tests_mfma.log"
[ $rc -ne 0 ] && exit $rc
for net in packnet packnet-san; do
  timeout -k 10 200 python -u tools/p3d_bench.py --net $net --dx mfma4,mfma2,mfma1,cl,mfma4,mfma2,mfma1,cl > "$OUT/p3d_bench_$net.log" 2>&1; rc=$?
  echo "[p3d bench $net] rc=$rc"; cut -c1-400 "$OUT/p3d_bench_$net.log" | tail -4
  [ $rc -ne 0 ] && exit $rc
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$ROOT/tools/p3d_bench.py" --net packnet --dx mfma --only pack64x192x640) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/prof.log"; exit $rc; }
S=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1); cp "$S" "$OUT/p3d_kernel_stats.csv"; cut -d, -f1-8 "$S" | head -8
rm -rf "$OUT/prof"
