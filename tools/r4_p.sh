#!/bin/bash
# pack3d dx: grouped matrix-core staging (PSFM_P3D_DX=mfmag) parity + microbench A/B against cl.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_pack3d.py -m gpu -q -x --timeout 250 --timeout-method thread -rfE -k dx_matrix_core \
  > "$OUT/p3d_dx_tests.log" 2>&1; rc=$?
echo "[p3d dx tests] rc=$rc"; tail -2 "$OUT/p3d_dx_tests.log"
[ $rc -ne 0 ] && exit $rc
for net in packnet packnet-san; do
  timeout -k 10 200 python -u tools/p3d_bench.py --net $net --dx mfmag,cl,mfmag,cl > "$OUT/p3d_bench_$net.log" 2>&1; rc=$?
  echo "[p3d bench $net] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p3d_bench_$net.log"; exit $rc; }
  python3 - "$OUT/p3d_bench_$net.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if " dx=" not in line: continue
    tag, form, js = line.split(" ", 2)
    d = json.loads(js)
    packs = {k: v[1] for k, v in d.items() if k.startswith("pack")}
    print(form, "dx per pack layer", packs, "total dx", d["total_fwd_bwdx_bwdw_us"][1])
PY
done
