#!/bin/bash
# pack3d: full parity suite (incl. the unpack dW matrix-core test), microbench A/B of the unpack dW forms.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 200 python -u -m pytest tests/test_pack3d.py -m gpu -q -x --timeout 150 --timeout-method thread -rfE -k "unpack_dw or dx_matrix" \
  > "$OUT/p3d_new_tests.log" 2>&1; rc=$?
echo "[p3d new tests] rc=$rc"; tail -2 "$OUT/p3d_new_tests.log"
[ $rc -ne 0 ] && exit $rc
for net in packnet packnet-san; do
  timeout -k 10 200 python -u tools/p3d_bench.py --net $net --dw mfma,generic,mfma,generic > "$OUT/p3d_bench_$net.log" 2>&1; rc=$?
  echo "[p3d bench $net] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p3d_bench_$net.log"; exit $rc; }
  python3 - "$OUT/p3d_bench_$net.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if " dw=" not in line: continue
    tag, dx, dw, js = line.split(" ", 3)
    d = json.loads(js)
    un = {k: v[2] for k, v in d.items() if k.startswith("unpack")}
    print(dw, "unpack dW", un, "sum", round(sum(un.values()), 1), "totals", d["total_fwd_bwdx_bwdw_us"])
PY
done
timeout -k 10 560 python -u -m pytest tests/test_pack3d.py -m gpu -q -x --timeout 500 --timeout-method thread -rfE \
  > "$OUT/p3d_tests.log" 2>&1; rc=$?
echo "[p3d all tests] rc=$rc"; tail -2 "$OUT/p3d_tests.log"
exit $rc
