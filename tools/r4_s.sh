#!/bin/bash
# pack3d forward on the matrix cores: parity (forms), microbench A/B of the forward forms.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 200 python -u -m pytest tests/test_pack3d.py -m gpu -q -x --timeout 150 --timeout-method thread -rfE -k "forward_matrix" \
  > "$OUT/p3d_fwd_tests.log" 2>&1; rc=$?
echo "[p3d fwd tests] rc=$rc"; tail -2 "$OUT/p3d_fwd_tests.log"; grep -E "^E .*(assert|Error)" "$OUT/p3d_fwd_tests.log" | head -5
[ $rc -ne 0 ] && exit $rc
for net in packnet packnet-san; do
  timeout -k 10 200 python -u tools/p3d_bench.py --net $net --fwd mfma,valu,mfma,valu > "$OUT/p3d_bench_$net.log" 2>&1; rc=$?
  echo "[p3d bench $net] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p3d_bench_$net.log"; exit $rc; }
  python3 - "$OUT/p3d_bench_$net.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if " fwd=" not in line: continue
    parts = line.split(" ", 4)
    d = json.loads(parts[4])
    f = {k: v[0] for k, v in d.items() if k.startswith(("pack", "unpack"))}
    print(parts[3], "fwd", f, "total", d["total_fwd_bwdx_bwdw_us"][0])
PY
done
