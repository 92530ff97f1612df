#!/bin/bash
# the fixed add_relu / gather tests, then tools/gn_bench.py's capture crash bisected from its own side
# (one configuration per process, stops at the first failure; the full sequence last).
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_netops.py tests/test_data_gather.py -m gpu -q -k "add_relu or gather" \
  --timeout 200 --timeout-method thread -rfE > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -2 "$OUT/tests.log"; grep -E "^(FAILED|ERROR)|^E " "$OUT/tests.log" | head
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
i=0
for flags in "--no-live-grad --fwd-only" "--fwd-only --no-events" "--fwd-only"; do
  i=$((i+1))
  timeout -k 10 200 python -u tools/gn_bench.py --max-shapes 1 --iters 20 $flags > "$OUT/gnb_$i.log" 2>&1; rc=$?
  echo "[gn_bench $i: $flags] rc=$rc"; grep -v amdgpu.ids "$OUT/gnb_$i.log" | tail -3
  [ $rc -ne 0 ] && exit $rc
done
exit 0
