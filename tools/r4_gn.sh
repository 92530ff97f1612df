#!/bin/bash
# Round-4 GroupNorm: GPU tests of the netops (both GN paths), the gn_bench capture-crash bisection
# (one configuration per process, the likeliest crash last; stops at the first failure), and the
# PackNet01 / PackNetSAN01 step A/B resident vs two-pass GN.   tools/r4_gn.sh <tag>
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_netops.py -m gpu -v --timeout 300 --timeout-method thread -rfE \
  > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 "$OUT/tests.log"; grep -E "^(FAILED|ERROR)" "$OUT/tests.log" | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
if [ "${SKIP_AB:-0}" != 1 ]; then
for cfg in kitti-packnet kitti-packnet-san; do
  for path in resident twopass resident twopass; do
    e=""; [ $path = twopass ] && e="PSFM_GN_PATH=twopass"
    env $e timeout -k 10 500 python -u bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing \
      > "$OUT/bench_${cfg}_$path.json" 2> "$OUT/bench_${cfg}_$path.err"; rc=$?
    [ $rc -ne 0 ] && { echo "[bench $cfg $path] rc=$rc"; tail -20 "$OUT/bench_${cfg}_$path.err"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/bench_${cfg}_$path.json'));print('$cfg $path', d['value'], d['ms_per_step'])"
  done
done
fi
i=0
for flags in "--keep" "" "--live-grad" "--live-grad --side-warmup --no-bench" "--live-grad --side-warmup --no-bench --cpu-model"; do
  i=$((i+1))
  timeout -k 10 200 python -u tools/diag_gn_capture.py $flags > "$OUT/cap_$i.log" 2>&1; rc=$?
  echo "[capture $i: $flags] rc=$rc"; grep -v amdgpu.ids "$OUT/cap_$i.log" | tail -4
  [ $rc -ne 0 ] && exit $rc
done
exit 0
