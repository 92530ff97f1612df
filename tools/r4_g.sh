#!/bin/bash
# GPU tests of this session's additions, default-config A/B (add_relu + HIP batch gather vs the op
# chains), and the capture-crash bisection (the likeliest crash last).   tools/r4_g.sh <tag>
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_netops.py tests/test_data_gather.py tests/test_networks.py -m gpu -q \
  --timeout 300 --timeout-method thread -rfE > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -2 "$OUT/tests.log"; grep -E "^(FAILED|ERROR)" "$OUT/tests.log" | head
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for rep in 1 2; do
  for v in new old; do
    f=""; [ $v = old ] && f="--no-add-relu --no-hip-gather"
    timeout -k 10 300 python -u bench.py --steps 50 --no-cpu-baseline --no-kernel-timing $f > "$OUT/bench_$v$rep.json" 2> "$OUT/bench_$v$rep.err"; rc=$?
    [ $rc -ne 0 ] && { tail -20 "$OUT/bench_$v$rep.err"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$v$rep.json'));print('$v', d['value'], d['ms_per_step'], d['k12_in_step']['us_mean'])"
  done
done
i=0
for flags in "--live-grad --side-warmup --no-bench --cpu-model --events" "--live-grad --side-warmup --no-bench --cpu-model --drop-all" "--live-grad --side-warmup --no-bench --cpu-model --drop-all --events"; do
  i=$((i+1))
  timeout -k 10 200 python -u tools/diag_gn_capture.py $flags > "$OUT/cap_$i.log" 2>&1; rc=$?
  echo "[capture $i: $flags] rc=$rc"; grep -v amdgpu.ids "$OUT/cap_$i.log" | tail -3
  [ $rc -ne 0 ] && exit $rc
done
exit 0
