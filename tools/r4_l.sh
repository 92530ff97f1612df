#!/bin/bash
# netops tests (incl. pipelined GN bitwise check), PackNet01 step A/B pipelined vs unpipelined two-pass
# GN (bench with MIOpen find, interleaved), GN in-step traces of both, then the DDAD traffic experiment.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 100); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_netops.py -m gpu -q --timeout 300 --timeout-method thread -rfE \
  > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -2 "$OUT/tests.log"; grep -E "^(FAILED|ERROR)" "$OUT/tests.log" | head
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for v in pipe nopipe pipe nopipe; do
  p=1; [ $v = nopipe ] && p=0
  PSFM_GN_PIPE=$p timeout -k 10 500 python -u bench.py --config kitti-packnet --steps 20 --warmup 5 --no-cpu-baseline \
    --no-kernel-timing > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err"; rc=$?
  [ $rc -ne 0 ] && { echo "[bench $v] rc=$rc"; tail -20 "$OUT/bench_$v.err"; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('$v', d['value'], d['ms_per_step'])"
done
for v in pipe nopipe; do
  p=1; [ $v = nopipe ] && p=0
  (cd /tmp && PSFM_GN_PIPE=$p timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_$v" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --config kitti-packnet --steps 6 --warmup 3 --no-cpu-baseline --no-kernel-timing) \
     > "$OUT/prof_$v.log" 2>&1; rc=$?
  echo "[prof $v] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/prof_$v.log"; exit $rc; }
  TR=$(find "$OUT/prof_$v" -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_grep.py "$TR" "k_gn" "$OUT/gn_$v.csv" --last-steps 2
  python3 tools/summarize_trace.py "$TR" "$OUT/step_summary_$v.txt" && head -3 "$OUT/step_summary_$v.txt" | cut -c1-150
  rm -rf "$OUT/prof_$v"
done
exit 0
