#!/bin/bash
# K12 wave-pair priority A/B (PSFM_K12_PRIO 0/1/2) on one box: kbench (isolated replays, B=4 and B=6)
# and the default bench's in-step K12 time per mode.   tools/r4_prio.sh <tag>
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 300 python -u tools/kbench.py --paths k12 --iters 50 --prio 0,1,2 --reps 3 > "$OUT/kbench_b4.log" 2>&1; rc=$?
echo "[kbench b4] rc=$rc"; grep -v "^\[" "$OUT/kbench_b4.log" | cut -c1-160; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/kbench.py --paths k12 --iters 50 --prio 0,1,2 --reps 3 --B 6 > "$OUT/kbench_b6.log" 2>&1; rc=$?
echo "[kbench b6] rc=$rc"; grep -v "^\[" "$OUT/kbench_b6.log" | cut -c1-160; [ $rc -ne 0 ] && exit $rc
for m in 0 1 2 0 1 2; do
  PSFM_K12_PRIO=$m PSFM_STAMP_DUMP=$OUT/stamps_m$m.npy timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline \
    > "$OUT/bench_m$m.json" 2> "$OUT/bench_m$m.err"; rc=$?
  [ $rc -ne 0 ] && { tail -20 "$OUT/bench_m$m.err"; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/bench_m$m.json'));r=d['roofline'];print('mode $m', d['value'], r['in_step']['us_mean'], r['in_step']['wave_us_mean'], r['in_step']['wave_us_max'], r['isolated_us_per_launch'])"
  python3 tools/k12_stamps.py "$OUT/stamps_m$m.npy" 4 4 192 640 18 | sed -n 3p
done
exit 0
