#!/bin/bash
# Round-4 diagnostics: K12 per-wave stamp dumps (KITTI default config and DDAD) and a kernel trace of
# the PackNet01 step (GN launches of the last steps + the full last step's timeline).
#   tools/r4_diag.sh <tag>
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
PSFM_STAMP_DUMP=$OUT/stamps_kitti.npy timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline \
  > "$OUT/bench_kitti.json" 2> "$OUT/bench_kitti.err"; rc=$?
echo "[kitti] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/bench_kitti.err"; exit $rc; }
python3 tools/k12_stamps.py "$OUT/stamps_kitti.npy" 4 4 192 640 18 | tee "$OUT/stamps_kitti.txt"
PSFM_STAMP_DUMP=$OUT/stamps_ddad.npy timeout -k 10 400 python -u bench.py --config ddad-packnet-san --steps 10 \
  --warmup 4 --no-cpu-baseline --no-miopen-find > "$OUT/bench_ddad.json" 2> "$OUT/bench_ddad.err"; rc=$?
echo "[ddad] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/bench_ddad.err"; exit $rc; }
cut -c1-300 "$OUT/bench_ddad.json"
RB=$(python3 -c "import json;print(json.load(open('$OUT/bench_ddad.json'))['roofline']['in_step']['waves'])")
echo "ddad waves $RB"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_pk" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --config kitti-packnet --steps 6 --warmup 3 --no-cpu-baseline --no-kernel-timing \
   --no-miopen-find) > "$OUT/prof_pk.log" 2>&1; rc=$?
echo "[prof packnet] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/prof_pk.log"; exit $rc; }
TR=$(find "$OUT/prof_pk" -name '*kernel_trace.csv' | head -1)
python3 tools/trace_grep.py "$TR" "." "$OUT/packnet_last_step.csv" --last-steps 1
python3 tools/trace_grep.py "$TR" "k_gn_" "$OUT/packnet_gn_last2.csv" --last-steps 2
rm -rf "$OUT/prof_pk"
exit 0
