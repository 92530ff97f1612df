#!/bin/bash
# (a) ordered kernel timeline of one default-config (ResNetSAN01 + PoseNet) step, with MIOpen find as
# the bench runs it; (b) PackNet01 two-pass GN grid targets 1024 / 2048 in the step (kernel trace);
# (c) tools/gn_bench.py's HIP-graph timing (the round-3 capture segfault) — last, it may crash.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_rs" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --steps 6 --warmup 4 --no-cpu-baseline --no-kernel-timing) > "$OUT/prof_rs.log" 2>&1; rc=$?
echo "[prof resnet] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/prof_rs.log"; exit $rc; }
TR=$(find "$OUT/prof_rs" -name '*kernel_trace.csv' | head -1)
python3 tools/trace_grep.py "$TR" "." "$OUT/resnet_last2.csv" --last-steps 2
rm -rf "$OUT/prof_rs"
for nb in 1024 2048; do
  (cd /tmp && PSFM_GN_BLOCKS=$nb timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof_$nb" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --config kitti-packnet --steps 6 --warmup 3 --no-cpu-baseline --no-kernel-timing \
     --no-miopen-find) > "$OUT/prof_$nb.log" 2>&1; rc=$?
  echo "[prof gn $nb] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/prof_$nb.log"; exit $rc; }
  TR=$(find "$OUT/prof_$nb" -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_grep.py "$TR" "." "$OUT/all_gn$nb.csv" --last-steps 2
  rm -rf "$OUT/prof_$nb"
done
timeout -k 10 300 python -u tools/gn_bench.py --iters 20 > "$OUT/gn_bench_graph.log" 2>&1; rc=$?
echo "[gn_bench graph] rc=$rc"; grep -v amdgpu.ids "$OUT/gn_bench_graph.log" | tail -6
exit 0
