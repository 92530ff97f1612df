#!/bin/bash
# PackNet hand-written kernels against their HBM roofline: fused GroupNorm+ELU at every PackNet01 /
# PackNetSAN01 layer shape (B=6, 192x640; HIP events + rocprof kernel stats) and the pack3d
# micro-benchmark
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3d; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 300 python -u tools/gn_bench.py --depth-net PackNet01 > "$OUT/gn_packnet01.log" 2>&1; rc=$?
echo "[gn01] rc=$rc"; tail -1 "$OUT/gn_packnet01.log"; [ $rc -ne 0 ] && exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/tools/gn_bench.py" --depth-net PackNet01) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"; [ $rc -ne 0 ] && exit $rc
find "$OUT/prof" -name '*kernel_trace.csv' -exec cp {} "$OUT/gn_packnet01_trace.csv" \;
rm -rf "$OUT/prof"
timeout -k 10 300 python -u tools/gn_bench.py --depth-net PackNetSAN01 > "$OUT/gn_packnetsan01.log" 2>&1; rc=$?
echo "[gnsan] rc=$rc"; tail -1 "$OUT/gn_packnetsan01.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/p3d_bench.py --net packnet > "$OUT/p3d_packnet01.log" 2>&1; rc=$?
echo "[p3d] rc=$rc"; tail -4 "$OUT/p3d_packnet01.log"
