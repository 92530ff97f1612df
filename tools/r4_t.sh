#!/bin/bash
# rocprofv3 kernel stats of the pack3d microbenchmark with the final default forms (both nets).
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
for net in packnet packnet-san; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$net" -o run \
     -- python3 "$ROOT/tools/p3d_bench.py" --net $net --iters 10) > "$OUT/prof_$net.log" 2>&1; rc=$?
  echo "[prof $net] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/prof_$net.log"; exit $rc; }
  S=$(find "$OUT/prof_$net" -name '*kernel_stats.csv' | head -1)
  [ -n "$S" ] && cp "$S" "$OUT/p3d_kernel_stats_$net.csv" && cut -d, -f1-8 "$S" | grep -i p3d | cut -c1-160
  rm -rf "$OUT/prof_$net"
done
