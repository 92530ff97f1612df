#!/bin/bash
# GroupNorm geometry A/B: tools/gn_bench.py per-shape timings for each library, PackNetSAN01 and PackNet01.
# usage: tools/r6_gnab.sh TAG LIB...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$ROOT"
i=0
for lib in "$@"; do
  i=$((i+1))
  for net in PackNetSAN01 PackNet01; do
    timeout -k 10 200 python -u tools/gn_bench.py --depth-net $net --batch 6 --lib "$lib" > "$OUT/l${i}_$net.txt" 2>&1 || exit $?
    echo "[lib $i $lib $net] $(tail -1 $OUT/l${i}_$net.txt)"
  done
done
