#!/bin/bash
# K12 A/B on one box: tools/kbench.py over build/variants/*.so (interleaved twice).
#   tools/r3_k12ab.sh <tag> name1 name2 ...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
libs=""
for rep in 1 2; do for n in "$@"; do libs="$libs --lib build/variants/$n.so"; done; done
timeout -k 10 600 python -u tools/kbench.py --paths k12 --iters ${ITERS:-50} ${KB_ARGS:-} $libs > "$OUT/kbench${KB_TAG:-}.log" 2>&1; rc=$?
echo "[kbench] rc=$rc"; grep -v "^\[" "$OUT/kbench${KB_TAG:-}.log" | cut -c1-300 | tail -20; [ $rc -ne 0 ] && { tail -20 "$OUT/kbench${KB_TAG:-}.log"; exit $rc; }
exit 0
