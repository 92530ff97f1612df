#!/bin/bash
# capture-crash cause: a captured autograd backward whose forward ran on another stream (the engine
# launches the backward on the forward's stream, outside the capture).  Passing case first, the
# suspected crash last (one process each; stops at the first failure).
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
i=0
for flags in "--capture-bwd --bwd-on-capture-stream" "--capture-bwd"; do
  i=$((i+1))
  timeout -k 10 200 python -u tools/diag_gn_capture.py $flags > "$OUT/capbwd_$i.log" 2>&1; rc=$?
  echo "[capture bwd $i: $flags] rc=$rc"; grep -v amdgpu.ids "$OUT/capbwd_$i.log" | tail -6
  [ $rc -ne 0 ] && exit $rc
done
exit 0
