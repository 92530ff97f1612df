#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2q; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
for v in default k1k2 eager_upsample serial_pose; do
  DIAG_VARIANT=$v timeout -k 10 200 python -u tools/diag_graph_alive.py > "$OUT/diag_$v.log" 2>&1; rc=$?
  echo "[$v] rc=$rc $(grep 'done' $OUT/diag_$v.log)"
  case $rc in 0) ;; *) tail -5 "$OUT/diag_$v.log"; exit $rc;; esac
done
