#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2t; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 200 python -u tools/diag_accgrad_nodes.py > "$OUT/nodes.log" 2>&1; rc=$?
echo "[nodes] rc=$rc"; grep -c persistent "$OUT/nodes.log"; tail -2 "$OUT/nodes.log"
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py tests/test_netops.py -m gpu -q -p no:cacheprovider --timeout 250 --timeout-method thread > "$OUT/trainer.log" 2>&1; rc=$?
echo "[trainer+netops] rc=$rc"; tail -2 "$OUT/trainer.log"
