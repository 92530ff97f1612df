#!/bin/bash
# is the AccumulateGrad warning of test_graph_replayed_step_equals_eager_step_exactly present at the
# r2l commit (a2a3447, worktree in build/wt) as well?
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2r; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT/build/wt"
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -k exactly -q -p no:cacheprovider --timeout 250 --timeout-method thread > "$OUT/old.log" 2>&1; rc=$?
echo "[a2a3447] rc=$rc"; tail -2 "$OUT/old.log"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -k exactly -q -p no:cacheprovider --timeout 250 --timeout-method thread > "$OUT/new.log" 2>&1; rc=$?
echo "[HEAD] rc=$rc"; tail -2 "$OUT/new.log"
