#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2p; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 300 python -u tools/diag_graph_alive.py > "$OUT/diag.log" 2>&1; rc=$?
echo "[diag] rc=$rc"; grep -v amdgpu.ids "$OUT/diag.log" | tail -40
