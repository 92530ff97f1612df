#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2t; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 200 python -u tools/diag_accgrad_trace.py > "$OUT/trace.log" 2>&1; rc=$?
echo "[trace] rc=$rc"; grep -v amdgpu.ids "$OUT/trace.log" | tail -60
