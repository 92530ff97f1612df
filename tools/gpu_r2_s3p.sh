#!/bin/bash
# op-level attribution of the PackNet01 B=6 eager step (which ops launch the big copies / casts)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3p; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 120); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 1000 python -u tools/op_profile.py --depth-net PackNet01 --batch 6 --steps 2 --out "$OUT/op_profile_packnet01.txt" > "$OUT/op_profile.log" 2>&1; rc=$?
echo "[op_profile] rc=$rc"; tail -2 "$OUT/op_profile.log"
