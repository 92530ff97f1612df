#!/bin/bash
# op-level attribution of the default ResNetSAN01 B=4 eager step (fills / small copies)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/s3r; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 600 python -u tools/op_profile.py --depth-net ResNetSAN01 --batch 4 --steps 2 --out "$OUT/op_profile_resnet.txt" > "$OUT/op_profile.log" 2>&1; rc=$?
echo "[op_profile] rc=$rc"; tail -1 "$OUT/op_profile.log"
