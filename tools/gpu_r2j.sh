#!/bin/bash
# attribute the step's glue kernels to ops (eager torch.profiler) + MIOpen solver A/B on the bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2j; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 300 python tools/op_profile.py --steps 2 --out "$OUT/op_profile.txt" > "$OUT/op_profile.log" 2>&1; rc=$?
echo "[op_profile] rc=$rc"; tail -2 "$OUT/op_profile.log"
case $rc in 124|134|137|139) exit $rc;; esac
bash tools/exp_miopen.sh base nowrw nowrwbwd noasm
