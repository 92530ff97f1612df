#!/bin/bash
# N = 2 launch rehearsal on one GPU over gloo (the driver's self-launch path, two ranks on cuda:0).
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
cd "$ROOT"
timeout -k 10 500 python -u bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing \
  > "$OUT/bench_g2.json" 2> "$OUT/bench_g2.err"; rc=$?
echo "[bench g2 gloo] rc=$rc"; tail -3 "$OUT/bench_g2.err"; cut -c1-300 "$OUT/bench_g2.json"
exit $rc
