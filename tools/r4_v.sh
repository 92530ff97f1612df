#!/bin/bash
# host enqueue time vs step time of the default bench (is the step host-bound?)
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
cd "$ROOT"
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-kernel-timing > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench.err"; exit $rc; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
