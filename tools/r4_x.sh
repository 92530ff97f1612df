#!/bin/bash
# MIOpen find mode A/B on the default bench (NORMAL = exhaustive find vs the default), own user db each.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
run() {
  local name=$1; shift
  env MIOPEN_USER_DB_PATH=/tmp/udb_$name "$@" timeout -k 10 300 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-kernel-timing \
    > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"; local rc=$?
  [ $rc -ne 0 ] && { echo "[bench $name] rc=$rc"; tail -5 "$OUT/bench_$name.err"; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$name.json'));print('$name', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
  grep "warmup step 0" "$OUT/bench_$name.err"
}
run base
run normal MIOPEN_FIND_MODE=1
run base2
run normal2 MIOPEN_FIND_MODE=1
