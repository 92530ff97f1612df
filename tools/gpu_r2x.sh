#!/bin/bash
# per-launch normalisation kernel times with the fused BN+act epilogue on (bias,gn,bn) vs the
# default (bias,gn; BN on MIOpen): step summaries by kernel and by grid
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2x; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
for v in "bias,gn" "bias,gn,bn"; do
  tag=$(echo $v | tr , _)
  timeout -k 10 300 python bench.py --no-cpu-baseline --fused-nets $v > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err"; rc=$?
  echo "[bench $v] rc=$rc"; python3 -c "import json,sys; d=json.loads(open('$OUT/bench_$tag.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
  [ $rc -ne 0 ] && exit $rc
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d "$OUT/prof_$tag" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --steps 6 --warmup 5 --no-cpu-baseline --fused-nets $v) > "$OUT/prof_$tag.log" 2>&1; rc=$?
  echo "[prof $v] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  python3 tools/summarize_trace.py "$OUT/prof_$tag/run_kernel_trace.csv" "$OUT/step_$tag.txt" | head -2
  rm -rf "$OUT/prof_$tag"
done
