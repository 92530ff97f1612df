#!/bin/bash
# Round-4 GPU check: full -m gpu suite, smoke, the default bench line, and a rocprofv3 kernel-trace
# step summary of the same bench command.  OUT=gpurun_out/<tag>.  Stops at the first failing GPU step.
#   tools/r3_check.sh <tag> [bench args...]
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
# heartbeat: MIOpen's first find on a cold box prints nothing for minutes
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread -rfE \
    > "$OUT/tests.log" 2>&1; rc=$?
  echo "[tests] rc=$rc"; tail -3 "$OUT/tests.log"; grep -E "^(FAILED|ERROR)" "$OUT/tests.log" | head -20
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
  echo "[smoke] rc=$rc"; tail -6 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 400 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "[bench] rc=$rc"; cut -c1-400 "$OUT/bench.json"; [ $rc -ne 0 ] && { tail -20 "$OUT/bench.err"; exit $rc; }
if [ "${SKIP_PROF:-0}" != 1 ]; then
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" "$@" --steps 8 --warmup 4 --no-cpu-baseline --no-kernel-timing) > "$OUT/prof.log" 2>&1; rc=$?
  echo "[prof] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/prof.log"; exit $rc; }
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  python3 tools/summarize_trace.py "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" "$OUT/step_summary.txt" \
    && head -40 "$OUT/step_summary.txt" | cut -c1-160
  rm -rf "$OUT/prof"
fi
