#!/bin/bash
# Interleaved bench A/B on one box: tools/r5_ab.sh TAG CONFIG ROUNDS "name:[VAR=v ...@@]extra args" ...
# (each variant runs once per round, in order), then an optional rocprof step summary of the first
# variant (PROF=1).  Lines go to gpurun_out/TAG/ab.txt.
set -u
TAG=$1; CFG=$2; ROUNDS=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
(for i in $(seq 1 200); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    name=${spec%%:*}; extra=${spec#*:}; envs=""
    if [[ "$extra" == *@@* ]]; then envs=${extra%%@@*}; extra=${extra#*@@}; fi
    env $envs timeout -k 10 400 python -u bench.py --config "$CFG" --steps 20 --warmup 5 --no-cpu-baseline $extra \
      > "$OUT/bench_${name}_$r.json" 2> "$OUT/bench_${name}_$r.err"; rc=$?
    [ $rc -ne 0 ] && { echo "[bench $name] rc=$rc"; tail -5 "$OUT/bench_${name}_$r.err"; exit $rc; }
    python3 -c "import json;d=json.load(open('$OUT/bench_${name}_$r.json'));print('$name', $r, d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d.get('roofline',{}).get('dominant_us_per_launch'))" | tee -a "$OUT/ab.txt"
  done
done
if [ "${PROF:-0}" = 1 ]; then
  spec=$1; name=${spec%%:*}; extra=${spec#*:}
  if [[ "$extra" == *@@* ]]; then extra=${extra#*@@}; fi
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --config "$CFG" --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing $extra) > "$OUT/prof_$name.log" 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "[prof $name] rc=$rc"; tail -5 "$OUT/prof_$name.log"; exit $rc; }
  python3 "$ROOT/tools/summarize_trace.py" "$OUT/prof_$name/run_kernel_trace.csv" "$OUT/step_summary_${CFG}_$name.txt" > /dev/null
  rm -f "$OUT/prof_$name/run_kernel_trace.csv"
  head -40 "$OUT/step_summary_${CFG}_$name.txt" | cut -c1-160
fi
