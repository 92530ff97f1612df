#!/bin/bash
# Round-3 measurement of the final library, per bench config: the bench line, a rocprofv3
# kernel-trace step summary of the same command, and the stamped PMC profile (3 passes,
# tools/gpu_pmc_bench.sh -> gpurun_out/pmc/<key>/<key>.json, copied by hand to profiles/pmc/).
#   tools/r3_final.sh <tag> config [config ...]      (CPU baseline only for kitti-resnet-san; SKIP_PMC=1, SKIP_BENCH=1)
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
for cfg in "$@"; do
  cb=--no-cpu-baseline; [ "$cfg" = kitti-resnet-san ] && cb=""
  if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 400 python -u bench.py --config $cfg $cb > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err"; rc=$?
  echo "[bench $cfg] rc=$rc"; cut -c1-240 "$OUT/bench_$cfg.json"; [ $rc -ne 0 ] && { tail -5 "$OUT/bench_$cfg.err"; exit $rc; }
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv \
     -- python3 "$ROOT/bench.py" --config $cfg --steps 8 --warmup 4 --no-cpu-baseline --no-kernel-timing) > "$OUT/prof_$cfg.log" 2>&1; rc=$?
  echo "[prof $cfg] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/prof_$cfg.log"; exit $rc; }
  find "$OUT/prof_$cfg" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$cfg.csv" \;
  python3 tools/summarize_trace.py "$(find "$OUT/prof_$cfg" -name '*kernel_trace.csv' | head -1)" "$OUT/step_summary_$cfg.txt" \
    && head -3 "$OUT/step_summary_$cfg.txt" | cut -c1-160
  rm -rf "$OUT/prof_$cfg"
  fi
  if [ "${SKIP_PMC:-0}" != 1 ]; then
    PMC_EXTRA=--no-miopen-find bash tools/gpu_pmc_bench.sh --config $cfg; rc=$?
    echo "[pmc $cfg] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  fi
done
exit 0
