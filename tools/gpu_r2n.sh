#!/bin/bash
# PackNet configs: PackNet01 B=6 (config 3 net), DDAD PackNetSAN01 1x4 cameras 384x640 (config 5),
# rocprof step summary of the PackNetSAN01 KITTI step
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2n; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
for cfg in ddad-packnet-san kitti-packnet; do
  timeout -k 10 500 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err"; rc=$?
  echo "[bench $cfg] rc=$rc"; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['kernels_us_per_step'])" "$OUT/bench_$cfg.json"
  [ $rc -ne 0 ] && { tail -5 "$OUT/bench_$cfg.err"; exit $rc; }
done
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
   -- python3 "$ROOT/bench.py" --config kitti-packnet-san --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing) > "$OUT/prof.log" 2>&1; rc=$?
echo "[prof] rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_trace.py "$OUT/prof/run_kernel_trace.csv" "$OUT/step_summary_san.txt" && head -40 "$OUT/step_summary_san.txt" | cut -c1-150
rm -rf "$OUT/prof"
