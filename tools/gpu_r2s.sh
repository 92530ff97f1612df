#!/bin/bash
# pack3d forward (thread = pixel x 8 k, 16-byte stores) + generic kernels without spills: parity
# tests, A/B against the previous build, PackNet benches
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2s; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_pack3d.py -m gpu -q --timeout 250 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
echo "[pack3d tests] rc=$rc"; tail -2 "$OUT/tests.log"
[ $rc -ne 0 ] && exit $rc
for net in packnet packnet-san; do
  timeout -k 10 300 python -u tools/p3d_bench.py --iters 10 --net $net --lib build/variants/p3d_prev.so --lib packnet-sfm-resnet-san_amd/libpsfm_hip.so > "$OUT/p3d_ab_$net.log" 2>&1; rc=$?
  echo "[p3d A/B $net] rc=$rc"; grep -o '"total_fwd_bwdx_bwdw_us": \[[^]]*\]' "$OUT/p3d_ab_$net.log"
  case $rc in 0) ;; *) exit $rc;; esac
done
for cfg in kitti-packnet kitti-packnet-san; do
  timeout -k 10 500 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err"; rc=$?
  echo "[bench $cfg] rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" "$OUT/bench_$cfg.json" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -5 "$OUT/bench_$cfg.err"; exit $rc; }
done
