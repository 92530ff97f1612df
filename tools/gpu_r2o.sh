#!/bin/bash
# fused GroupNorm + ELU (PackNet Conv2D / ResidualConv): GPU tests, PackNet benches with it on / off
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2o; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -m gpu -q --timeout 250 --timeout-method thread > "$OUT/tests_trainer_alone.log" 2>&1; rc=$?
echo "[trainer alone] rc=$rc"; tail -3 "$OUT/tests_trainer_alone.log"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 500 python -u -m pytest tests/test_netops.py tests/test_networks.py tests/test_pack3d.py -m gpu -q --timeout 250 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 "$OUT/tests.log"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u tools/p3d_bench.py --iters 10 --lib build/variants/p3d_old.so --lib packnet-sfm-resnet-san_amd/libpsfm_hip.so > "$OUT/p3d_ab.log" 2>&1; rc=$?
echo "[p3d A/B packnet01] rc=$rc"; tail -2 "$OUT/p3d_ab.log" | cut -c1-400
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u tools/p3d_bench.py --iters 10 --net packnet-san --lib build/variants/p3d_old.so --lib packnet-sfm-resnet-san_amd/libpsfm_hip.so > "$OUT/p3d_ab_san.log" 2>&1; rc=$?
echo "[p3d A/B san] rc=$rc"; tail -2 "$OUT/p3d_ab_san.log" | cut -c1-400
case $rc in 124|134|137|139) exit $rc;; esac
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?
  echo "[$name] rc=$rc $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'])" "$OUT/$name.json" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -5 "$OUT/$name.err"; exit $rc; }
}
run san_gn --config kitti-packnet-san
run san_nogn --config kitti-packnet-san --fused-nets bias
run packnet01_gn --config kitti-packnet
run ddad_gn --config ddad-packnet-san
run resnet_default
