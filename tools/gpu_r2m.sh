#!/bin/bash
# K12 context-pair build: parity tests, A/B against the previous K12 (kbench), pack3d micro-bench,
# PackNetSAN01 KITTI bench (config 3) with a rocprof step summary
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r2m; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_hip_photometric.py tests/test_fisheye.py tests/test_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 "$OUT/tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/kbench.py --lib build/variants/k12_old.so --lib packnet-sfm-resnet-san_amd/libpsfm_hip.so --paths k12 > "$OUT/kbench.log" 2>&1; rc=$?
echo "[kbench] rc=$rc"; tail -6 "$OUT/kbench.log"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u tools/p3d_bench.py --iters 10 > "$OUT/p3d_packnet.log" 2>&1; rc=$?
echo "[p3d packnet] rc=$rc"; tail -14 "$OUT/p3d_packnet.log"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u tools/p3d_bench.py --iters 10 --net packnet-san > "$OUT/p3d_san.log" 2>&1; rc=$?
echo "[p3d san] rc=$rc"; tail -3 "$OUT/p3d_san.log"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 700 python bench.py --config kitti-packnet-san --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_san.json" 2> "$OUT/bench_san.err"; rc=$?
echo "[bench packnet-san] rc=$rc"; cat "$OUT/bench_san.json"; grep -v amdgpu.ids "$OUT/bench_san.err" | tail -3
exit 0
