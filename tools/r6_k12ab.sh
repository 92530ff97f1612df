#!/bin/bash
# K12 A/B (kbench, previous library vs in-tree) + the photometric GPU tests on the in-tree library.
# usage: tools/r6_k12ab.sh TAG OLD.so
set -u
TAG=$1; OLD=$2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u tools/kbench.py --paths k12 --reps 3 --iters 40 --lib "$OLD" ${EXTRA:-} \
  --lib packnet-sfm-resnet-san_amd/libpsfm_hip.so > "$OUT/kab.log" 2>&1; rc=$?
echo "[kab] rc=$rc"; grep K12 "$OUT/kab.log" | sed 's/"prepass".*"K12_photometric_fwd_grad"/K12/; s/, "finalize.*total_us"/ total/'
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_hip_photometric.py tests/test_fisheye.py tests/test_fisheye_camera.py \
  -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 "$OUT/tests.log"
exit $rc
