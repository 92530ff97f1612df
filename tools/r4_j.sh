#!/bin/bash
# K12 variant A/B (kbench over build/variants/*.so, interleaved) + photometric GPU tests on the tree's
# library + the attribution of the capture crash to torch's own op chain (last: it may crash).
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_hip_photometric.py tests/test_fisheye.py -m gpu -q --timeout 300 \
  --timeout-method thread -rfE > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -2 "$OUT/tests.log"; grep -E "^(FAILED|ERROR)" "$OUT/tests.log" | head
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
libs=""; for rep in 1 2 3; do for n in "$@"; do libs="$libs --lib build/variants/$n.so"; done; done
for B in 4 6; do
  timeout -k 10 400 python -u tools/kbench.py --paths k12 --iters 50 --B $B $libs > "$OUT/kbench_b$B.log" 2>&1; rc=$?
  echo "[kbench B=$B] rc=$rc"; grep -v "^\[\|amdgpu" "$OUT/kbench_b$B.log" | cut -c1-120; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python -u tools/diag_gn_capture.py --capture-bwd --torch-chain > "$OUT/cap_torch.log" 2>&1; rc=$?
echo "[capture bwd, torch chain] rc=$rc"; grep -v amdgpu.ids "$OUT/cap_torch.log" | tail -4
exit 0
