#!/bin/bash
# One GPU cycle of round 6: K12 A/B (previous library vs in-tree), the full -m gpu suite + smoke(),
# the --comm auto probe at N = 1 over RCCL with the bench model's shapes.  usage: tools/r6_cycle.sh TAG [OLD.so]
set -u
TAG=$1; OLD=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$OLD" ]; then
  timeout -k 10 300 python -u tools/kbench.py --paths k12 --reps 3 --iters 40 --lib "$OLD" \
    --lib packnet-sfm-resnet-san_amd/libpsfm_hip.so > "$OUT/kab.log" 2>&1; rc=$?
  echo "[kab] rc=$rc"; grep K12 "$OUT/kab.log" | sed 's/"prepass".*"K12_photometric_fwd_grad"/K12/; s/, "finalize.*total_us"/ total/'
  [ $rc -ne 0 ] && exit $rc
fi
bash tools/r4_suite.sh "$TAG/suite"; rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --gpus 1 --comm auto --probe-backend nccl --probe-only > "$OUT/probe_n1.json" 2> "$OUT/probe_n1.err"; rc2=$?
echo "[probe] rc=$rc2"; grep "comm probe" "$OUT/probe_n1.err" | tail -2; cat "$OUT/probe_n1.json"
exit $rc
