#!/bin/bash
# K12 XCD dealing by image parts (sweep::work_item_parts): photometric parity, kbench timing and
# FETCH_SIZE at 192x640 (B = 4, 6) and 384x640 (B = 4) with PSFM_K12_PARTS=1 (old dealing) vs auto.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_hip_photometric.py -m gpu -q -x --timeout 400 --timeout-method thread -rfE \
  > "$OUT/photometric_tests.log" 2>&1; rc=$?
echo "[photometric tests] rc=$rc"; tail -2 "$OUT/photometric_tests.log"
[ $rc -ne 0 ] && exit $rc
for cfg in "4 192" "6 192" "4 384"; do
  set -- $cfg
  for P in 1 auto 1 auto; do
    if [ $P = auto ]; then unset PSFM_K12_PARTS; else export PSFM_K12_PARTS=$P; fi
    timeout -k 10 120 python -u tools/kbench.py --paths k12 --B $1 --H $2 --iters 20 > "$OUT/kb_$1_$2_$P.log" 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "[kbench $cfg P=$P] rc=$rc"; tail -5 "$OUT/kb_$1_$2_$P.log"; exit $rc; }
    echo "B=$1 H=$2 P=$P $(tail -1 "$OUT/kb_$1_$2_$P.log" | cut -c1-250)"
  done
done
unset PSFM_K12_PARTS
cd /tmp
for cfg in "4 384" "4 192"; do
  set -- $cfg
  for P in 1 auto; do
    if [ $P = auto ]; then unset PSFM_K12_PARTS; else export PSFM_K12_PARTS=$P; fi
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k12_fwd_grad --output-format csv -d "$OUT/p_$1_$2_$P" -o run \
      -- python3 "$ROOT/tools/kbench.py" --paths k12 --B $1 --H $2 --iters 3 > "$OUT/p_$1_$2_$P.log" 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "[pmc $cfg P=$P] rc=$rc"; tail -5 "$OUT/p_$1_$2_$P.log"; exit $rc; }
    python3 - "$OUT/p_$1_$2_$P" $2 "B=$1 H=$2 P=$P" <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
v = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == "FETCH_SIZE"]
H = int(sys.argv[2]); alg = H * 640 * 120 * 4
fb = sorted(v)[len(v) // 2] * 2 * 1024 if v else float("nan")
print(f"{sys.argv[3]}: K12 read bytes per launch {fb/1e6:.1f} MB = {fb/alg:.2f}x algorithmic")
PY
    rm -rf "$OUT/p_$1_$2_$P"
  done
done
unset PSFM_K12_PARTS
exit 0
