#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over the first PackNet01 pack layer's fused
# Conv3d fwd / dx / dW (tools/p3d_bench.py --only pack64x192x640).  OUT=gpurun_out/<tag>.
set -u
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 60); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/p3d_bench.py" --only ${ONLY:-pack64x192x640} --iters 3 > "$OUT/p$i.log" 2>&1; rc=$?
  echo "[pass $i] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
  f=$(find "$OUT/p$i" -name '*counter_collection.csv' | head -1); [ -n "$f" ] && cp "$f" "$OUT/counters_$i.csv"; rm -rf "$OUT/p$i"
done
exit 0
