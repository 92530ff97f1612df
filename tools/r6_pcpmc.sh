#!/bin/bash
# PMC passes (one counter group per run) of the composed pack layer's kernels k_pc_conv / k_pc_wgrad
# at the first PackNet01 pack layer, + the counter list of this box.  usage: tools/r6_pcpmc.sh TAG
set -u
TAG=$1; LIB=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
LIBARG=""; [ -n "$LIB" ] && LIBARG="--lib $ROOT/$LIB"
(for i in $(seq 1 60); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$ROOT/tools/pc_layer_run.py" --iters 3 $LIBARG > "$OUT/trace.log" 2>&1 || exit $?
i=0
for grp in "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "k_pc_conv|k_pc_wgrad" --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/pc_layer_run.py" --iters 1 $LIBARG > "$OUT/p$i.log" 2>&1; rc=$?
  echo "[pass $i] rc=$rc"
  crash $rc && exit $rc
done
exit 0
