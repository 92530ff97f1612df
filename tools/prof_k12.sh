#!/bin/bash
# SQ counter passes over the K12 photometric micro-bench (one pass per counter group).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/k12prof
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM_NORM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "(k12_fwd_grad|k0_unwarped|k_sig_sum|k_finalize|k_grad_finish|k_pose_reduce)" --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/kbench.py" --iters 2 --paths ${PATHS:-k12} > "$OUT/p$i.log" 2>&1; rc=$?
  echo "[pass $i] rc=$rc"; crash $rc && exit $rc
done
exit 0
