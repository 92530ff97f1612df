#!/bin/bash
# K12 wave-cycle attribution: counter passes (one group per run) over the K12 micro-bench, plus the
# counter list of this box.  usage: tools/r5_k12pmc.sh TAG
set -u
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
(for i in $(seq 1 60); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_INSTS_SENDMSG SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "k12_fwd_grad" --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/kbench.py" --iters 2 --paths k12 > "$OUT/p$i.log" 2>&1; rc=$?
  echo "[pass $i] rc=$rc $(grep -c k12_fwd_grad $OUT/p$i/run_counter_collection.csv 2>/dev/null)"
  crash $rc && exit $rc
done
exit 0
