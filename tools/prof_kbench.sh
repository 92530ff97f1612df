#!/bin/bash
# rocprofv3 passes over the photometric micro-bench: kernel trace, then SQ counters (separate pass).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/kprof
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$ROOT/tools/kbench.py" --iters 10 > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/sq" -o run --output-format csv -- python3 "$ROOT/tools/kbench.py" --iters 3 > "$OUT/sq.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS -d "$OUT/mem" -o run --output-format csv -- python3 "$ROOT/tools/kbench.py" --iters 3 > "$OUT/mem.log" 2>&1 || exit $?
echo done
