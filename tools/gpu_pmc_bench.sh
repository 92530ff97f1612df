#!/bin/bash
# PMC passes over bench.py for one config -> profiles/pmc/<config_key>.json (tools/pmc_bench.py).
# One rocprofv3 run per counter group (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass; at most
# 8 SQ counters per pass).  Stops at the first crash-like exit.
# usage: tools/gpu_pmc_bench.sh [bench.py args...]   (PMC_EXTRA: more bench args for the passes only,
# e.g. --no-miopen-find: on a fresh box MIOpen's find compiles every candidate convolution kernel
# under the profiler, which took a PackNet pass past 5 minutes; this library's kernels, the only
# ones counted, do not depend on the convolution solvers)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
KEY=$(cd "$ROOT" && python3 -c "import sys, bench; print(bench.config_key(bench.parse(sys.argv[1:])))" "$@")
OUT=$ROOT/gpurun_out/pmc/$KEY
rm -rf "$OUT"; mkdir -p "$OUT"
echo "[pmc] config $KEY"
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  # counters on this library's kernels only (PMC_ALL=1: every kernel): MIOpen's find and the
  # convolutions run uninstrumented, so a PackNet pass fits its time limit
  filt="--kernel-include-regex (k12_fwd_grad|k0_unwarped|k_sig_sum|k_finalize|k_grad_finish|k_pose_reduce|k_p3d_|k_gn_|k_gnp_|k_gnr_|k_bnr_|k_pc_|k_bias_act|k_adam|k_upcat|k_cols_finish)"
  [ "${PMC_ALL:-0}" = 1 ] && filt=""
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp $filt --output-format csv -d "$OUT/p$i" -o run \
     -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 --no-cpu-baseline --no-kernel-timing ${PMC_EXTRA:-} "$@") > "$OUT/p$i.log" 2>&1; rc=$?
  echo "[pmc pass $i: $grp] rc=$rc"; tail -2 "$OUT/p$i.log"
  crash $rc && exit $rc
  [ $rc -ne 0 ] && exit $rc
done
python3 "$ROOT/tools/pmc_bench.py" "$KEY" "$OUT/$KEY.json" "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 && rm -rf "$OUT"/p1 "$OUT"/p2 "$OUT"/p3
