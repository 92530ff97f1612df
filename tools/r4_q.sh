#!/bin/bash
# Config-2 glue: attribute the MIOpen / ATen glue kernels to the ops launching them (eager step,
# torch.profiler), then bench A/B of MIOpen solver families whose solutions carry a zero-fill /
# cast (each variant with its own MIOpen user db, baseline twice).
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
MIOPEN_USER_DB_PATH=/tmp/udb_op timeout -k 10 300 python -u tools/op_profile.py --steps 3 --out "$OUT/op_profile.txt" > "$OUT/op_profile.log" 2>&1; rc=$?
echo "[op_profile] rc=$rc"; [ $rc -ne 0 ] && { tail -20 "$OUT/op_profile.log"; exit $rc; }
sed -n '/=== glue kernels/,$p' "$OUT/op_profile.txt" | head -40
run() {  # name, env assignments...
  local name=$1; shift
  env MIOPEN_USER_DB_PATH=/tmp/udb_$name "$@" timeout -k 10 240 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline \
    > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"; local rc=$?
  [ $rc -ne 0 ] && { echo "[bench $name] rc=$rc"; tail -5 "$OUT/bench_$name.err"; exit $rc; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$name.json'));print('$name', d['value'], d['ms_per_step'])"
}
run base
run no_asm_wrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
run no_ck_wrw MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS=0
run no_asm_bwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
run base2
run no_wrw_both MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_GROUP_CONV_IMPLICIT_GEMM_HIP_WRW_XDLOPS=0
exit 0
