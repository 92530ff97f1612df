#!/bin/bash
# A/B of MIOpen solver restrictions on the bench step (each variant its own process).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/miopen; mkdir -p "$OUT"
cd "$ROOT"
run() {  # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --no-cpu-baseline --no-kernel-timing > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?; echo "[$name] rc=$rc $(cat "$OUT/$name.json")"
  case $rc in 124|134|137|139) exit $rc;; esac
}
for v in "$@"; do
  case $v in
    base) run base X=1 ;;
    nowrw) run nowrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 ;;
    nowrwbwd) run nowrwbwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 ;;
    noasm) run noasm MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 ;;
  esac
done
