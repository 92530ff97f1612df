#!/bin/bash
# A/B of libpsfm_hip.so variants (build/variants/*.so, tools/build_variants.sh) on the K12 path.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
cd "$ROOT"
libs=""
for v in "$@"; do libs="$libs --lib build/variants/$v.so"; done
timeout -k 10 300 python tools/kbench.py --iters 20 --paths ${PATHS:-k12} $libs > "$OUT/kab.log" 2>&1; rc=$?
grep -v Warning "$OUT/kab.log" | grep "{" ; exit $rc
