#!/bin/bash
# pack3d suite on the default dx forms, then the DDAD K12 traffic experiment.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 560 python -u -m pytest tests/test_pack3d.py -m gpu -q -x --timeout 500 --timeout-method thread -rfE -s \
  > "$OUT/p3d_tests.log" 2>&1; rc=$?
echo "[p3d tests] rc=$rc"; tail -2 "$OUT/p3d_tests.log"; grep "^mode" "$OUT/p3d_tests.log"
[ $rc -ne 0 ] && exit $rc
bash tools/r4_k.sh ${TAG}_ddad || exit 1
