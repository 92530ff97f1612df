#!/bin/bash
# Full -m gpu suite (one pytest process) + smoke() on the current tree.
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp MIOPEN_USER_DB_PATH=/tmp/miopen_udb MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p $MIOPEN_USER_DB_PATH $MIOPEN_CUSTOM_CACHE_DIR
cd "$ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread -rfE \
  > "$OUT/tests.log" 2>&1; rc=$?
echo "[tests] rc=$rc"; tail -3 "$OUT/tests.log"; grep -E "^(FAILED|ERROR)" "$OUT/tests.log" | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc2=$?
echo "[smoke] rc=$rc2"; tail -6 "$OUT/smoke.log"
exit $(( rc > rc2 ? rc : rc2 ))
