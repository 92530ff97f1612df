#!/bin/bash
# pack3d A/B on one box: tools/p3d_bench.py over build/variants/<name>.so (interleaved twice), both
# nets; optional pack3d GPU tests of the in-tree build first (TESTS=1).  OUT=gpurun_out/<tag>.
#   tools/r3_p3dab.sh <tag> name1 name2 ...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 80); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
cd "$ROOT"
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests/test_pack3d.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests_pack3d.log" 2>&1; rc=$?
  echo "[tests] rc=$rc"; tail -2 "$OUT/tests_pack3d.log"; [ $rc -ne 0 ] && exit $rc
fi
libs=""
for rep in 1 2; do for n in "$@"; do libs="$libs --lib build/variants/$n.so"; done; done
for net in packnet packnet-san; do
  timeout -k 10 400 python -u tools/p3d_bench.py --net $net $libs > "$OUT/p3d_$net.log" 2>&1; rc=$?
  echo "[p3d $net] rc=$rc"; grep -o '^build[^ ]* {"pack[^]]*\]' "$OUT/p3d_$net.log"; grep -o 'build[^ ]*\|"total[^]]*\]' "$OUT/p3d_$net.log" | paste - - ; [ $rc -ne 0 ] && exit $rc
done
exit 0
