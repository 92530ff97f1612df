#!/bin/bash
# rocprofv3 kernel statistics of the composed pack layer (tools/pc_layer_run.py) for each given library.
# usage: tools/r6_pcprof.sh TAG LIB...
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG; rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d "$OUT/l$i" -o run -- python3 "$ROOT/tools/pc_layer_run.py" --iters 5 --lib "$ROOT/$lib" > "$OUT/l$i.log" 2>&1; rc=$?
  echo "[lib $i: $lib] rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  f=$(find "$OUT/l$i" -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'   {r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
done
exit 0
