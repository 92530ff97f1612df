#!/bin/bash
# GroupNorm A/B: tools/gn_bench.py --eager (each PackNet01 GN shape, fwd and bwd) under rocprofv3
# --kernel-trace --stats per library variant -> per-kernel GPU time totals (host overhead excluded).
#   tools/r3_gnab.sh <tag> name1 name2 ...     (build/variants/<name>.so)
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
(for i in $(seq 1 60); do date >> "$OUT/heartbeat.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
for rep in 1 2; do
  for v in "$@"; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p_$v" -o run --output-format csv \
       -- python3 "$ROOT/tools/gn_bench.py" --depth-net ${NET:-PackNet01} --eager --iters 10 --lib "$ROOT/build/variants/$v.so") > "$OUT/gn_$v.log" 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "[$v] rc=$rc"; tail -5 "$OUT/gn_$v.log"; exit $rc; }
    f=$(find "$OUT/p_$v" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = {}
for r in rows:
    n = r["Name"]
    if "k_gn_" in n:
        k = n.split("<")[0].split("::")[-1]
        tot[k] = tot.get(k, 0.0) + float(r["TotalDurationNs"]) / 1e3
print(sys.argv[2], {k: round(v, 1) for k, v in sorted(tot.items())}, "sum_us", round(sum(tot.values()), 1))
PY
    rm -rf "$OUT/p_$v"
  done
done
exit 0
