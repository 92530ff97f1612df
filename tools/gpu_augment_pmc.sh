#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per pass) over the augment micro-bench; per-call
# traffic of the three augment kernels -> gpurun_out/augment/pmc_traffic.json
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/augment; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$OUT/pmc_$ctr"
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc_$ctr" -o run -- python3 "$ROOT/tools/augment_bench.py" --iters 10 --no-cpu-baseline > "$OUT/pmc_$ctr.log" 2>&1; rc=$?
  echo "[pmc $ctr] rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
res = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{out}/pmc_{ctr}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if "resize" in n or "jitter" in n:
                acc[n].append(float(r["Counter_Value"]))
    res[ctr] = {k: sum(v) / len(v) for k, v in acc.items()}
fetch = sum(res["FETCH_SIZE"].values()) * 1024
write = sum(res["WRITE_SIZE"].values()) * 1024
res["per_call_bytes"] = {"fetch_raw": fetch, "fetch_x2_gfx950": 2 * fetch, "write": write,
                         "traffic": 2 * fetch + write}
json.dump(res, open(f"{out}/pmc_traffic.json", "w"), indent=1)
print(json.dumps(res["per_call_bytes"]))
PY
