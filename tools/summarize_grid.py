"""Summarise a rocprofv3 kernel-trace CSV by (kernel, grid): average duration per launch."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2].split(",") if len(sys.argv) > 2 else None
agg = collections.defaultdict(lambda: [0, 0])
for r in rows:
    name = r["Kernel_Name"]
    if pat and not any(p in name for p in pat):
        continue
    grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
    short = re.sub(r"\(anonymous namespace\)::", "", name).replace("void ", "").split("(")[0][-48:]
    a = agg[(short, int(grid) if str(grid).isdigit() else grid)]
    a[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    a[1] += 1
for (k, gsz), v in sorted(agg.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
    print(f"{v[0] / 1e3 / v[1]:8.2f} us  n={v[1]:5d}  grid={gsz!s:>8}  {k}")
