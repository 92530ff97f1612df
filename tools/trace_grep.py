"""Compact view of a rocprofv3 kernel_trace.csv: the rows whose kernel name matches REGEX, as
name, grid (workgroups), queue, start / end (ns, relative to the first row), duration (us).

  python tools/trace_grep.py run_kernel_trace.csv REGEX out.csv [--last-steps K --step-regex R]

--last-steps K keeps only rows after the K-th last launch of the kernel matching --step-regex (one
launch per training step, e.g. K12), so the file holds the final K steps' timelines."""
import argparse
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("regex")
ap.add_argument("out")
ap.add_argument("--last-steps", type=int, default=0)
ap.add_argument("--step-regex", default="k12_fwd_grad")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if a.last_steps:
    marks = [i for i, r in enumerate(rows) if re.search(a.step_regex, r["Kernel_Name"])]
    if len(marks) > a.last_steps:
        # from the end of the step before the kept ones
        rows = rows[marks[-a.last_steps - 1] + 1:]
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
pat = re.compile(a.regex)
with open(a.out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["name", "grid_wg", "wg_size", "queue", "start_ns", "end_ns", "dur_us"])
    for r in rows:
        name = r["Kernel_Name"]
        if not pat.search(name):
            continue
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(wg, 1)
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        w.writerow([name[:120], grid, wg, r["Queue_Id"], s, e, round((e - s) / 1000, 2)])
