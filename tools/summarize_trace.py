"""Summarise a rocprofv3 kernel-trace CSV of bench.py: steady-state per-step kernel time by name
(steps delimited by the K1 launches of the last N steps).  Writes a small text summary."""
import collections
import csv
import sys

trace, out = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# steps are delimited by the fused Adam launch (once per training step; bench.py's photometric
# kernel timing replays after the timed steps launch K12 but never Adam)
names = {r["Kernel_Name"] for r in rows}
key = next(k for k in ("k_adam", "k12_fwd_grad", "k1_forward") if any(k in n for n in names))
k1 = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
lines = [f"rows {len(rows)}  k1 launches {len(k1)}"]
if len(k1) >= 3:
    n = min(len(k1) - 1, 8)  # the last graph replays only (warm-up includes MIOpen find)
    i0, i1 = k1[-n - 1], k1[-1]
    t0, t1 = int(rows[i0]["Start_Timestamp"]), int(rows[i1]["Start_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    busy = 0
    for r in rows[i0:i1]:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy += d
        a = agg[r["Kernel_Name"][:110]]
        a[0] += d
        a[1] += 1
    lines.append(f"steps {n}  wall ms/step {(t1 - t0) / 1e6 / n:.3f}  busy ms/step {busy / 1e6 / n:.3f}  "
                 f"kernels/step {(i1 - i0) / n:.1f}")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:60]:
        lines.append(f"{v[0] / 1e3 / n:9.1f} us/step  n/step={v[1] / n:6.1f}  {k}")
    # normalisation / epilogue kernels by launch grid (one line per layer shape)
    pat = ("k_bn_", "k_gn_", "k_bias_act", "MIOpenBatchNorm", "RowwiseMoments", "ComputeInternalGradients")
    bygrid = collections.defaultdict(lambda: [0, 0])
    for r in rows[i0:i1]:
        name = r["Kernel_Name"]
        if any(p in name for p in pat):
            grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
            b = bygrid[(name.split("(")[0][-40:], grid)]
            b[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            b[1] += 1
    if bygrid:
        lines.append("--- normalisation / epilogue kernels by grid (avg us per launch, launches/step) ---")
        for (k, gsz), v in sorted(bygrid.items(), key=lambda kv: (kv[0][0], -kv[1][0])):
            lines.append(f"{v[0] / 1e3 / v[1]:8.2f} us  x{v[1] / n:4.1f}  grid={gsz:>8}  {k}")
    # timeline of the last step: start offset, duration, queue, gap to the previous kernel's end
    # (any queue) -- where the step waits on the host or on a cross-stream dependency
    lines.append("--- last step timeline (us: start, dur, idle-before, queue, kernel) ---")
    j0 = k1[-2]
    t0 = int(rows[j0]["Start_Timestamp"])
    last_end = t0
    idle = 0
    for r in rows[j0:i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(0, s - last_end)
        idle += gap
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        lines.append(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap / 1e3:7.1f}  q{q:>3}  "
                     f"{r['Kernel_Name'][:90]}")
        last_end = max(last_end, e)
    lines.append(f"idle (no kernel running) in last step: {idle / 1e3:.1f} us")
open(out, "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:3]))
