"""Stamp a rocprofv3 kernel-trace step summary for bench.py's roofline: K12's mean in-step
dispatch-to-completion duration (tools/summarize_trace.py output of a tools/r5_bench.sh --prof run)
-> profiles/rocprof/<config_key>.json with the library's source hash (bench.py ignores a stale one).
  python tools/rocprof_stamp.py STEP_SUMMARY.txt --config kitti-resnet-san"""
import argparse
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("--config", required=True)
    a = ap.parse_args()
    import bench
    args = bench.parse(["--config", a.config])
    txt = open(a.summary).read()
    m = re.search(r"^\s*([\d.]+) us/step\s+n/step=\s*([\d.]+)\s+[^\n]*?k12_fwd_grad", txt, re.M)
    if not m:
        raise SystemExit("no k12_fwd_grad row in " + a.summary)
    us, n = float(m.group(1)), float(m.group(2))
    out = {"config_key": bench.config_key(args), "source_hash": bench.source_hash(),
           "k12_us_mean": round(us / n, 2), "k12_launches_per_step": n,
           "summary": os.path.relpath(os.path.abspath(a.summary), ROOT),
           "note": "rocprofv3 --kernel-trace of bench.py on this config, mean K12 duration per launch inside the "
                   "replayed step graph (dispatch to completion)"}
    d = os.path.join(ROOT, "profiles", "rocprof")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, out["config_key"] + ".json"), "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
