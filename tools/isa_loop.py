#!/usr/bin/env python3
"""Instruction classes of a kernel's longest loop, from the gfx950 ISA of one csrc/*.hip file.
  python tools/isa_loop.py FILE.hip KERNEL_REGEX [--dump OUT.s] [--flags "..."]"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("kernel")
ap.add_argument("--dump", default=None)
ap.add_argument("--flags", default="")
a = ap.parse_args()
with tempfile.TemporaryDirectory() as d:
    s = os.path.join(d, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                    *a.flags.split(), "-I", os.path.join(ROOT, "include"), a.src, "-o", s], check=True)
    lines = open(s).read().split("\n")
name = next(m.group(1) for ln in lines if (m := re.match(r"^(_Z\w+):", ln)) and re.search(a.kernel, m.group(1)))
start = next(i for i, ln in enumerate(lines) if ln.startswith(name + ":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
lab = {m.group(1): i for i, ln in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", ln))}
loops = [(i - lab[m.group(2)], lab[m.group(2)], i) for i, ln in enumerate(body)
         if (m := re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", ln)) and m.group(2) in lab and lab[m.group(2)] < i]
_, lo, hi = max(loops)
loop = [x.strip() for x in body[lo:hi + 1]]
if a.dump:
    open(a.dump, "w").write("\n".join(loop) + "\n")
c = collections.Counter()
for ln in loop:
    if not ln or ln.startswith((";", ".")) or ln.endswith(":"):
        continue
    op = ln.split()[0]
    k = ("mfma" if "mfma" in op else "v_pk" if op.startswith("v_pk") else "VALU" if op.startswith("v_") else
         "ds_read" if op.startswith(("ds_read", "ds_load")) else "ds_write" if op.startswith(("ds_write", "ds_store")) else
         "vmem" if op.startswith(("global_", "buffer_")) else "smem" if op.startswith("s_load") else
         "waitcnt" if op.startswith("s_waitcnt") else "nop" if op.startswith("s_nop") else "SALU" if op.startswith("s_") else op)
    c[k] += 1
print(name, f"loop lines {hi - lo + 1}:", dict(c.most_common()))
