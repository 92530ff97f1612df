#!/usr/bin/env python3
"""Per-phase VALU instruction counts of K12's main sweep loop, from the gfx950 ISA.

Compiles csrc/psfm_photometric.hip to device assembly, takes k12_fwd_grad<2, true, PINHOLE>
(the training default), finds its main loop (the longest backward branch: 4 unrolled sweep steps)
and splits it at the sched_barrier markers (PSFM_PHASE between issue | p-eval | q-eval | resolve,
PSFM_CHAN between the SSIM channels).  Prints VALU / packed / DPP / memory counts per phase.
  python tools/isa_phases.py [--kernel NAME]
"""
import argparse
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default=None, help="mangled name (default: the first k12_fwd_grad<2, true, 0, RB>)")
ap.add_argument("--classes", action="store_true", help="per-step instruction classes of the whole loop")
ap.add_argument("--dump", default=None, help="write the main loop's assembly here")
ap.add_argument("--root", default=ROOT, help="tree whose csrc/ to compile (A/B against another checkout)")
a = ap.parse_args()
with tempfile.TemporaryDirectory() as d:
    s = os.path.join(d, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                    "-fno-slp-vectorize", "-I", os.path.join(a.root, "include"),   # the TU's build flags (TU_FLAGS)
                    os.path.join(a.root, "packnet-sfm-resnet-san_amd", "csrc", "psfm_photometric.hip"), "-o", s],
                   check=True, capture_output=True)
    lines = open(s).read().split("\n")
if a.kernel is None:
    a.kernel = next(m.group(1) for ln in lines if (m := re.match(r"^(_ZN4psfm5fused12k12_fwd_gradILi2ELb1ELi0ELi18E\w*):", ln)))
start = next(i for i, ln in enumerate(lines) if ln.startswith(a.kernel + ":"))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
lab = {m.group(1): i for i, ln in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", ln))}
loops = []
for i, ln in enumerate(body):
    m = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", ln)
    if m and m.group(2) in lab and lab[m.group(2)] < i:
        loops.append((i - lab[m.group(2)], lab[m.group(2)], i))
_, lo, hi = max(loops)
if a.dump:
    open(a.dump, "w").write("\n".join(body[lo:hi + 1]) + "\n")
phases, cur = [], []
for ln in body[lo:hi + 1]:
    if "sched_barrier" in ln:
        phases.append(cur)
        cur = []
    else:
        cur.append(ln.strip())
phases.append(cur)
tot = 0
print(f"{a.kernel}: main loop {hi - lo + 1} lines, {len(phases)} segments between sched_barriers (4 sweep steps)")
for k, ph in enumerate(phases):
    if len(ph) < 4:
        continue
    v = sum(ln.startswith("v_") and not ln.startswith(("v_readlane", "v_writelane")) for ln in ph)
    pk = sum(ln.startswith("v_pk_") for ln in ph)
    dpp = sum(("row_" in ln or "quad_perm" in ln) for ln in ph)
    mem = sum(ln.startswith(("global_load", "buffer_load", "ds_", "s_load", "global_store")) for ln in ph)
    tot += v
    print(f"  segment {k:2d}: VALU {v:4d} (v_pk {pk:3d}, DPP {dpp:3d})  memory {mem:3d}")
print(f"  loop total VALU {tot} = {tot / 4:.0f} per sweep step (one issued row of 64 lanes)")

if a.classes:
    # every instruction of the 4-step loop by class, per sweep step; issue-cycle weights for a wave64
    # (MI355X_MICROARCH.md: VALU 2 cycles at two waves / 4 alone, s_nop N = N+1 wait states)
    ins = [ln.split()[0] for ln in (x.strip() for x in body[lo:hi + 1]) if ln and not ln.startswith((";", ".", "s_nop")) and not ln.endswith(":")]
    nops = [int(m.group(1)) + 1 for ln in body[lo:hi + 1] if (m := re.match(r"\s*s_nop\s+(\d+)", ln))]
    cls = {}

    def add(k):
        cls[k] = cls.get(k, 0) + 1
    for op in ins:
        if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
            add("v_readlane/writelane")
        elif op.startswith("v_mov"):
            add("v_mov")
        elif op.startswith("v_pk_"):
            add("v_pk (packed f32)")
        elif op.startswith("v_cndmask"):
            add("v_cndmask")
        elif op.startswith("v_"):
            add("VALU other")
        elif op.startswith("ds_read") or op.startswith("ds_load"):
            add("ds_read")
        elif op.startswith("ds_write") or op.startswith("ds_store"):
            add("ds_write")
        elif op.startswith("ds_"):
            add("ds_other")
        elif op.startswith(("global_load", "buffer_load")):
            add("vmem load")
        elif op.startswith(("global_store", "buffer_store")):
            add("vmem store")
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            add("smem load")
        elif op.startswith("s_waitcnt"):
            add("s_waitcnt")
        elif op.startswith(("s_setprio", "s_barrier", "s_sleep")):
            add("s_setprio/barrier")
        elif op.startswith(("s_cbranch", "s_branch")):
            add("branch")
        elif op.startswith("s_"):
            add("SALU")
        else:
            add("other " + op)
    dpp = sum(("row_" in ln or "quad_perm" in ln or "row_bcast" in ln) for ln in body[lo:hi + 1])
    waits = [ln.strip() for ln in body[lo:hi + 1] if ln.strip().startswith("s_waitcnt")]
    lgkm = sum("lgkmcnt" in w for w in waits)
    vm = sum("vmcnt" in w for w in waits)
    print("per sweep step (loop / 4):")
    for k, v in sorted(cls.items(), key=lambda kv: -kv[1]):
        print(f"  {k:24s} {v / 4:7.1f}")
    print(f"  {'s_nop (instructions)':24s} {len(nops) / 4:7.1f}   wait states {sum(nops) / 4:.1f}")
    print(f"  {'DPP-modified VALU':24s} {dpp / 4:7.1f}")
    print(f"  s_waitcnt with lgkmcnt {lgkm / 4:.1f}, with vmcnt {vm / 4:.1f}")
