"""Timing probes / A-B variants (tools/build_k12_variant.sh name:WAVES:probe[+probe]): edits a COPY
of csrc/ (argument: that copy's psfm_fused.h; pack3d probes edit psfm_pack3d.hip beside it).
coal / nogath builds are for kbench timing only — their results are wrong by construction.

  coal   : every bilinear gather reads the lane's own column of rows 0/1 (perfect locality):
           how much of K12's time is gather latency / cache misses
  sgcam  : camera records kept in SGPRs across the sweep (no per-use s_load re-read)
  nogath : gathers replaced by constants (no vector-memory gathers at all)
  launder: the pinhole camera pair re-read through a laundered pointer at every use (s_load)
  noopq  : the sweep step index visible to the compiler (strength-reduced addresses)
  rb20   : band height 20 for every launch (the round-2 shape)
  rb40   : band height 40 for every launch (one wave per SIMD at B = 4, 192 x 640)
  p3dold : pack3d forward / MFMA dW on the round-3 3-D grids (no XCD grouping)
  fcpw2 / wcpwN : two / N 32-k chunks per workgroup in the pack3d forward / MFMA dW
  u8 / t1024 : netops row steps in flight per thread 8 / 1024 target workgroups
  prio   : K12 wave priority raised (s_setprio 2) over the issue phase, so its gathers go out first
  prioq  : ... and over the q-eval phase (LDS read-modify-write chain)   [adopted in the source]
  prior  : (on the adopted source) priority 2 also over the rotate + resolve of the step
  noprio : (on the adopted source) no wave priorities
"""
import os
import sys

path, probe = sys.argv[1], sys.argv[2]
if probe in ("p3dold", "fcpw2", "wcpw2", "wcpw4", "wcpw1"):
    path = os.path.join(os.path.dirname(path), "psfm_pack3d.hip")
if probe in ("u8", "t1024"):
    path = os.path.join(os.path.dirname(path), "psfm_netops.hip")
src = open(path).read()
if probe == "coal":
    old = "    const TapAddr t = tap_addr(ix, iy, H, W);\n#pragma unroll\n    for (int c = 0; c < 3; ++c) {\n        g.q[c][0]"
    new = ("    TapAddr t = tap_addr(ix, iy, H, W);\n    t.nw = threadIdx.x * 4u; t.ne = t.nw + 4u; t.sw = t.nw + (uint32_t)W * 4u; t.se = t.sw + 4u;\n"
           "#pragma unroll\n    for (int c = 0; c < 3; ++c) {\n        g.q[c][0]")
elif probe == "sgcam":
    old = "        uint64_t rp = reinterpret_cast<uint64_t>(campair);\n        asm volatile(\"\" : \"+s\"(rp));"
    new = "        uint64_t rp = reinterpret_cast<uint64_t>(campair);"
elif probe == "nogath":
    old = "        g.q[c][0] = ldg(img, c * pb + t.nw);\n        g.q[c][1] = ldg(img, c * pb + t.ne);\n        g.q[c][2] = ldg(img, c * pb + t.sw);\n        g.q[c][3] = ldg(img, c * pb + t.se);"
    new = ("        g.q[c][0] = __uint_as_float(t.nw) * 1e-30f;\n        g.q[c][1] = __uint_as_float(t.ne) * 1e-30f;\n"
           "        g.q[c][2] = __uint_as_float(t.sw) * 1e-30f;\n        g.q[c][3] = __uint_as_float(t.se) * 1e-30f;")
elif probe == "launder":
    old = "        CamPair c;\n        c.load(reinterpret_cast<cf2*>(reinterpret_cast<uint64_t>(campair)), H, W);"
    new = ("        uint64_t rp = reinterpret_cast<uint64_t>(campair);\n        asm volatile(\"\" : \"+s\"(rp));\n"
           "        CamPair c;\n        c.load(reinterpret_cast<cf2*>(rp), H, W);")
elif probe == "noopq":
    old = '        asm volatile("" : "+s"(k));\n'
    new = ""
elif probe == "rb20":
    old = "constexpr int RB_LO = 18, RB_HI = 28;"
    new = "constexpr int RB_LO = 20, RB_HI = 20;"
elif probe == "rb40":
    old = "constexpr int RB_LO = 18, RB_HI = 28;"
    new = "constexpr int RB_LO = 40, RB_HI = 40;"
elif probe == "p3dold":
    src = src.replace("grid = grid_lin(a, 4, 16, 32, P3D_FWD_CPW);", "")
    old = "grid = grid_lin(aw, 4, 16, 32, P3D_DW_CPW);"
    new = "grid = grid_of(aw, 4, 16, 32);"
elif probe == "fcpw2":
    old = "constexpr int P3D_FWD_CPW = 1;"
    new = "constexpr int P3D_FWD_CPW = 2;"
elif probe in ("wcpw1", "wcpw2", "wcpw4"):
    old = "constexpr int P3D_DW_CPW = 2;"
    new = "constexpr int P3D_DW_CPW = %s;" % probe[-1]
elif probe == "u8":
    old = "constexpr int U = 4;"
    new = "constexpr int U = 8;"
elif probe == "t1024":
    old = "constexpr int TARGET_BLOCKS = 512;"
    new = "constexpr int TARGET_BLOCKS = 1024;"
elif probe in ("prio", "prioq"):
    old = "        if (LOAD) {\n            const float sg = S.sg_next;"
    new = "        __builtin_amdgcn_s_setprio(2);\n        if (LOAD) {\n            const float sg = S.sg_next;"
    assert src.count(old) == 1
    src = src.replace(old, new)
    old = "        PSFM_PHASE();\n        if (PEVAL) peval<IA, IB, IC>(S, v - 2);"
    new = "        __builtin_amdgcn_s_setprio(0);\n        PSFM_PHASE();\n        if (PEVAL) peval<IA, IB, IC>(S, v - 2);"
    if probe == "prioq":
        assert src.count(old) == 1
        src = src.replace(old, new)
        old = "        PSFM_PHASE();\n        if (QEVAL) qeval<IA>(S, v - 3, k);\n        PSFM_PHASE();"
        new = "        PSFM_PHASE();\n        __builtin_amdgcn_s_setprio(2);\n        if (QEVAL) qeval<IA>(S, v - 3, k);\n        __builtin_amdgcn_s_setprio(0);\n        PSFM_PHASE();"
elif probe == "prior":
    old = "        if (QEVAL) qeval<IA>(S, v - 3, k);\n        __builtin_amdgcn_s_setprio(0);"
    new = "        if (QEVAL) qeval<IA>(S, v - 3, k);"
elif probe == "noprio":
    src = src.replace("        __builtin_amdgcn_s_setprio(2);\n", "").replace("        __builtin_amdgcn_s_setprio(0);\n", "")
    old = new = "__builtin_amdgcn_s_setprio"   # none left: count 0 -> assert below skipped
    open(path, "w").write(src)
    sys.exit(0)
else:
    sys.exit("unknown probe " + probe)
assert src.count(old) == 1, (probe, src.count(old))
open(path, "w").write(src.replace(old, new))
