"""Build K12 source variants as separate libraries for an interleaved A/B with tools/kbench.py --lib:
each variant is a named list of exact-text edits of csrc/ (asserted to apply).
  python tools/k12_variants.py NAME [NAME ...]    -> build/k12var/k12_<NAME>.so"""
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

VARIANTS = {
    "base": [],
    # the context-paired camera record re-loaded (s_load) at each use instead of held in SGPRs
    "launder": [("psfm_fused.h", """        CamPair c;
        c.load(reinterpret_cast<cf2*>(reinterpret_cast<uint64_t>(campair)), H, W);
        return c;""", """        CamPair c;
        uint64_t rp = reinterpret_cast<uint64_t>(campair);
        asm volatile("" : "+s"(rp));
        c.load(reinterpret_cast<cf2*>(rp), H, W);
        return c;""")],
    # priority mode 2 only: no young / mode test around the high-priority setprio
    "prio2": [("psfm_fused.h", """        if (young && prio_mode == 1) __builtin_amdgcn_s_setprio(3);
        else __builtin_amdgcn_s_setprio(2);""", """        __builtin_amdgcn_s_setprio(2);""")],
}
VARIANTS["launder_prio2"] = VARIANTS["launder"] + VARIANTS["prio2"]
# ("FLAGS", extra hipcc flags) entries add compile flags instead of editing text
VARIANTS["noslp"] = [("FLAGS", "-fno-slp-vectorize")]
VARIANTS["noslp_launder"] = VARIANTS["noslp"] + VARIANTS["launder"]


def build(name):
    d = tempfile.mkdtemp(prefix=f"k12_{name}_", dir=os.path.join(ROOT, "build"))
    try:
        src = os.path.join(d, "csrc")
        shutil.copytree(os.path.join(ROOT, "packnet-sfm-resnet-san_amd", "csrc"), src)
        extra = [f for fn, f, _ in [(e[0], e[1], None) for e in VARIANTS[name]] if fn == "FLAGS"]
        for fn, old, new in [e for e in VARIANTS[name] if e[0] != "FLAGS"]:
            p = os.path.join(src, fn)
            s = open(p).read()
            assert old in s, (name, fn, old[:80])
            s = s.replace(old, new)
            open(p, "w").write(s)
        for f in os.listdir(src):
            p = os.path.join(src, f)
            txt = open(p).read()
            open(p, "w").write(txt.replace('"../../include/', '"' + os.path.join(ROOT, "include") + "/"))
        out = os.path.join(ROOT, "build", "k12var", f"k12_{name}.so")   # travels to the GPU box
        os.makedirs(os.path.dirname(out), exist_ok=True)
        import __graft_entry__ as G
        srcs = sorted(os.path.join(src, f) for f in os.listdir(src) if f.endswith(".hip"))
        r = subprocess.run(["/opt/rocm/bin/hipcc", *G.FLAGS, *extra, "-I", os.path.join(ROOT, "include"),
                            f'-DPSFM_SRC_HASH="variant-{name[:8]:8s}"', *srcs, "-o", out], capture_output=True, text=True)
        if r.returncode or os.path.getsize(out) < 1 << 20:
            raise RuntimeError(f"variant {name}: build failed rc={r.returncode}\n{r.stdout[-1500:]}\n{r.stderr[-2000:]}")
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(build, sys.argv[1:]):
            print(o)
