"""Which library build changes the fisheye multi-resolution gradients: the fisheye_small multires
golden case through several libpsfm_hip.so builds (--lib), dL/dsig per scale vs the golden and vs the
first build (the pixels that differ and by how much)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", action="append", default=[])
ap.add_argument("--tag", default="_multires")
a = ap.parse_args()
import __graft_entry__  # noqa: E402
__graft_entry__.build()
import golden_util as gu  # noqa: E402
from packnet_sfm_amd import _hip  # noqa: E402
import test_fisheye as TF  # noqa: E402

z = gu.load_golden("fisheye_small")
dev = torch.device("cuda:0")
first = None
for lib in a.lib or [None]:
    if lib:
        _hip.LIB_PATH = lib
        _hip._lib = None
    out, sigs, vec = TF._run(z, a.tag, dev)
    gs = [s.grad.cpu() for s in sigs]
    print(f"== {lib or 'in-tree'}: loss {float(out['loss']):.9f}")
    for i, g in enumerate(gs):
        ok, msg = gu.grad_check(g, z[f"grad_sig{i}{a.tag}"], None, TF.GRAD_TOL)
        line = f"  dsig{i}: {'ok' if ok else 'FAIL'} {msg}"
        if first is not None:
            d = (g - first[i]).abs()
            n = int((d > 0).sum())
            line += f" | vs first build: {n} px differ, max {float(d.max()):.3e}"
            if n:
                idx = torch.nonzero(d > 1e-3 * float(first[i].abs().max()))[:5].tolist()
                line += f" big at {idx}"
        print(line, flush=True)
    if first is None:
        first = gs
