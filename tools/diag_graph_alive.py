"""Which object keeps the graph trainer's warm-up autograd graph alive into the capture (the
AccumulateGrad stream-mismatch warning)?  Weak references to the warm-up step's output tensors,
checked after the warm-up + gc.collect(); for survivors, the referrer chain."""
import gc
import os
import sys
import weakref

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
__graft_entry__.build()
import bench  # noqa: E402
from packnet_sfm_amd.trainers import ddp_trainer as T  # noqa: E402

dev = torch.device("cuda:0")


class A:
    depth_net, pose_net, batch, height, width = "ResNetSAN01", "PoseNet", 2, 64, 192


def describe(o):
    t = type(o).__name__
    if isinstance(o, dict):
        return f"dict keys={list(o.keys())[:8]}"
    if isinstance(o, (list, tuple)):
        return f"{t} len={len(o)}"
    return t + (f" {getattr(o, '__qualname__', '')}" if hasattr(o, '__qualname__') else "")


def chain(obj, depth=4, seen=None):
    seen = seen or set()
    if depth == 0:
        return
    for r in gc.get_referrers(obj):
        if id(r) in seen or r is sys._getframe() or isinstance(r, type(sys._getframe())):
            continue
        seen.add(id(r))
        print("  " * (5 - depth), "<-", describe(r), flush=True)
        chain(r, depth - 1, seen)


VARIANT = os.environ.get("DIAG_VARIANT", "default")
if VARIANT == "k1k2":
    from packnet_sfm_amd.losses import _hip_photometric as HP
    HP.FUSED_GRAD = False
torch.manual_seed(0)
m = bench.to_channels_last(bench.build_model(A, dev))
if VARIANT == "eager_upsample":
    m.lazy_upsample = False
if VARIANT == "serial_pose":
    m.overlap_pose_net = False
print("[diag] variant", VARIANT, flush=True)
tr = T.DDPTrainer(m, T.make_optimizer(m, 1e-4, 1e-4, capturable=True), dev, amp_dtype=None, graph=True)
b = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)
refs = []
orig = tr._forward_backward


def fb(batch, progress):
    out = orig(batch, progress)
    if not torch.cuda.is_current_stream_capturing():
        refs.append(("loss", weakref.ref(out["loss"])))
        inv = out["inv_depths"]
        for i, t in enumerate(getattr(inv, "stored", inv)):
            refs.append((f"inv{i}", weakref.ref(t)))
        for j, p in enumerate(out["poses"]):
            refs.append((f"pose{j}", weakref.ref(p.mat)))
    return out


tr._forward_backward = fb
orig_restore = tr._restore


def restore(snap):
    orig_restore(snap)
    gc.collect()
    alive = [(n, r()) for n, r in refs if r() is not None]
    print(f"[diag] after warm-up: {len(alive)} of {len(refs)} warm-up output tensors alive", flush=True)
    for n, t in alive[:3]:
        print(f"[diag] {n} grad_fn={type(t.grad_fn).__name__ if t.grad_fn is not None else None}", flush=True)
        chain(t)
    del alive


tr._restore = restore
import warnings  # noqa: E402
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    tr.train_step(b)
    torch.cuda.synchronize()
print("[diag] done; AccumulateGrad warnings:", sum("AccumulateGrad" in str(x.message) for x in w), flush=True)
