"""Where do the graph-replayed and eager bf16 steps differ?  Per-parameter relative gradient
differences of (graph vs eager), (eager vs eager) and (graph vs graph: two graph trainers), the
largest first — a systematic difference shows up as parameters far above the eager noise."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import __graft_entry__  # noqa: E402

__graft_entry__.build()
import bench  # noqa: E402
from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer  # noqa: E402
from test_trainer_gpu import _build, _grads  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False
b = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)


def static():
    return {k: (v.clone() if torch.is_tensor(v) else [c.clone() for c in v]) for k, v in b.items()}


def graph_grads():
    m = _build(dev)
    t = DDPTrainer(m, make_optimizer(m, 1e-4, 1e-4), dev, amp_dtype=torch.bfloat16, graph=True, bf16_weights=True)
    out = t.train_step(static())
    torch.cuda.synchronize()
    return float(out["loss"]), _grads(m)


def eager_grads(n=2):
    m = _build(dev)
    t = DDPTrainer(m, make_optimizer(m, 1e-4, 1e-4), dev, amp_dtype=torch.bfloat16, graph=False, flat=True,
                   bf16_weights=True, fused_optim=True)
    res = []
    for _ in range(n):
        t._zero_grad()
        out = t._forward_backward(b, 0.0)
        torch.cuda.synchronize()
        res.append((float(out["loss"]), _grads(m)))
    return res


lg1, g1 = graph_grads()
lg2, g2 = graph_grads()
(le1, e1), (le2, e2) = eager_grads()
print(f"loss graph {lg1:.7f} {lg2:.7f} eager {le1:.7f} {le2:.7f}")


def rel(a, c):
    out = {}
    for (n, x), (_, y) in zip(a, c):
        if x is not None and y is not None:
            out[n] = float((x - y).norm() / y.norm().clamp_min(1e-30))
    return out


pairs = {"graph-eager": rel(g1, e1), "eager-eager": rel(e2, e1), "graph-graph": rel(g2, g1),
         "graph2-eager2": rel(g2, e2)}
for k, v in pairs.items():
    s = sorted(v.values())
    print(f"{k:14s} median {s[len(s) // 2]:.3e}  p90 {s[int(len(s) * 0.9)]:.3e}  max {s[-1]:.3e}")
ge, ee = pairs["graph-eager"], pairs["eager-eager"]
print("largest graph-eager / eager-eager ratios:")
for n in sorted(ge, key=lambda n: -ge[n] / max(ee[n], 1e-12))[:25]:
    print(f"  {n:60s} graph-eager {ge[n]:.3e}  eager-eager {ee[n]:.3e}  graph-graph {pairs['graph-graph'][n]:.3e}")
