"""How far apart are the bf16 weight gradients of the training step between (a) an eager step,
(b) the same eager step again, (c) the HIP-graph-replayed step, and (d) an fp32 step on the same
(bf16-rounded) weights?  Relative norm differences per parameter, worst first."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
__graft_entry__.build()
import bench  # noqa: E402
from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False


class A:
    depth_net, pose_net, batch, height, width = "ResNetSAN01", "PoseNet", 2, 64, 192


def build():
    torch.manual_seed(0)
    return bench.to_channels_last(bench.build_model(A, dev))


batch = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)


def grads(model):
    return {n: (p.grad.float().clone() if p.grad is not None else None) for n, p in model.named_parameters()}


def eager_grads(model, amp):
    for p in model.parameters():
        p.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp, cache_enabled=False):
        out = model(batch)
    out["loss"].sum().backward()
    torch.cuda.synchronize()
    return grads(model), float(out["loss"])


mg = build()
tg = DDPTrainer(mg, make_optimizer(mg, 0.0, 0.0, capturable=True, fused=True), dev, amp_dtype=torch.bfloat16,
                graph=True, bf16_weights=True)
out = tg.train_step(batch)
torch.cuda.synchronize()
g_graph, l_graph = grads(mg), float(out["loss"])
me = build()
te = DDPTrainer(me, make_optimizer(me, 0.0, 0.0), dev, amp_dtype=torch.bfloat16, graph=False, flat=True,
                bf16_weights=True, fused_optim=True)
g_e1, l_e1 = eager_grads(me, True)
g_e2, l_e2 = eager_grads(me, True)
# fp32 model with the bf16-rounded weights
mf = build()
with torch.no_grad():
    for p, q in zip(mf.parameters(), me.parameters()):
        p.copy_(q.float())
g_f, l_f = eager_grads(mf, False)
print(f"loss graph {l_graph:.6f} eager {l_e1:.6f} {l_e2:.6f} fp32 {l_f:.6f}")


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


rows = []
for n in g_f:
    if g_f[n] is None or g_e1[n] is None:
        continue
    rows.append((rel(g_graph[n], g_e1[n]), rel(g_e2[n], g_e1[n]), rel(g_e1[n], g_f[n]), rel(g_graph[n], g_f[n]), n))
rows.sort(reverse=True)
print("graph-vs-eager  eager-vs-eager  eager-vs-fp32  graph-vs-fp32  param")
for r in rows[:25]:
    print(f"{r[0]:14.3e}  {r[1]:14.3e}  {r[2]:13.3e}  {r[3]:13.3e}  {r[4]}")
print("median graph-vs-eager", sorted(r[0] for r in rows)[len(rows) // 2],
      "median eager-vs-fp32", sorted(r[2] for r in rows)[len(rows) // 2])
