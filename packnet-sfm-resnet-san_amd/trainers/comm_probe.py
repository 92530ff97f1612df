"""Pre-flight check of the overlapped gradient all-reduce (comm='overlap') on THIS node's ranks.

The bucketed all-reduce launched from gradient hooks and captured into the step's HIP graph
(trainers/grad_buckets.py; the reference's Horovod fusion buffer, utils/horovod.py:46-70, driven by
trainers/horovod_trainer.py:222-284) hides all but the last bucket behind the backward.  A
collective that fails DURING a graph capture leaves the stream capturing and the process unusable
(Multi-GPU), so the choice cannot be made by trying it in the training process.  Instead
every rank of `bench.py --gpus N --comm auto` starts ONE short-lived child process before it touches
the GPU; the N children form their own process group and run `run_probe`: a stand-in with the bench
model's parameter shapes (ShapeNet: the same buckets and RCCL message sizes as the real step) through
the exact trainer path (DDPTrainer comm='overlap', fused mixed-precision Adam, hooks -> bucket packs
-> RCCL all-reduces on a side stream, all captured into one HIP graph, replayed) on different data
per rank, then check that

  * every rank holds bit-identical fp32 master weights after the replayed steps,
  * the captured bucket all-reduce equals an eager all-reduce of a fresh pack of the same
    gradients (within fp32 summation-order rounding), and the loss is finite.

A child that fails, crashes or hangs (killed at the timeout) takes only itself down; the training
ranks then run comm='split' (the all-reduce between two graph replays), and bench.py records which
path ran and why in its JSON line (config.comm).  On the CPU the same probe runs eagerly over gloo
(the bucket path without graphs): tests/test_distributed.py covers the selection there.
"""
import math

import torch
import torch.distributed as dist
import torch.nn as nn


class ShapeNet(nn.Module):
    """The bench model's parameters — the same shapes, in the same order, in the same 'Depth' /
    'Pose' optimizer groups (make_optimizer) — without its layers: the trainer then cuts the same
    gradient buckets and the probe's captured RCCL calls carry the real step's bucket count and
    message sizes, with no MIOpen kernel to find on a cold box.  Loss: sum_p c * <p, p> (every
    parameter gets the gradient 2 c p; c differs per rank)."""

    def __init__(self, depth_shapes, pose_shapes):
        super().__init__()
        mk = lambda shapes: nn.ParameterList([nn.Parameter(0.01 * torch.randn(s)) for s in shapes])  # noqa: E731
        self.depth_net, self.pose_net = mk(depth_shapes), mk(pose_shapes)

    def forward(self, batch, progress=0.0):
        c = batch["c"]
        loss = sum((p.float() * p.float()).sum() for p in self.parameters()) * c
        return {"loss": loss.reshape(1)}


def bucket_cuts(trainer):
    """The trainer's gradient buckets as flat element ranges [(start, end)] and their sizes in MB."""
    ranges = [tuple(int(v) for v in r) for r in trainer.buckets.ranges]
    return ranges, [round((e - s) * 4 / 2 ** 20, 3) for s, e in ranges]


class ProbeNet(nn.Module):
    """Three linear layers (83 k parameters): several buckets at a small bucket size, and no MIOpen
    kernels to build on a cold box."""

    def __init__(self, d=64, h=256):
        super().__init__()
        self.l1, self.l2, self.l3 = nn.Linear(d, h), nn.Linear(h, h), nn.Linear(h, d)

    def forward(self, batch, progress=0.0):
        x = batch["x"]
        y = self.l3(torch.relu(self.l2(torch.relu(self.l1(x)))))
        return {"loss": (y.float() - x.float()).pow(2).mean()}


def run_probe(device, steps=3, bucket_mb=0.05, seed=0, shapes=None):
    """Run the overlapped step `steps` times on this rank (process group already initialised) and
    check it against the eager collective.  `shapes` = (depth shapes, pose shapes) of the bench
    model (ShapeNet: the real bucket layout at `bucket_mb`), or None (ProbeNet, small buckets).
    Returns a dict of what was checked (with the bucket cuts); raises RuntimeError on a mismatch."""
    from .ddp_trainer import DDPTrainer, make_optimizer
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(seed)
    gpu = device.type == "cuda"
    if shapes is not None:
        model = ShapeNet(*shapes).to(device)
        opt = make_optimizer(model, 1e-4, 1e-4, capturable=gpu, fused=gpu) if gpu else make_optimizer(model)
    else:
        model = ProbeNet().to(device)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, capturable=gpu)
    if gpu:
        t = DDPTrainer(model, opt, device, amp_dtype=torch.bfloat16, graph=True, bf16_weights=True,
                       comm="overlap", overlap_bucket_mb=bucket_mb, force_comm=world == 1)
    else:
        t = DDPTrainer(model, opt, device, amp_dtype=None, graph=False, flat=True, comm="overlap",
                       overlap_bucket_mb=bucket_mb, force_comm=world == 1)
    g = torch.Generator().manual_seed(1000 + rank)
    if shapes is not None:
        batches = [{"c": torch.full((1,), 0.5 + 0.25 * rank + 0.1 * i, device=device)} for i in range(steps)]
    else:
        batches = [{"x": torch.randn(32, 64, generator=g).to(device)} for _ in range(steps)]
    loss = None
    for b in batches:
        loss = float(t.train_step(b)["loss"].detach().sum())
    if gpu:
        torch.cuda.synchronize(device)
    if t.buckets is None or len(t.buckets.buckets) < 2:
        raise RuntimeError(f"probe: expected >= 2 gradient buckets, got "
                           f"{0 if t.buckets is None else len(t.buckets.buckets)}")
    if not math.isfinite(loss):
        raise RuntimeError(f"probe: non-finite loss {loss}")
    err = 0.0
    if t.fused is not None:
        # the last replay's reduced buffer (a SUM: Adam scales by 1 / world) vs an eager all-reduce of
        # a fresh pack of the gradients that replay left in the parameters' .grad
        fresh = t.fused.new_flat_grad()
        t.fused.pack(fresh)
        dist.all_reduce(fresh)
        err = float((t.flat_grad - fresh).abs().max()) / max(float(fresh.abs().max()), 1e-30)
        if not err <= 1e-5:
            raise RuntimeError(f"probe: captured bucket all-reduce differs from the eager one by {err:.3e}")
    else:
        # eager bucket path: the averaged gradient was unpacked into every rank's .grad
        gsum = torch.cat([p.grad.reshape(-1) for p in t._grads()[0]])
        g0 = gsum.clone()
        dist.broadcast(g0, src=0)
        err = float((gsum - g0).abs().max())
        if err != 0.0:
            raise RuntimeError(f"probe: ranks hold different averaged gradients ({err:.3e})")
    # every rank holds the same weights
    w = t.fused.master if t.fused is not None else torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    w0 = w.clone()
    dist.broadcast(w0, src=0)
    same = torch.tensor([float(torch.equal(w, w0))], device=device)
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    if float(same) != 1.0:
        raise RuntimeError("probe: ranks hold different weights after the overlapped steps")
    ranges, mb = bucket_cuts(t)
    return {"buckets": len(t.buckets.buckets), "bucket_mb": mb, "cuts": ranges, "loss": loss,
            "allreduce_rel_err": err, "world": world, "model": "bench shapes" if shapes is not None else "ProbeNet"}
