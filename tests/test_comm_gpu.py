"""The gradient all-reduce of the data-parallel step over RCCL on one device (a world-size-1
'nccl' process group; `force_comm=True` makes the trainer run its world > 1 communication path):
the bucketed all-reduce launched from gradient hooks during the backward and captured into the
step's HIP graph (comm='overlap', trainers/grad_buckets.py) must reduce every gradient of every
replayed step, and give the same step as one flat all-reduce after the backward (comm='graph')."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_world1():
    import __graft_entry__
    __graft_entry__.build()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    yield dev
    dist.destroy_process_group()


def _trainer(dev, comm, fp32, seed=0):
    import bench
    from test_trainer_gpu import _build
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    m = _build(dev, seed)
    if fp32:
        opt = make_optimizer(m, 1e-4, 1e-4, capturable=True)
        t = DDPTrainer(m, opt, dev, amp_dtype=None, graph=True, comm=comm, force_comm=True,
                       overlap_bucket_mb=2.0)
    else:
        t = DDPTrainer(m, make_optimizer(m, 1e-4, 1e-4), dev, amp_dtype=torch.bfloat16, graph=True,
                       bf16_weights=True, comm=comm, force_comm=True, overlap_bucket_mb=2.0)
    return m, t, bench


def test_overlap_buckets_reduce_every_gradient_of_every_replay(rccl_world1):
    """Production configuration (bf16 nets, fused Adam): after each replay the all-reduced flat
    buffer equals a fresh pack of that replay's gradients, bit for bit (a bucket whose pack or
    collective were not captured would hold the previous step's values), and every step updates
    the weights once."""
    dev = rccl_world1
    m, t, bench = _trainer(dev, "overlap", fp32=False)
    batches = [bench.synthetic_batch(2, 64, 192, dev, seed=s, channels_last=True) for s in range(3)]
    static = {k: (v.clone() if torch.is_tensor(v) else [c.clone() for c in v]) for k, v in batches[0].items()}
    for i, b in enumerate(batches):
        t.train_step(static if i == 0 else b)
        torch.cuda.synchronize()
        nb = len(t.buckets.buckets)
        assert nb >= 4, nb
        fresh = t.fused.new_flat_grad()
        t.fused.pack(fresh)
        torch.cuda.synchronize()
        assert torch.equal(fresh, t.flat_grad), (i, float((fresh - t.flat_grad).abs().max()))
    assert int(t.fused.step_count) == 3
    print(f"buckets: {nb}, launch order {t.buckets.launch_order}")


def test_overlap_step_equals_single_allreduce_step(rccl_world1):
    """fp32 nets with deterministic MIOpen algorithms: comm='overlap' (bucketed, captured on a
    side stream) and comm='graph' (one flat all-reduce after the backward) give the same loss,
    gradients and parameters bit for bit over 3 replayed steps."""
    dev = rccl_world1
    old = torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    try:
        mo, to, bench = _trainer(dev, "overlap", fp32=True)
        mg, tg, _ = _trainer(dev, "graph", fp32=True)
        batches = [bench.synthetic_batch(2, 64, 192, dev, seed=s, channels_last=True) for s in range(3)]
        so = {k: (v.clone() if torch.is_tensor(v) else [c.clone() for c in v]) for k, v in batches[0].items()}
        sg = {k: (v.clone() if torch.is_tensor(v) else [c.clone() for c in v]) for k, v in batches[0].items()}
        for i, b in enumerate(batches):
            oo = to.train_step(so if i == 0 else b)
            og = tg.train_step(sg if i == 0 else b)
            torch.cuda.synchronize()
            assert torch.equal(oo["loss"], og["loss"]), i
            for (n, po), pg in zip(mo.named_parameters(), mg.parameters()):
                assert (po.grad is None) == (pg.grad is None), n
                if po.grad is not None:
                    assert torch.equal(po.grad, pg.grad), (i, n)
        for (n, po), pg in zip(mo.named_parameters(), mg.parameters()):
            assert torch.equal(po, pg), n
        assert len(to.buckets.buckets) >= 4
    finally:
        torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = old
