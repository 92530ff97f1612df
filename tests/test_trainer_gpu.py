"""The training step as the bench runs it: the HIP-graph-replayed DDPTrainer step against the
same step run eagerly, and the world-size > 1 gradient algebra (flat all-reduce payload ->
fused Adam with 1/world) against torch.optim.Adam on the averaged gradient."""
import copy
import warnings

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _build(dev, seed=0):
    import bench

    class A:
        depth_net, pose_net, batch, height, width = "ResNetSAN01", "PoseNet", 2, 64, 192

    torch.manual_seed(seed)
    return bench.to_channels_last(bench.build_model(A, dev))


def test_graph_replayed_step_equals_eager_step():
    """One replay == one eager step on the same batch: same loss, same gradients (bf16 nets;
    MIOpen's weight-gradient kernels may reduce in a different order between calls, so the
    gradients are compared by relative norm), same number of optimizer steps, and no
    AccumulateGrad stream-mismatch warning (the pose net runs on a forked stream)."""
    import __graft_entry__
    __graft_entry__.build()
    import bench
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = False
    mg, me = _build(dev), _build(dev)
    tg = DDPTrainer(mg, make_optimizer(mg, 1e-4, 1e-4, capturable=True, fused=True), dev,
                    amp_dtype=torch.bfloat16, graph=True, bf16_weights=True)
    te = DDPTrainer(me, make_optimizer(me, 1e-4, 1e-4), dev, amp_dtype=torch.bfloat16, graph=False, flat=True,
                    bf16_weights=True, fused_optim=True)
    batches = [bench.synthetic_batch(2, 64, 192, dev, seed=s, channels_last=True) for s in range(3)]
    static = {k: (v.clone() if torch.is_tensor(v) else [c.clone() for c in v]) for k, v in batches[0].items()}
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for i, b in enumerate(batches):
            og = tg.train_step(static if i == 0 else b)
            oe = te.train_step(b)
            torch.cuda.synchronize()
            lg, le = float(og["loss"]), float(oe["loss"])
            assert abs(lg - le) <= 1e-3 * abs(le), (i, lg, le)
            for (n, pg), pe in zip(mg.named_parameters(), me.parameters()):
                if pe.grad is None:
                    assert pg.grad is None, n
                    continue
                d = (pg.grad.float() - pe.grad.float()).norm() / pe.grad.float().norm().clamp_min(1e-20)
                assert float(d) < 2e-2, (i, n, float(d))
    msgs = [str(w.message) for w in caught if "AccumulateGrad" in str(w.message)]
    assert not msgs, msgs[0]
    assert int(tg.fused.step_count) == int(te.fused.step_count) == 3
    # per-step outputs are this step's own values, not views of the graph's static output
    assert og["loss"].data_ptr() != tg.static_output["loss"].data_ptr()
    dm = (tg.fused.master - te.fused.master).abs().mean()
    assert float(dm) < 0.05 * 1e-4, float(dm)


def test_world2_flat_allreduce_algebra_on_fused_adam():
    """What a world-size-2 step does on each rank, on one device: every rank packs its gradients
    into the flat fp32 payload, RCCL sums the payloads, fused Adam reads the sum scaled by
    1/world.  Must equal torch.optim.Adam on the averaged fp32 gradient."""
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.trainers.fused_adam import FusedMixedAdam
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(), nn.Conv2d(8, 5, 1),
                        nn.Flatten(), nn.Linear(5 * 6 * 7, 3)).to(dev).to(memory_format=torch.channels_last)
    ref = copy.deepcopy(net)
    ps, qs = list(net.parameters()), list(ref.parameters())
    groups = lambda a: [{"name": "Depth", "params": a[:4], "lr": 2e-3}, {"name": "Pose", "params": a[4:], "lr": 5e-4}]  # noqa: E731,E501
    fused = FusedMixedAdam(net, torch.optim.Adam(groups(ps)), dev)
    ref_opt = torch.optim.Adam(groups(qs))
    world = 2
    g = torch.Generator(device=dev).manual_seed(3)
    for step in range(3):
        per_rank = [[torch.empty_strided(p.shape, p.stride(), device=dev, dtype=p.dtype)
                     .copy_(torch.randn(q.shape, device=dev, generator=g)) for p, q in zip(ps, qs)]
                    for _ in range(world)]
        total = fused.new_flat_grad()
        for grads in per_rank:
            for p, gr in zip(ps, grads):
                p.grad = gr
            flat = fused.new_flat_grad()
            fused.pack(flat)
            total += flat                      # the all_reduce(SUM)
        fused.step(total, 1.0 / world)
        for q, *gs in zip(qs, *per_rank):
            q.grad = sum(x.float() for x in gs) / world
        ref_opt.step()
        torch.cuda.synchronize()
        for p, q in zip(ps, qs):
            torch.testing.assert_close(fused.master_view(p), q.detach(), rtol=2e-6, atol=1e-7)
