"""Fused mixed-precision Adam (include/psfm_optim.h, trainers/fused_adam.py) against
torch.optim.Adam on the same fp32 master weights and the same gradients; the graph-captured
trainer step on the kernel."""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _net():
    torch.manual_seed(0)
    net = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(),
                        nn.Conv2d(8, 5, 1), nn.Flatten(), nn.Linear(5 * 6 * 7, 3))
    return net


def _opt(params_depth, params_pose, cls=torch.optim.Adam):
    return cls([{"name": "Depth", "params": params_depth, "lr": 2e-3, "weight_decay": 0.0},
                {"name": "Pose", "params": params_pose, "lr": 5e-4, "weight_decay": 1e-2}],
               betas=(0.9, 0.999), eps=1e-8)


@pytest.mark.parametrize("channels_last", [False, True])
def test_fused_adam_matches_torch_adam(channels_last):
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.trainers.fused_adam import FusedMixedAdam, storage_flat
    dev = torch.device("cuda:0")
    net = _net().to(dev)
    if channels_last:
        net = net.to(memory_format=torch.channels_last)
    ref = copy.deepcopy(net)
    ps = list(net.parameters())
    ps_ref = list(ref.parameters())
    opt = _opt(ps[:4], ps[4:])
    ref_opt = _opt(ps_ref[:4], ps_ref[4:])
    fused = FusedMixedAdam(net, opt, dev)
    lowp = [p.dtype == torch.bfloat16 for p in ps]
    assert lowp == [True, True, False, False, True, True, True, True]
    g = torch.Generator(device=dev).manual_seed(1)
    for step in range(4):
        for p, q, lp in zip(ps, ps_ref, lowp):
            gr = torch.randn(q.shape, device=dev, generator=g).to(memory_format=torch.channels_last) \
                if q.dim() == 4 and channels_last else torch.randn(q.shape, device=dev, generator=g)
            gr = gr * (10.0 ** (step - 2))
            if lp:
                gr = gr.to(torch.bfloat16)
            p.grad = gr
            q.grad = gr.float()
        fused.step()
        ref_opt.step()
        torch.cuda.synchronize()
        for p, q in zip(ps, ps_ref):
            m = fused.master_view(p)
            torch.testing.assert_close(m, q.detach(), rtol=2e-6, atol=1e-7)
            assert torch.equal(storage_flat(p.detach()), storage_flat(m.to(p.dtype)))


def test_grad_pack_is_a_flat_concatenation():
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.trainers.fused_adam import FusedMixedAdam, storage_flat
    dev = torch.device("cuda:0")
    net = _net().to(dev).to(memory_format=torch.channels_last)
    ps = list(net.parameters())
    fused = FusedMixedAdam(net, _opt(ps[:4], ps[4:]), dev)
    for p in ps:
        p.grad = torch.randn_like(p)
    flat = fused.new_flat_grad()
    fused.pack(flat)
    torch.cuda.synchronize()
    for p, off in zip(fused.params, fused.offsets):
        assert torch.equal(flat[off:off + p.numel()], storage_flat(p.grad).float())
    pad = torch.ones_like(flat, dtype=torch.bool)
    for p, off in zip(fused.params, fused.offsets):
        pad[off:off + p.numel()] = False
    assert torch.count_nonzero(flat[pad]) == 0


def test_graph_trainer_step_on_fused_adam():
    """World-size-1 HIP-graph step (fwd+bwd+fused Adam in ONE graph) on the full model: the
    replay advances the device step count, keeps weights == round(master) and trains."""
    import __graft_entry__
    __graft_entry__.build()
    import bench
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    from packnet_sfm_amd.trainers.fused_adam import storage_flat
    dev = torch.device("cuda:0")

    class A:
        depth_net, pose_net, batch, height, width = "ResNetSAN01", "PoseNet", 2, 64, 192

    torch.manual_seed(0)
    model = bench.build_model(A, dev).to(memory_format=torch.channels_last)
    opt = make_optimizer(model, 1e-4, 1e-4, capturable=True, fused=True)
    tr = DDPTrainer(model, opt, dev, amp_dtype=torch.bfloat16, graph=True, bf16_weights=True)
    assert tr.fused is not None
    batch = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)
    losses = [float(tr.train_step(batch)["loss"]) for _ in range(12)]
    torch.cuda.synchronize()
    tr.check_finite()
    assert int(tr.fused.step_count) == 12  # warm-up steps inside capture() are rolled back
    assert losses[-1] < losses[0]
    for p in tr.fused.params:
        assert torch.equal(storage_flat(p.detach()), storage_flat(tr.fused.master_view(p).to(p.dtype)))
    # BatchNorm step counters were taken out of the replayed step: the trainer's state_dict has
    # them (one per optimizer step) and the fp32 master weights (reference checkpoint format)
    sd = tr.state_dict()
    ref_keys = set(k for k in model.state_dict()) | {k for k in sd if k.endswith("num_batches_tracked")}
    assert set(sd) == ref_keys
    bns = [n for n, m in model.named_modules() if isinstance(m, torch.nn.BatchNorm2d)]
    assert bns and all(int(sd[n + ".num_batches_tracked"]) == 12 for n in bns)
    pname = {id(p): n for n, p in model.named_parameters()}
    for p in tr.fused.params:
        assert sd[pname[id(p)]].dtype == torch.float32
        assert torch.equal(sd[pname[id(p)]], tr.fused.master_view(p))
    tr.bn_counters_to_model()
    tr.bn_counters_to_model()   # idempotent
    assert all(int(m.num_batches_tracked) == 12 for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d))
