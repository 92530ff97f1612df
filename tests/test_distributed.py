"""Multi-process data-parallel logic on CPU (gloo, world size 2): the trainer's gradient
averaging (flat-buffer all-reduce = the graph mode's algebra, the bucketed all-reduce launched from
gradient hooks during the backward (comm='overlap'), and torch-DDP eager mode) must give
every rank the same parameters, equal to a single process stepping on the averaged gradient."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import golden_util as gu


class TinyModel(torch.nn.Module):
    """SfmModel-shaped toy: depth_net / pose_net attributes, batch-dict forward with a 'loss'."""

    def __init__(self):
        super().__init__()
        self.depth_net = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.ReLU(),
                                             torch.nn.Conv2d(8, 1, 3, padding=1))
        self.pose_net = torch.nn.Linear(3, 6)
        self.unused = None

    def forward(self, batch, progress=0.0):
        d = torch.sigmoid(self.depth_net(batch["rgb"]))
        p = self.pose_net(batch["rgb"].mean((2, 3)))
        loss = (d - batch["target"]).abs().mean() + 0.1 * (p ** 2).mean()
        return {"loss": loss.unsqueeze(0)}


def _batch(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return {"rgb": gu.smooth_texture(g, 2, 3, 16, 24), "target": torch.rand(2, 1, 16, 24, generator=g)}


def _worker(rank, world, init_file, mode, out_dir):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    os.environ["WORLD_SIZE"] = str(world)
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    torch.manual_seed(0)
    model = TinyModel()
    opt = make_optimizer(model, 1e-2, 1e-2)
    kw = dict(comm="overlap", overlap_bucket_mb=300 / 2 ** 20) if mode == "overlap" else {}
    tr = DDPTrainer(model, opt, torch.device("cpu"), amp_dtype=None, graph=False, flat=(mode != "ddp"), **kw)
    for _ in range(3):
        tr.train_step(_batch(rank))
    if mode == "overlap":   # the first step cut the buckets; steps 2-3 reduced them during the backward
        assert tr.buckets is not None and len(tr.buckets.buckets) >= 3, tr.buckets
        assert sorted(tr.buckets.launch_order) == list(range(len(tr.buckets.buckets)))
    torch.save({k: v.detach().clone() for k, v in model.state_dict().items()}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["flat", "ddp", "overlap"])
def test_two_rank_gradient_average(mode):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        init = os.path.join(d, "init")
        mp.spawn(_worker, args=(world, init, mode, d), nprocs=world, join=True)
        s0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        s1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    # single-process reference: Adam on the average of the two ranks' gradients
    torch.manual_seed(0)
    ref = TinyModel()
    opt = torch.optim.Adam([{"params": ref.depth_net.parameters(), "lr": 1e-2},
                            {"params": ref.pose_net.parameters(), "lr": 1e-2}])
    for _ in range(3):
        opt.zero_grad()
        loss = sum(ref(_batch(r))["loss"].sum() for r in range(world)) / world
        loss.backward()
        opt.step()
    for k, v in ref.state_dict().items():
        assert torch.allclose(s0[k], v, atol=1e-6, rtol=1e-5), k


def test_comm_api_single_process_is_identity():
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.utils import horovod as hvd
    assert hvd.rank() == 0 and hvd.world_size() == 1
    t = torch.ones(3)
    assert torch.equal(hvd.allreduce(t), t)
    assert hvd.reduce_value(2.5) == 2.5


# -------------------------------------------------------------------------------------------------
# data partition (DistributedSampler, model_wrapper.py:1138-1144) and the eval reduction
# (utils/reduce.py all_reduce_metrics, reduce.py:31-80) with two real ranks
class _EvalNet(torch.nn.Module):
    """SfmModel-shaped eval stand-in: depth_net-like output of a sigmoid map per image."""

    def forward(self, batch):
        s = batch["rgb"].mean(1, keepdim=True) * 0.15 + 0.02
        return {"inv_depths": [s]}


def _eval_dataset():
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.datasets.synthetic import SyntheticSfmDataset

    class WithDepth(SyntheticSfmDataset):
        def __getitem__(self, i):
            s = super().__getitem__(i)
            g = torch.Generator().manual_seed(500 + i)
            d = 1.0 + 70.0 * torch.rand(1, self.H, self.W, generator=g)
            d[torch.rand(1, self.H, self.W, generator=g) < 0.5] = 0.0
            s["depth"] = d
            return s
    return WithDepth(9, 24, 80, seed=3)   # odd length: the sampler pads rank 1 with a repeat


def _oracle_metrics(cfg, gt, pred, use_gt_scale=True):
    from oracle import photometric_oracle as O
    return O.depth_metrics(gt, pred, cfg.min_depth, cfg.max_depth, crop=cfg.crop, use_gt_scale=use_gt_scale)


def _dist_worker(rank, world, init_file, out_dir):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.datasets.synthetic import ResidentLoader, get_datasampler, setup_dataloader
    from packnet_sfm_amd.models.evaluate import validate
    ds = _eval_dataset()
    # training partition: resident loader over this rank's sampler indices
    loader = ResidentLoader(ds, 2, get_datasampler(ds, "train"), torch.device("cpu"))
    seen, parts = [], []
    for _ in range(3 * len(loader)):   # three epochs (reshuffled by set_epoch)
        if loader.step_in_epoch == 0 or loader.step_in_epoch >= loader.steps_per_epoch:
            b = loader.next_into(None)
            parts.append(list(loader.partition))
        else:
            b = loader.next_into(None)
        seen.append((len(parts) - 1, b["rgb"].reshape(b["rgb"].shape[0], -1)[:, :4].clone()))
    # validation: per-rank partition -> all_reduce_metrics
    vloaders = setup_dataloader([ds], batch_size=1, mode="validation")  # default_config validation batch 1
    res = validate(_EvalNet(), vloaders, [ds], 0.0, 80.0, crop="", metrics_fn=_oracle_metrics)
    torch.save({"parts": parts, "seen": seen, "metrics": dict(res[0])},
               os.path.join(out_dir, f"d{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sampler_partition_and_eval_reduction():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_dist_worker, args=(world, os.path.join(d, "init"), d), nprocs=world, join=True)
        r = [torch.load(os.path.join(d, f"d{k}.pt"), weights_only=True) for k in range(world)]
    ds = _eval_dataset()
    # every epoch the two partitions cover the dataset (the shorter rank padded with one repeat)
    # and reshuffle between epochs
    assert len(r[0]["parts"]) == 3
    for e in range(3):
        p0, p1 = r[0]["parts"][e], r[1]["parts"][e]
        assert sorted(set(p0) | set(p1)) == list(range(len(ds))) and len(p0) == len(p1) == 5
        assert len(set(p0) & set(p1)) <= 1
    assert r[0]["parts"][0] != r[0]["parts"][1]
    # every gathered batch row is one of that epoch's samples of that rank
    for k in range(world):
        for e, rows in r[k]["seen"]:
            keys = {tuple(ds[i]["rgb"].reshape(-1)[:4].tolist()) for i in r[k]["parts"][e]}
            assert all(tuple(row.tolist()) in keys for row in rows)
    # both ranks report the same reduced metrics, equal to a single-process evaluation of every
    # sample once (the padded repeat is averaged out by the seen count)
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.models.evaluate import evaluate_depth
    net = _EvalNet()
    per = []
    for i in range(len(ds)):
        s = ds[i]
        b = {"rgb": s["rgb"][None], "depth": s["depth"][None]}
        per.append(evaluate_depth(net, b, 0.0, 80.0, crop="", metrics_fn=_oracle_metrics)["metrics"])
    for key in r[0]["metrics"]:
        ref = torch.stack([p[key] for p in per]).double().mean(0).float()
        torch.testing.assert_close(r[0]["metrics"][key], r[1]["metrics"][key])
        torch.testing.assert_close(r[0]["metrics"][key], ref, rtol=1e-5, atol=1e-6)


def test_all_reduce_metrics_asserts_every_sample_seen():
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.utils.reduce import all_reduce_metrics
    outs = [{"idx": torch.tensor([0, 1]), "depth": torch.ones(7)}]
    with pytest.raises(AssertionError):
        all_reduce_metrics(outs, [list(range(3))])
    res = all_reduce_metrics(outs + [{"idx": torch.tensor([2]), "depth": 3 * torch.ones(7)}], [list(range(3))])
    torch.testing.assert_close(res[0]["depth"], torch.full((7,), 5.0 / 3))


def test_multicamera_batches_fold_cameras_into_the_batch():
    """DDAD samples carry [cameras, 3, H, W] per key (train_packnet_san_ddad.yaml: 4 cameras); the
    resident loader and the models fold cameras into the batch like model_utils.stack_batch, with
    each camera keeping its own intrinsics."""
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.datasets.synthetic import ResidentLoader, SyntheticSfmDataset, flatten_cameras
    from packnet_sfm_amd.models.model_utils import stack_batch
    ds = SyntheticSfmDataset(4, 16, 32, cameras=4, seed=1)
    s = ds[2]
    assert s["rgb"].shape == (4, 3, 16, 32) and s["intrinsics"].shape == (4, 3, 3)
    one = {"rgb": s["rgb"][None], "rgb_context": [c[None] for c in s["rgb_context"]],
           "intrinsics": s["intrinsics"][None]}
    flat, ref = flatten_cameras(dict(one)), stack_batch(dict(one))
    assert torch.equal(flat["rgb"], ref["rgb"]) and torch.equal(flat["intrinsics"], ref["intrinsics"])
    assert all(torch.equal(a, b) for a, b in zip(flat["rgb_context"], ref["rgb_context"]))
    loader = ResidentLoader(ds, 2, torch.utils.data.SequentialSampler(ds), torch.device("cpu"))
    b = loader.next_into(None)
    assert b["rgb"].shape == (8, 3, 16, 32) and b["intrinsics"].shape == (8, 3, 3)
    assert torch.equal(b["rgb"][4:8], ds[1]["rgb"]) and torch.equal(b["intrinsics"][4:8], ds[1]["intrinsics"])


@pytest.mark.parametrize("bad", [float("nan"), float("inf")])
def test_check_finite_flags_a_nonfinite_loss_seen_steps_earlier(bad):
    """The trainer's sticky non-finite flag (0 * loss accumulated per step) reports a NaN / inf
    loss at the next check even when the steps after it were finite."""
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer

    class Poisoned(TinyModel):
        def __init__(self):
            super().__init__()
            self.calls = 0

        def forward(self, batch, progress=0.0):
            out = super().forward(batch, progress)
            self.calls += 1
            if self.calls == 2:
                out["loss"] = out["loss"] * bad
            return out

    torch.manual_seed(0)
    model = Poisoned()
    tr = DDPTrainer(model, make_optimizer(model, 1e-3, 1e-3), torch.device("cpu"), amp_dtype=None, graph=False,
                    flat=True)
    tr.train_step(_batch(0))
    tr.check_finite()   # finite so far
    for _ in range(3):
        tr.train_step(_batch(0))
    with pytest.raises(ValueError, match="Non-finite"):
        tr.check_finite()


# -------------------------------------------------------------------------------------------------
# a parameter that stops receiving gradients after the bucket-learning step, and the
# bucket launch order agreed across ranks
class DroppingHead(TinyModel):
    """`extra` contributes to the loss in the first step only (as an inverse-depth head of a scale
    that ProgressiveScaling drops later): from step 2 on its gradient is None."""

    def __init__(self):
        super().__init__()
        self.extra = torch.nn.Linear(3, 1)
        self.calls = 0

    def forward(self, batch, progress=0.0):
        out = super().forward(batch, progress)
        self.calls += 1
        if self.calls == 1:
            out["loss"] = out["loss"] + 0.1 * self.extra(batch["rgb"].mean((2, 3))).pow(2).mean()
        return out


def _drop_worker(rank, world, init_file, out_dir):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer
    torch.manual_seed(0)
    model = DroppingHead()
    opt = torch.optim.Adam([{"params": list(model.depth_net.parameters()) + list(model.extra.parameters()),
                             "lr": 1e-2}, {"params": model.pose_net.parameters(), "lr": 1e-2}])
    tr = DDPTrainer(model, opt, torch.device("cpu"), amp_dtype=None, graph=False, flat=True, comm="overlap",
                    overlap_bucket_mb=300 / 2 ** 20)
    for _ in range(3):
        tr.train_step(_batch(rank))
    assert model.extra.weight.grad is None
    torch.save({k: v.detach().clone() for k, v in model.state_dict().items()}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_overlap_buckets_with_a_parameter_that_loses_its_gradient():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_drop_worker, args=(world, os.path.join(d, "init"), d), nprocs=world, join=True)
        s0 = torch.load(os.path.join(d, "r0.pt"), weights_only=True)
        s1 = torch.load(os.path.join(d, "r1.pt"), weights_only=True)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    torch.manual_seed(0)
    ref = DroppingHead()
    opt = torch.optim.Adam([{"params": list(ref.depth_net.parameters()) + list(ref.extra.parameters()), "lr": 1e-2},
                            {"params": ref.pose_net.parameters(), "lr": 1e-2}])
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        calls = ref.calls
        loss = 0
        for r in range(world):
            ref.calls = calls   # both ranks see the same step index
            loss = loss + ref(_batch(r))["loss"].sum()
        (loss / world).backward()
        opt.step()
    for k, v in ref.state_dict().items():
        assert torch.allclose(s0[k], v, atol=1e-6, rtol=1e-5), k


def _order_worker(rank, world, init_file, out_dir):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.trainers.grad_buckets import GradBuckets
    ps = [torch.nn.Parameter(torch.zeros(10)) for _ in range(4)]
    flat = torch.zeros(40)
    # each rank "observed" a different gradient order in its learning step
    order = ps[::-1] if rank == 0 else [ps[1], ps[0], ps[3], ps[2]]
    gb = GradBuckets(ps, [0, 10, 20, 30], flat, 40, torch.device("cpu"), order=order)
    torch.save(torch.tensor(gb.launch_order), os.path.join(out_dir, f"o{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_launch_order_is_rank0s_on_every_rank():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_order_worker, args=(world, os.path.join(d, "init"), d), nprocs=world, join=True)
        o = [torch.load(os.path.join(d, f"o{r}.pt"), weights_only=True).tolist() for r in range(world)]
    assert o[0] == o[1] == [3, 2, 1, 0]


def test_checkpoint_round_trips_through_load_network(tmp_path):
    """DDPTrainer.checkpoint() is the reference's checkpoint dict (model_checkpoint.py:66-76, keys
    under 'model.'); the reference's prefix-stripping loader (utils/load.py:114-163) restores the
    depth and pose nets from the saved file."""
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    from packnet_sfm_amd.utils.load import load_network
    torch.manual_seed(0)
    model = TinyModel()
    tr = DDPTrainer(model, make_optimizer(model, 1e-2, 1e-2), torch.device("cpu"), amp_dtype=None, graph=False,
                    flat=True)
    tr.train_step(_batch(0))
    ck = tr.checkpoint(config={"name": "tiny"}, epoch=3)
    assert set(ck) == {"config", "epoch", "state_dict", "optimizer", "scheduler"}
    assert all(k.startswith("model.") for k in ck["state_dict"])
    path = tmp_path / "epoch=3.ckpt"
    torch.save(ck, path)
    torch.manual_seed(1)
    fresh = TinyModel()
    _, n, total = load_network(fresh.depth_net, str(path), "depth_net")
    assert n == total == len(fresh.depth_net.state_dict())
    load_network(fresh.pose_net, str(path), ["pose_net"])
    for k, v in model.state_dict().items():
        assert torch.equal(fresh.state_dict()[k], v), k


def _half_none_worker(rank, world, init_file, out_dir):
    """Rank 1 has NO gradient for parameter 1 this step, rank 0 has one: after the bucketed
    all-reduce both ranks must hold the same averaged gradient for it (rank 1 used to keep
    None and skip the update the other rank applied); parameter 3 has no gradient anywhere and stays
    None on both ranks."""
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.trainers.grad_buckets import GradBuckets
    ps = [torch.nn.Parameter(torch.zeros(10)) for _ in range(4)]
    flat = torch.zeros(40)
    gb = GradBuckets(ps, [0, 10, 20, 30], flat, 80, torch.device("cpu"))
    gb.arm()
    for i, p in enumerate(ps):
        if i == 3 or (i == 1 and rank == 1):
            continue
        p.grad = torch.full((10,), float(rank + 1 + 10 * i))
        gb.on_grad(p)
    gb.finish()
    gb.unpack(1.0 / world)
    torch.save([None if p.grad is None else p.grad.clone() for p in ps], os.path.join(out_dir, f"g{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_unpack_agrees_on_missing_gradients():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_half_none_worker, args=(world, os.path.join(d, "init"), d), nprocs=world, join=True)
        g = [torch.load(os.path.join(d, f"g{r}.pt"), weights_only=True) for r in range(world)]
    for i in range(3):
        assert torch.equal(g[0][i], g[1][i]), i
    assert torch.equal(g[0][1], torch.full((10,), (11.0 + 0.0) / 2))   # rank 0's 11, rank 1's zeros
    assert g[0][3] is None and g[1][3] is None


def _cut_worker(rank, world, init_file, out_dir):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.trainers.grad_buckets import GradBuckets
    ps = [torch.nn.Parameter(torch.zeros(10)) for _ in range(4)]
    try:   # the ranks cut different buckets (different caps): both must refuse
        GradBuckets(ps, [0, 10, 20, 30], torch.zeros(40), 80 if rank == 0 else 160, torch.device("cpu"))
        msg = "no error"
    except RuntimeError as e:
        msg = str(e)
    with open(os.path.join(out_dir, f"c{rank}.txt"), "w") as f:
        f.write(msg)
    dist.destroy_process_group()


def test_mismatched_bucket_cuts_are_refused():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_cut_worker, args=(world, os.path.join(d, "init"), d), nprocs=world, join=True)
        msgs = [open(os.path.join(d, f"c{r}.txt")).read() for r in range(world)]
    assert all("ranks cut different buckets" in m for m in msgs), msgs


def _capture_presence_worker(rank, world, init_file, out_dir):
    """A captured unpack must not run the presence collective: it uses the presence the
    last eager unpack agreed, and refuses to run before any eager agreement."""
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.trainers import grad_buckets as GBM
    ps = [torch.nn.Parameter(torch.zeros(10)) for _ in range(3)]
    gb = GBM.GradBuckets(ps, [0, 10, 20], torch.zeros(30), 80, torch.device("cpu"))

    def step():
        gb.arm()
        for i, p in enumerate(ps):
            if i == 2 and rank == 1:
                continue
            p.grad = torch.full((10,), float(rank + 1))
            gb.on_grad(p)
        gb.finish()

    calls = []
    real = GBM.dist.all_reduce

    def counting(t, *a, **k):
        calls.append(tuple(t.shape))
        return real(t, *a, **k)

    GBM.dist.all_reduce = counting
    captured = [False]
    GBM.torch.cuda.is_current_stream_capturing = lambda: captured[0]
    GBM.torch.cuda.is_available = lambda: True
    msgs = []
    try:
        step()
        captured[0] = True
        try:
            gb.unpack(0.5)
            msgs.append("no error")
        except RuntimeError as e:
            msgs.append(str(e))
        captured[0] = False
        for p in ps:
            p.grad = None
        step()
        gb.unpack(0.5)          # eager: agrees (one flag all-reduce)
        n_eager = len([c for c in calls if c == (3,)])
        for p in ps:
            p.grad = None
        step()
        captured[0] = True
        gb.unpack(0.5)          # "captured": no flag all-reduce
        n_capt = len([c for c in calls if c == (3,)]) - n_eager
    finally:
        GBM.dist.all_reduce = real
    torch.save({"msgs": msgs, "n_eager": n_eager, "n_capt": n_capt,
                "g2": ps[2].grad.clone()}, os.path.join(out_dir, f"p{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_captured_bucket_unpack_uses_the_eagerly_agreed_presence():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_capture_presence_worker, args=(world, os.path.join(d, "init"), d), nprocs=world, join=True)
        res = [torch.load(os.path.join(d, f"p{r}.pt"), weights_only=True) for r in range(world)]
    for r in res:
        assert "must be agreed in an eager step" in r["msgs"][0]
        assert r["n_eager"] == 1 and r["n_capt"] == 0
    assert torch.equal(res[0]["g2"], res[1]["g2"])   # rank 1 had no gradient: it gets the average too


# ---------------------------------------------------------------------------------------------
# bench.py --comm auto: the overlap path is chosen only when every rank's
# short-lived probe child (trainers/comm_probe.py) passed; every rank picks the same path.
def test_choose_comm_every_rank_reads_every_probe_status():
    import threading

    import bench
    for rcs, want in (((0, 0), "overlap"), ((0, 1), "split"), ((124, 0), "split")):
        store, out = dist.HashStore(), {}

        def rank_fn(r):
            out[r] = bench.choose_comm(store, r, 2, lambda port: rcs[r])

        th = [threading.Thread(target=rank_fn, args=(r,)) for r in (1, 0)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert out[0] == out[1] and out[0][0] == want, (rcs, out)
        if want == "split":
            assert "failed" in out[0][1]


def _torchrun_probe(extra_env, *extra):
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(root, "bench.py"), "--gpus", "2",
           "--dist-backend", "gloo", "--probe-backend", "gloo", "--probe-only", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="1", **extra_env)
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1]), out.stderr


def test_comm_auto_probe_children_over_gloo_world2():
    """The whole selection on CPU: two torch.distributed.run ranks, each starting its probe child
    (own process group, the bucketed overlap path eagerly over gloo); both pass.  The run itself is
    gloo, so it must still train with split — and says why."""
    res, err = _torchrun_probe({})
    assert res["world"] == 2 and res["comm"] == "split", res
    assert "probe passed on 2 ranks" in res["comm_note"] and "gloo run" in res["comm_note"], res
    assert err.count("[comm probe] rank") == 2, err[-2000:]


def test_comm_auto_probe_failure_and_hang_select_split():
    """Rank 1's child fails at once; rank 0's child then waits for its peer and is killed at the
    timeout: both ranks see the failures and pick split."""
    res, err = _torchrun_probe({"PSFM_TEST_PROBE_FAIL_RANK": "1"}, "--comm-probe-timeout", "20")
    assert res["comm"] == "split" and "failed" in res["comm_note"], res
    assert "3" in res["comm_note"] and "124" in res["comm_note"], res


class _NetsOnly(torch.nn.Module):
    """The bench model's depth / pose nets with a loss that reaches every output (so the same
    parameters get gradients as under the photometric loss), for the bucket-cut comparison."""

    def __init__(self, model):
        super().__init__()
        self.depth_net, self.pose_net = model.depth_net, model.pose_net

    def forward(self, batch, progress=0.0):
        inv = self.depth_net(batch["rgb"])["inv_depths"]
        vec = self.pose_net(batch["rgb"], batch["rgb_context"])
        return {"loss": (sum(i.float().mean() for i in inv) + vec.float().mean()).reshape(1)}


def _cuts_worker(rank, world, init_file, config, out_dir):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    os.environ["WORLD_SIZE"] = str(world)
    import json

    import bench
    from packnet_sfm_amd.trainers import comm_probe
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    torch.set_num_threads(4)
    args = bench.parse(["--config", config, "--bucket-mb", "16"])
    probe = comm_probe.run_probe(torch.device("cpu"), steps=2, bucket_mb=args.bucket_mb, shapes=bench.param_shapes(args))
    torch.manual_seed(0)
    model = _NetsOnly(bench.build_model(args, torch.device("cpu")))
    tr = DDPTrainer(model, make_optimizer(model), torch.device("cpu"), amp_dtype=None, graph=False, flat=True,
                    comm="overlap", overlap_bucket_mb=args.bucket_mb, force_comm=True)
    g = torch.Generator().manual_seed(rank)
    batch = {"rgb": torch.rand(1, 3, 64, 192, generator=g), "rgb_context": [torch.rand(1, 3, 64, 192, generator=g)
                                                                            for _ in range(2)]}
    for _ in range(2):
        tr.train_step(batch)
    real = comm_probe.bucket_cuts(tr)
    if rank == 0:
        with open(os.path.join(out_dir, "cuts.json"), "w") as f:
            json.dump({"probe": [list(r) for r in probe["cuts"]], "probe_mb": probe["bucket_mb"],
                       "real": [list(r) for r in real[0]], "real_mb": real[1]}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("config", ["kitti-resnet-san", "kitti-packnet"])
def test_comm_probe_cuts_the_same_buckets_as_the_training_step(config):
    """the --comm auto probe's stand-in (trainers/comm_probe.ShapeNet: the bench
    model's parameter shapes, built on the meta device) cuts exactly the gradient buckets the real
    model's trainer cuts at the bench's 16 MB bucket size — the same number of RCCL calls with the same
    message sizes — on 2 gloo ranks."""
    import json
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_cuts_worker, args=(world, os.path.join(d, "init"), config, d), nprocs=world, join=True)
        with open(os.path.join(d, "cuts.json")) as f:
            res = json.load(f)
    assert len(res["real"]) >= 2 and res["probe"] == res["real"], res
    assert res["probe_mb"] == res["real_mb"]
