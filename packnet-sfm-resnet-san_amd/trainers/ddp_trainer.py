"""Data-parallel trainer: one process per GPU, RCCL all-reduce of gradients over xGMI (replaces
packnet_sfm/trainers/horovod_trainer.py, whose Horovod is a mock — SURVEY.md §0.2).

Per step (horovod_trainer.py:222-284): zero_grad -> forward (depth/pose nets under bf16
autocast, photometric loss in fp32 on the HIP kernels) -> backward -> gradient average across
ranks -> optimizer.step() — exactly one optimizer step per batch.

Execution modes:
  * graph (default on a ROCm device): the step is captured into HIP graphs once and replayed —
    the eager step is host-bound (~1.5k launches, MIOpen host overhead).
    Warm-up steps before the capture (MIOpen algorithm search, allocator) run on a snapshot of
    the training state that is restored afterwards, so they do not train.  Autograd writes each
    gradient into its own graph-static tensor; for world size > 1 they are packed into ONE flat
    fp32 buffer and averaged by RCCL:
      - comm='split': fwd+bwd+pack graph | all_reduce (host-enqueued, async) | Adam graph;
      - comm='graph': the all_reduce is captured into the same graph (RCCL graph capture);
      - comm='overlap': bucketed all-reduce launched from gradient hooks while the backward
        runs, on a side stream inside the same graph (grad_buckets.py).
    At world size 1 the whole step is one graph.
  * eager: torch DDP (bucketed all-reduce overlapped with backward) — CPU/gloo and debugging;
    `flat=True` runs the graph mode's flat-buffer algebra eagerly.
Host-side values a graph would freeze are guarded: ProgressiveScaling's scale count triggers a
re-capture when it changes; random flips (flip_lr_prob > 0) are refused in graph mode; a plain
torch optimizer's float learning rates must not change after capture (the fused optimizer
re-reads them every step).  The reference's per-step anomaly detection and `.item()` syncs are
not on the hot path: the non-finite check accumulates on the device, tested every
`check_every` steps.
"""
import contextlib
import math
import gc

import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP

from ..utils import horovod as hvd


def make_optimizer(model, depth_lr=1e-4, pose_lr=1e-4, name="Adam", **kw):
    """Adam with 'Depth' / 'Pose' param groups (model_wrapper.py:172-233)."""
    opt_cls = getattr(torch.optim, name)
    groups = []
    if getattr(model, "depth_net", None) is not None:
        groups.append({"name": "Depth", "params": list(model.depth_net.parameters()), "lr": depth_lr})
    if getattr(model, "pose_net", None) is not None:
        groups.append({"name": "Pose", "params": list(model.pose_net.parameters()), "lr": pose_lr})
    return opt_cls(groups, **kw)


class DDPTrainer:
    def __init__(self, model, optimizer, device, amp_dtype=torch.bfloat16, bucket_cap_mb=64,
                 check_every=0, graph=None, flat=None, bf16_weights=False, fused_optim=None, comm="split",
                 overlap_bucket_mb=16.0, force_comm=False):
        self.device = device
        self.model = model
        self.optimizer = optimizer
        self.amp_dtype = amp_dtype
        self.check_every = check_every
        self.step_idx = 0
        self.nonfinite = torch.zeros((), device=device)
        self.world = hvd.world_size()
        # dp: the gradient all-reduce runs (force_comm: also at world size 1, to exercise the
        # collective path on one device)
        self.dp = self.world > 1 or force_comm
        self.use_graph = (device.type == "cuda") if graph is None else graph
        if comm not in ("split", "graph", "overlap"):
            raise ValueError(f"comm must be 'split', 'graph' or 'overlap', got {comm!r}")
        self.comm = comm
        if comm != "split" and self.world > 1:
            import warnings
            warnings.warn(f"comm={comm!r} captures the RCCL collectives into the step graph; with more than one "
                          "rank this path has no recorded multi-GPU run yet (the default 'split' keeps the "
                          "all-reduce outside the graphs)", RuntimeWarning, stacklevel=2)
        # flat: gradients packed into one flat buffer + one all-reduce per step (the graph mode's
        # algebra; also runnable eagerly, e.g. on CPU/gloo for tests)
        self.flat = self.use_graph if flat is None else (flat or self.use_graph)
        self.graphs = None
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.mp = self.fused = None
        if bf16_weights:
            assert self.flat, "bf16 master weights need the flat (graph) gradient path"
            if fused_optim is None:
                fused_optim = device.type == "cuda"
            if fused_optim:  # one HIP kernel: grad widening + Adam + weight rounding (fused_adam.py)
                from .fused_adam import FusedMixedAdam
                self.fused = FusedMixedAdam(model, optimizer, device, lowp_dtype=amp_dtype or torch.bfloat16)
            else:
                from .mixed_precision import Bf16MasterWeights
                self.mp = Bf16MasterWeights(model, optimizer, dtype=amp_dtype or torch.bfloat16)
        # comm='overlap': gradient hooks feed the all-reduce buckets; the first backward only
        # records the order gradients become ready (the buckets' launch order)
        self.buckets, self._ready_order, self._capturing = None, None, False
        self.overlap = comm == "overlap" and self.flat and self.dp
        if self.overlap:
            if self.mp is not None:
                raise NotImplementedError("comm='overlap' needs the fused optimizer or fp32 weights")
            self.overlap_bytes = int(overlap_bucket_mb * (1 << 20))
            self._ready_order = []
            for p in self.params:
                p.register_post_accumulate_grad_hook(self._grad_ready)
        # BatchNorm step counters: host-side while graphs replay (see _detach_bn_counters)
        self._bn, self._bn_step0 = [], 0
        if self.flat:
            self._broadcast_initial()
            self.ddp = model
        elif self.world > 1:
            # static_graph: unused parameters (ResNetSAN01's LiDAR fusion weights) are detected once
            self.ddp = DDP(model, device_ids=[device.index] if device.type == "cuda" else None,
                           bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True, static_graph=True)
        else:
            self.ddp = model

    # ------------------------------------------------------------------------------------------
    def _broadcast_initial(self):
        if self.world > 1:  # identical initial weights on every rank
            for p in self.params:
                dist.broadcast(p.data, src=0)
            for b in self.model.buffers():
                dist.broadcast(b, src=0)
            if self.fused is not None:
                dist.broadcast(self.fused.master, src=0)
            if self.mp is not None:
                for mp in self.mp.master:
                    dist.broadcast(mp, src=0)

    def _grads(self):
        """(optimizer params with a gradient, their grads) — unused parameters keep grad None,
        like the reference (Adam then skips them).  With bf16 weights these are the fp32 masters."""
        ps = [p for g in self.optimizer.param_groups for p in g["params"] if p.grad is not None]
        return ps, [p.grad for p in ps]

    def _pack(self, capturing=False):
        if self.fused is not None:
            if not hasattr(self, "flat_grad"):
                self.flat_grad = self.fused.new_flat_grad()
            self.fused.pack(self.flat_grad, capturing)
            return
        _, grads = self._grads()
        if not hasattr(self, "flat_grad") or self.flat_grad.numel() != sum(g.numel() for g in grads):
            self.flat_grad = torch.empty(sum(g.numel() for g in grads), device=self.device, dtype=torch.float32)
        torch.cat([g.reshape(-1).float() for g in grads], out=self.flat_grad)

    def _unpack(self, scale):
        _, grads = self._grads()
        views, off = [], 0
        for g in grads:
            views.append(self.flat_grad[off:off + g.numel()].view_as(g))
            off += g.numel()
        if scale != 1.0:
            self.flat_grad.mul_(scale)
        torch._foreach_copy_(grads, views)

    def _grad_ready(self, p):
        if self.buckets is not None:
            self.buckets.on_grad(p)
        elif self._ready_order is not None:
            self._ready_order.append(p)

    def _build_buckets(self):
        from .grad_buckets import GradBuckets
        if self.fused is not None:
            ps = [p for p in self.fused.params if p.grad is not None]
            offs = [self.fused.offsets[self.fused._index[id(p)]] for p in ps]
        else:
            ps, _ = self._grads()
            offs, o = [], 0
            for p in ps:
                offs.append(o)
                o += p.numel()
        self.buckets = GradBuckets(ps, offs, self.flat_grad, self.overlap_bytes, self.device,
                                   fused=self.fused, order=self._ready_order)
        self._ready_order = None

    def autocast(self):
        if self.amp_dtype is None or self.device.type != "cuda":
            return contextlib.nullcontext()
        # no weight-cast cache: casts must be re-done inside every graph replay
        return torch.autocast(device_type="cuda", dtype=self.amp_dtype, cache_enabled=False)

    def _forward_backward(self, batch, progress):
        with self.autocast():
            output = self.ddp(batch, progress=progress)
        loss = output["loss"]
        if self.buckets is not None:
            self.buckets.arm(self._capturing)
        elif self._ready_order is not None:
            self._ready_order.clear()
        loss.sum().backward()
        if self.buckets is not None:   # join the bucket all-reduces launched during the backward
            self.buckets.finish()
        # sticky non-finite flag in one launch: 0 * loss is 0 for a finite loss, NaN otherwise
        # (the isfinite / any / cast / add chain was five kernels at the end of every step)
        ld = loss.detach()
        self.nonfinite.add_(ld.reshape(()) if ld.numel() == 1 else ld.float().sum(), alpha=0.0)
        if self.mp is not None:
            self.mp.grads_to_master()
        return output

    def _opt_step(self, capturing=False):
        if self.fused is not None:  # world > 1: Adam reads the all-reduced flat buffer directly
            if self.dp:
                if self.buckets is not None:  # bucket packs bound their own tables
                    self.fused.bind(capturing)
                self.fused.step(self.flat_grad, 1.0 / self.world, capturing)
            else:
                self.fused.step(None, 1.0, capturing)
            return
        self.optimizer.step()
        if self.mp is not None:
            self.mp.master_to_model()

    # ------------------------------------------------------------------------------------------
    def _snapshot(self):
        """Training state the warm-up steps mutate: weights, buffers (BN running stats),
        optimizer state (fused flat buffers or torch.optim per-parameter state)."""
        snap = {"params": [p.detach().clone() for p in self.params],
                "buffers": [b.detach().clone() for b in self.model.buffers()],
                "opt": {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                        for p, st in self.optimizer.state.items()}}
        if self.fused is not None:
            f = self.fused
            snap["fused"] = [t.clone() for t in (f.master, f.exp_avg, f.exp_avg_sq, f.step_count)]
        if self.mp is not None:
            snap["mp"] = [m.detach().clone() for m in self.mp.master]
        return snap

    @torch.no_grad()
    def _restore(self, snap):
        """In-place restore (the tensors keep their addresses: captured graphs hold them).
        Optimizer state created by the warm-up (lazy Adam state) is reset to its initial value."""
        for p, v in zip(self.params, snap["params"]):
            p.copy_(v)
        for b, v in zip(self.model.buffers(), snap["buffers"]):
            b.copy_(v)
        for p, st in self.optimizer.state.items():
            old = snap["opt"].get(id(p))
            for k, v in st.items():
                if not torch.is_tensor(v):
                    if old is not None and k in old:
                        st[k] = old[k]
                    continue
                if old is not None and k in old:
                    v.copy_(old[k])
                else:
                    v.zero_()
        if self.fused is not None:
            f = self.fused
            for t, v in zip((f.master, f.exp_avg, f.exp_avg_sq, f.step_count), snap["fused"]):
                t.copy_(v)
        if self.mp is not None:
            for m, v in zip(self.mp.master, snap["mp"]):
                m.copy_(v)

    def capture(self, static_batch, warmup=3, progress=0.0):
        """Warm up on a side stream (MIOpen algorithm selection, allocator) from a snapshot of
        the training state, restore it, then capture: the captured step is the first update."""
        assert self.use_graph
        if getattr(self.model, "flip_lr_prob", 0.0) > 0.0:
            raise NotImplementedError("graph mode freezes the host-side random flip (flip_lr_prob > 0): "
                                      "use graph=False")
        self.static_batch = static_batch
        self._detach_bn_counters()
        snap = self._snapshot()
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._zero_grad()
                self._forward_backward(static_batch, progress)
                self._allreduce()
                self._opt_step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._restore(snap)
        del snap
        gc.collect()   # nothing of the warm-up's autograd graphs may survive into the capture
        self.nonfinite.zero_()
        torch.cuda.synchronize(self.device)
        # grads None before capture: autograd allocates them from the graph pool (static
        # addresses, no accumulate kernels); every replay rewrites them
        self._zero_grad()
        inv_world = 1.0 / self.world
        if not self.dp or self.comm in ("graph", "overlap"):
            g = torch.cuda.CUDAGraph()
            self._capturing = True
            try:
                with torch.cuda.graph(g):
                    self.static_output = self._forward_backward(static_batch, progress)
                    if self.buckets is not None:
                        if self.fused is None:
                            self.buckets.unpack(inv_world)
                    elif self.dp:
                        self._pack(capturing=True)
                        dist.all_reduce(self.flat_grad, op=dist.ReduceOp.SUM)
                        if self.fused is None:
                            self._unpack(inv_world)
                    self._opt_step(capturing=True)
            finally:
                self._capturing = False
            self.graphs = (g,)
        else:
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1):
                self.static_output = self._forward_backward(static_batch, progress)
                self._pack(capturing=True)
            with torch.cuda.graph(g2, pool=g1.pool()):
                if self.fused is None:
                    self._unpack(inv_world)
                self._opt_step(capturing=True)
            self.graphs = (g1, g2)
        if self.fused is not None:  # gradient addresses of the captured graph -> kernel tables
            self.fused.finish_capture()
        if self.buckets is not None:
            self.buckets.finish_capture()
        self._captured_n = self._scale_count(progress)
        self._captured_lr = [g["lr"] for g in self.optimizer.param_groups]

    def _scale_count(self, progress):
        loss = getattr(self.model, "_photometric_loss", None)
        return loss.progressive_scaling(progress) if loss is not None else None

    def _detach_bn_counters(self):
        """BatchNorm's `num_batches_tracked += 1` is one kernel per BN layer per step and is only
        read when momentum is None (cumulative average).  With a fixed momentum the counters are
        taken out of the replayed step and kept on the host (base value + steps replayed);
        `state_dict()` / `bn_counters_to_model()` put the current value back."""
        if self._bn:
            return
        for m in self.model.modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and m.track_running_stats \
                    and m.momentum is not None and m.num_batches_tracked is not None:
                self._bn.append((m, int(m.num_batches_tracked)))
                m.num_batches_tracked = None
        self._bn_step0 = self.step_idx

    def _bn_count(self, base):
        return base + self.step_idx - self._bn_step0

    def bn_counters_to_model(self):
        """Write the BatchNorm step counters (value at capture + steps run) into the modules.
        Idempotent; replays keep counting on the host (the graphs never touch the tensors)."""
        for m, base in self._bn:
            m.num_batches_tracked = torch.tensor(self._bn_count(base), dtype=torch.long,
                                                 device=m.running_mean.device)

    def state_dict(self):
        """The SfmModel's own state_dict (keys 'depth_net.…' / 'pose_net.…', the layout
        SfmModel.load_state_dict takes) with fp32 master weights in place of the bf16 working
        copies and every BatchNorm `num_batches_tracked` present and current.  The reference's
        checkpoint FILE wraps ModelWrapper keys ('model.depth_net.…'): see checkpoint()."""
        sd = self.model.state_dict()
        names = {id(m): n for n, m in self.model.named_modules()}
        for m, base in self._bn:
            key = (names[id(m)] + "." if names[id(m)] else "") + "num_batches_tracked"
            sd[key] = torch.tensor(self._bn_count(base), dtype=torch.long)
        if self.fused is not None or self.mp is not None:
            pname = {id(p): n for n, p in self.model.named_parameters()}
            if self.fused is not None:
                for p in self.fused.params:
                    sd[pname[id(p)]] = self.fused.master_view(p).detach().clone()
            else:
                for p, m in zip(self.mp.lp, self.mp.master):
                    sd[pname[id(p)]] = m.detach().clone()
        return sd

    def checkpoint(self, config=None, epoch=0, scheduler=None):
        """The dict the reference's ModelCheckpoint saves (models/model_checkpoint.py:66-76):
        {'config', 'epoch', 'state_dict', 'optimizer', 'scheduler'} with 'state_dict' keyed as
        ModelWrapper.state_dict() is — the SfmModel under 'model.' — so utils/load.py
        load_network(net, ckpt['state_dict'], 'depth_net') strips the prefix as for a reference
        checkpoint.  Written with torch.save(), it loads with weights_only=True when `config` is None
        or a plain dict / list / scalar tree (a yacs CfgNode or another object would need the
        unpickling loader; pass config as a dict)."""
        sd = {"model." + k: v.detach().cpu() for k, v in self.state_dict().items()}
        return {"config": config, "epoch": int(epoch), "state_dict": sd,
                "optimizer": self.optimizer.state_dict(),
                "scheduler": scheduler.state_dict() if scheduler is not None else None}

    def _zero_grad(self):
        """Model grads -> None (autograd then owns fresh, graph-static tensors); the fp32 master
        grads of the bf16 path are persistent buffers, overwritten every step."""
        for p in self.params:
            p.grad = None
        if self.mp is None and self.fused is None:
            self.optimizer.zero_grad(set_to_none=True)

    def _allreduce(self):
        if not self.dp:
            return
        if self.buckets is not None:  # reduced bucket by bucket during the backward
            if self.fused is None:
                self.buckets.unpack(1.0 / self.world)
            return
        self._pack()
        dist.all_reduce(self.flat_grad, op=dist.ReduceOp.SUM)
        if self.fused is None:
            self._unpack(1.0 / self.world)
        if self.overlap and self._ready_order:   # first backward seen: cut the buckets
            self._build_buckets()

    # ------------------------------------------------------------------------------------------
    def train_step(self, batch, progress=0.0):
        """One optimizer step on `batch`.  Returns {'loss', 'metrics', ...}: loss and metrics are
        this step's own (detached copies — a replayed graph rewrites its static outputs); the
        other entries (inv_depths, poses) are the graph's static tensors in graph mode."""
        if self.fused is not None:
            self.fused.sync_hparams()  # lr schedulers act on optimizer.param_groups
        if self.use_graph:
            if self.graphs is not None and self._scale_count(progress) != self._captured_n:
                self._release_graphs()   # ProgressiveScaling changed the scale count: re-capture
            if self.graphs is None:
                self.capture(batch, progress=progress)
            elif batch is not self.static_batch:
                _copy_into(self.static_batch, batch)
            if self.fused is None and [g["lr"] for g in self.optimizer.param_groups] != self._captured_lr:
                raise RuntimeError("learning rate changed after the step was captured: a plain torch optimizer "
                                   "bakes float lr into the graph (use bf16_weights=True for the fused "
                                   "optimizer, or graph=False)")
            self.graphs[0].replay()
            if len(self.graphs) == 2:
                dist.all_reduce(self.flat_grad, op=dist.ReduceOp.SUM)
                self.graphs[1].replay()
            output = _step_output(self.static_output)
        elif self.flat:
            self._zero_grad()
            output = self._forward_backward(batch, progress)
            self._allreduce()
            self._opt_step()
        else:
            self.optimizer.zero_grad(set_to_none=True)
            output = self._forward_backward(batch, progress)
            self.optimizer.step()
        self.step_idx += 1
        if self.check_every and self.step_idx % self.check_every == 0:
            self.check_finite()
        return output

    def _release_graphs(self):
        torch.cuda.synchronize(self.device)
        self.graphs = None
        self.static_output = None
        for p in self.params:
            p.grad = None

    def check_finite(self):
        flag = self.nonfinite.clone()
        if self.dp and dist.is_initialized():
            dist.all_reduce(flag)
        if not math.isfinite(float(flag)):
            raise ValueError(f"Non-finite loss within the last steps (step {self.step_idx})")


def _step_output(static):
    out = dict(static)
    out["loss"] = static["loss"].detach().clone()
    if "metrics" in static:
        out["metrics"] = {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in static["metrics"].items()}
    return out


def _copy_into(dst, src):
    if torch.is_tensor(dst):
        dst.copy_(src, non_blocking=True)
    elif isinstance(dst, dict):
        for k in dst:
            _copy_into(dst[k], src[k])
    elif isinstance(dst, (list, tuple)):
        for d, s in zip(dst, src):
            _copy_into(d, s)
