"""Data-parallel trainer: one process per GPU, RCCL all-reduce of gradients over xGMI (replaces
packnet_sfm/trainers/horovod_trainer.py, whose Horovod is a mock — SURVEY.md §0.2).

Per step (horovod_trainer.py:222-284): zero_grad -> forward (depth/pose nets under bf16
autocast, photometric loss in fp32 on the HIP kernels) -> backward -> gradient average across
ranks -> optimizer.step().

Two execution modes:
  * graph (default on a ROCm device): the step is captured into HIP graphs once and replayed —
    the eager step is host-bound (~1.5k launches, MIOpen host overhead).
    Autograd writes each gradient into its own (graph-static) tensor; for world size > 1 they are
    packed into ONE flat fp32 buffer (one batched copy), averaged by a single RCCL all-reduce
    between two graph replays (fwd+bwd+pack graph | all_reduce | unpack+Adam graph) and unpacked
    (one foreach copy).  At world size 1 the whole step is one graph.
  * eager: torch DDP (bucketed all-reduce overlapped with backward) — CPU/gloo and debugging.
The reference's per-step anomaly detection and `.item()` syncs are not on the hot path: the
non-finite check accumulates on the device and is tested every `check_every` steps.
"""
import contextlib

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
                 check_every=0, graph=None, flat=None, bf16_weights=False, fused_optim=None):
        self.device = device
        self.model = model
        self.optimizer = optimizer
        self.amp_dtype = amp_dtype
        self.check_every = check_every
        self.step_idx = 0
        self.nonfinite = torch.zeros((), device=device)
        self.world = hvd.world_size()
        self.use_graph = (device.type == "cuda") if graph is None else graph
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

    def autocast(self):
        if self.amp_dtype is None or self.device.type != "cuda":
            return contextlib.nullcontext()
        # no weight-cast cache: casts must be re-done inside every graph replay
        return torch.autocast(device_type="cuda", dtype=self.amp_dtype, cache_enabled=False)

    def _forward_backward(self, batch, progress):
        with self.autocast():
            output = self.ddp(batch, progress=progress)
        loss = output["loss"]
        loss.sum().backward()
        self.nonfinite += (~torch.isfinite(loss.detach())).any().float()
        if self.mp is not None:
            self.mp.grads_to_master()
        return output

    def _opt_step(self, capturing=False):
        if self.fused is not None:  # world > 1: Adam reads the all-reduced flat buffer directly
            if self.world > 1:
                self.fused.step(self.flat_grad, 1.0 / self.world, capturing)
            else:
                self.fused.step(None, 1.0, capturing)
            return
        self.optimizer.step()
        if self.mp is not None:
            self.mp.master_to_model()

    # ------------------------------------------------------------------------------------------
    def capture(self, static_batch, warmup=3, progress=0.0):
        """Warm up on a side stream (MIOpen algorithm selection, allocator), then capture."""
        assert self.use_graph
        self.static_batch = static_batch
        self._detach_bn_counters(warmup)
        inv_world = 1.0 / self.world
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
        self.nonfinite.zero_()
        # grads None before capture: autograd allocates them from the graph pool (static
        # addresses, no accumulate kernels); every replay rewrites them
        self._zero_grad()
        if self.world == 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.static_output = self._forward_backward(static_batch, progress)
                self._opt_step(capturing=True)
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

    def _detach_bn_counters(self, warmup):
        """BatchNorm's `num_batches_tracked += 1` is one kernel per BN layer per step and is only
        read when momentum is None (cumulative average).  With a fixed momentum the counters are
        taken out of the replayed step and kept on the host; `bn_counters_to_model()` writes them
        back (state_dict compatible with the reference's checkpoints)."""
        self._bn = []
        for m in self.model.modules():
            if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and m.track_running_stats \
                    and m.momentum is not None and m.num_batches_tracked is not None:
                self._bn.append((m, m.num_batches_tracked))
                m.num_batches_tracked = None
        self._bn_warmup, self._bn_step0 = warmup, self.step_idx

    def bn_counters_to_model(self):
        """Re-attach the BatchNorm step counters (value = counter at capture + steps run)."""
        for m, t in getattr(self, "_bn", []):
            t.add_(self._bn_warmup + self.step_idx - self._bn_step0)
            m.num_batches_tracked = t
        self._bn = []

    def _zero_grad(self):
        """Model grads -> None (autograd then owns fresh, graph-static tensors); the fp32 master
        grads of the bf16 path are persistent buffers, overwritten every step."""
        for p in self.params:
            p.grad = None
        if self.mp is None and self.fused is None:
            self.optimizer.zero_grad(set_to_none=True)

    def _allreduce(self):
        if self.world > 1:
            self._pack()
            dist.all_reduce(self.flat_grad, op=dist.ReduceOp.SUM)
            if self.fused is None:
                self._unpack(1.0 / self.world)

    # ------------------------------------------------------------------------------------------
    def train_step(self, batch, progress=0.0):
        if self.fused is not None:
            self.fused.sync_hparams()  # lr schedulers act on optimizer.param_groups
        if self.use_graph:
            if self.graphs is None:
                self.capture(batch, progress=progress)
            elif batch is not self.static_batch:
                _copy_into(self.static_batch, batch)
            if self.world == 1:
                self.graphs[0].replay()
            else:
                self.graphs[0].replay()
                dist.all_reduce(self.flat_grad, op=dist.ReduceOp.SUM)
                self.graphs[1].replay()
            output = self.static_output
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

    def check_finite(self):
        flag = self.nonfinite.clone()
        if self.world > 1 and dist.is_initialized():
            dist.all_reduce(flag)
        if float(flag) > 0:
            raise ValueError(f"Non-finite loss within the last steps (step {self.step_idx})")


def _copy_into(dst, src):
    if torch.is_tensor(dst):
        dst.copy_(src, non_blocking=True)
    elif isinstance(dst, dict):
        for k in dst:
            _copy_into(dst[k], src[k])
    elif isinstance(dst, (list, tuple)):
        for d, s in zip(dst, src):
            _copy_into(d, s)
