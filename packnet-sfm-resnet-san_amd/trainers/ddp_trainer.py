"""Data-parallel trainer: one process per GPU, DDP with RCCL bucketed all-reduce over xGMI
(replaces packnet_sfm/trainers/horovod_trainer.py, whose Horovod is a mock — SURVEY.md §0.2).

Per step (horovod_trainer.py:222-284): zero_grad -> forward (depth/pose nets under bf16
autocast, photometric loss in fp32 on the HIP kernels) -> loss.backward() (DDP overlaps the
gradient all-reduce with backward) -> optimizer.step().  The reference's per-step
`torch.autograd.set_detect_anomaly(True)` and per-step `.item()` host syncs are not on the hot
path: the non-finite check accumulates on the device and is checked every `check_every` steps.
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
                 check_every=0):
        self.device = device
        self.model = model
        self.optimizer = optimizer
        self.amp_dtype = amp_dtype
        self.check_every = check_every
        self.step_idx = 0
        self.nonfinite = torch.zeros((), device=device)
        self.world = hvd.world_size()
        if self.world > 1:
            # static_graph: unused parameters (e.g. ResNetSAN01's LiDAR fusion weights) are
            # detected once; gradient buckets then reduce in a fixed order, overlapped with backward
            self.ddp = DDP(model, device_ids=[device.index] if device.type == "cuda" else None,
                           bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True, static_graph=True)
        else:
            self.ddp = model

    def autocast(self):
        if self.amp_dtype is None or self.device.type != "cuda":
            return contextlib.nullcontext()
        return torch.autocast(device_type="cuda", dtype=self.amp_dtype)

    def train_step(self, batch, progress=0.0):
        self.optimizer.zero_grad(set_to_none=True)
        with self.autocast():
            output = self.ddp(batch, progress=progress)
        loss = output["loss"]
        loss.sum().backward()
        self.optimizer.step()
        self.nonfinite += (~torch.isfinite(loss.detach())).any().float()
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
