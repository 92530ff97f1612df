"""Communication API of packnet_sfm/utils/horovod.py (hvd_init, rank, world_size, reduce_value,
allreduce, broadcast_*, DistributedOptimizer, print0, on_rank_0) backed by torch.distributed —
RCCL (backend 'nccl' on ROCm) over xGMI on GPUs, gloo on CPU.  The reference mocks every one of
these as an identity; here they are real collectives, and single-process runs
(no process group) behave like the mock."""
import os

import torch
import torch.distributed as dist


def _active():
    return dist.is_available() and dist.is_initialized()


def hvd_init(backend=None):
    """Initialise the process group from torchrun's env (RANK / WORLD_SIZE / MASTER_*)."""
    if _active() or int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local_rank())
    dist.init_process_group(backend=backend)


def on_rank_0(func):
    def wrapper(*args, **kwargs):
        if rank() == 0:
            func(*args, **kwargs)
    return wrapper


def rank():
    return dist.get_rank() if _active() else 0


def local_rank():
    return int(os.environ.get("LOCAL_RANK", "0"))


def size():
    return world_size()


def world_size():
    return dist.get_world_size() if _active() else 1


@on_rank_0
def print0(string="\n"):
    print(string)


def allreduce(tensor, average=True, name=""):
    if not _active():
        return tensor
    out = tensor.clone()
    dist.all_reduce(out, op=dist.ReduceOp.SUM)
    return out / world_size() if average else out


def reduce_value(value, average=True, name=""):
    """All-reduce a python scalar or tensor; returns the same kind it was given."""
    if not _active():
        return value
    is_t = torch.is_tensor(value)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = (value.detach().to(dev, torch.float64) if is_t else torch.tensor(float(value), dtype=torch.float64,
                                                                          device=dev))
    t = allreduce(t, average=average)
    return t.to(value.device, value.dtype) if is_t else float(t)


def broadcast_parameters(params, root_rank=0):
    if not _active():
        return
    items = params.items() if hasattr(params, "items") else params
    for _, p in items:
        dist.broadcast(p.data if hasattr(p, "data") else p, src=root_rank)


def broadcast_optimizer_state(optimizer, root_rank=0):
    if not _active():
        return
    for state in optimizer.state.values():
        for v in state.values():
            if torch.is_tensor(v):
                dist.broadcast(v, src=root_rank)


def DistributedOptimizer(optimizer, **kwargs):
    """Gradient averaging is done by DDP (bucketed RCCL all-reduce overlapped with backward,
    trainers/ddp_trainer.py); the optimizer itself is unchanged."""
    return optimizer


class Compression:
    none = None
    fp16 = None
