"""Fused mixed-precision Adam on the HIP C-ABI (include/psfm_optim.h).

Same update as `torch.optim.Adam` over the optimizer's param groups ('Depth' / 'Pose',
reference packnet_sfm/models/model_wrapper.py:172-216), with bf16 conv/linear weights and fp32
master weights — numerically the bf16 autocast training step of the reference's AMP path:
  * conv / linear weights are stored as bf16 = round(master); their gradients arrive in bf16 and
    are widened exactly inside the kernel; normalisation parameters stay fp32;
  * master weights and both Adam moments live in three flat fp32 buffers (one offset per tensor);
  * ONE kernel per step reads every gradient through a device table of tensor descriptors,
    updates master / exp_avg / exp_avg_sq and writes the rounded model weights back — instead of
    ~70 per-tensor cast kernels + the multi-tensor Adam launches.
The tables are read by the kernel at run time, so the launch is graph-capturable: gradients that
autograd allocates inside a HIP-graph capture have fixed addresses, recorded at capture and
uploaded once the capture has ended (`finish_capture`).
"""
import ctypes

import numpy as np
import torch
import torch.nn as nn

from .. import _hip

_LOWP_MODULES = (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.Linear)
GRAD_BF16, PARAM_BF16 = 1, 2
TENSOR_DT = np.dtype([("grad", "<u8"), ("param", "<u8"), ("numel", "<i8"), ("offset", "<i8"),
                      ("group", "<i4"), ("flags", "<i4")])
assert TENSOR_DT.itemsize == 40


def storage_flat(t):
    """1-D view of a dense tensor's elements in STORAGE order (channels_last included)."""
    if not (t.is_contiguous() or t.is_contiguous(memory_format=torch.channels_last)
            or t.is_contiguous(memory_format=torch.channels_last_3d)):
        raise RuntimeError(f"fused Adam needs dense parameters/gradients, got strides {t.stride()}")
    return t.as_strided((t.numel(),), (1,))


class FusedMixedAdam:
    def __init__(self, model, optimizer, device, lowp_dtype=torch.bfloat16):
        assert lowp_dtype == torch.bfloat16, "the kernel stores bf16 model weights"
        assert not optimizer.state, "build the fused optimizer before the first optimizer step"
        for g in optimizer.param_groups:
            if g.get("amsgrad") or g.get("maximize") or g.get("decoupled_weight_decay"):
                raise NotImplementedError("fused Adam: amsgrad / maximize / AdamW not supported")
        self.optimizer = optimizer
        self.device = device
        lowp = {id(p) for m in model.modules() if isinstance(m, _LOWP_MODULES)
                for p in m.parameters(recurse=False)}
        self.params, self.groups, self.offsets = [], [], []
        off, inits = 0, []
        for gi, g in enumerate(optimizer.param_groups):
            for p in g["params"]:
                if not p.requires_grad:
                    continue
                init = storage_flat(p.detach()).float().clone()
                if id(p) in lowp and p.dtype == torch.float32:
                    p.data = p.data.to(lowp_dtype)  # preserve_format keeps channels_last strides
                self.params.append(p)
                self.groups.append(gi)
                self.offsets.append(off)
                inits.append((off, init))
                off += (p.numel() + 3) // 4 * 4
        self.total = off
        self._index = {id(p): k for k, p in enumerate(self.params)}
        f32 = dict(device=device, dtype=torch.float32)
        self.master = torch.zeros(off, **f32)
        for o, init in inits:
            self.master[o:o + init.numel()].copy_(init)
        self.exp_avg = torch.zeros(off, **f32)
        self.exp_avg_sq = torch.zeros(off, **f32)
        self.flat_grad = None
        self.step_count = torch.zeros(1, device=device, dtype=torch.int32)
        self.hparams = torch.zeros((len(optimizer.param_groups), 8), **f32)
        self._hp_host = None
        self.sync_hparams()
        # device tables: fixed capacity + address (captured kernels hold these pointers)
        self.table = torch.zeros(len(self.params) * TENSOR_DT.itemsize, device=device, dtype=torch.uint8)
        max_chunks = sum((p.numel() + 1023) // 1024 for p in self.params)
        self.chunks = torch.zeros(2 * max(max_chunks, 1), device=device, dtype=torch.int32)
        self.nchunks = 0
        self._pending = None
        self._bound_key = None

    # -------------------------------------------------------------------------------------------
    def sync_hparams(self):
        """Copy lr / betas / eps / weight_decay of every param group to the device when they
        changed (e.g. by an lr scheduler) — host-side check, H2D copy only on change."""
        hp = np.zeros((len(self.optimizer.param_groups), 8), np.float32)
        for i, g in enumerate(self.optimizer.param_groups):
            b1, b2 = g.get("betas", (0.9, 0.999))
            hp[i, :5] = (float(g["lr"]), b1, b2, g.get("eps", 1e-8), g.get("weight_decay", 0.0))
        if self._hp_host is None or not np.array_equal(hp, self._hp_host):
            self.hparams.copy_(torch.from_numpy(hp))
            self._hp_host = hp

    def bind(self, capturing=False):
        """Describe the current gradients to the kernel (parameters without a gradient are
        skipped, like torch.optim.Adam).  Inside a graph capture the upload is deferred."""
        rows = self.rows_for(self.params)
        numels = [r[2] for r in rows]
        table = np.array(rows, dtype=TENSOR_DT)
        key = tuple(numels), tuple(r[3] for r in rows)
        if key != self._bound_key:
            n = np.asarray(numels, np.int64)
            L = _hip.lib()
            cnt = L.psfm_optim_plan_chunks(len(n), n.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), None, 0)
            _hip.check(min(cnt, 0), "psfm_optim_plan_chunks")
            ch = np.zeros(2 * max(cnt, 1), np.int32)
            rc = L.psfm_optim_plan_chunks(len(n), n.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                          ch.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(ch) // 2)
            _hip.check(min(rc, 0), "psfm_optim_plan_chunks")
            if capturing:
                raise RuntimeError("fused Adam: the set of gradients changed inside a graph capture")
            self.chunks[:ch.size].copy_(torch.from_numpy(ch))
            self.nchunks = cnt
            self._bound_key = key
        blob = torch.from_numpy(table.view(np.uint8).copy())
        if capturing:
            self._pending = blob
        else:
            self.table[:blob.numel()].copy_(blob)

    def rows_for(self, params):
        """Table rows (grad, param, numel, offset, group, flags) of those of `params` that have a
        gradient, in the given order."""
        rows = []
        for p in params:
            g = p.grad
            if g is None:
                continue
            k = self._index[id(p)]
            if g.dtype not in (torch.float32, torch.bfloat16) or g.stride() != p.stride():
                raise RuntimeError(f"fused Adam: gradient {g.dtype} {g.stride()} vs parameter {p.stride()}")
            storage_flat(g)
            flags = (GRAD_BF16 if g.dtype == torch.bfloat16 else 0) | \
                    (PARAM_BF16 if p.dtype == torch.bfloat16 else 0)
            rows.append((g.data_ptr(), p.data_ptr(), p.numel(), self.offsets[k], self.groups[k], flags))
        return rows

    def finish_capture(self):
        if self._pending is not None:
            self.table[:self._pending.numel()].copy_(self._pending)
            self._pending = None

    # -------------------------------------------------------------------------------------------
    def pack(self, flat_grad, capturing=False):
        """Gradients -> flat fp32 buffer (the all-reduce payload); padding stays zero."""
        self.bind(capturing)
        L = _hip.lib()
        _hip.check(L.psfm_grad_pack(_hip.ptr(self.table), _hip.ptr(self.chunks), self.nchunks,
                                    _hip.ptr(flat_grad), _hip.stream(self.device)), "psfm_grad_pack")

    def step(self, flat_grad=None, grad_scale=1.0, capturing=False):
        if flat_grad is None:
            self.bind(capturing)
        L = _hip.lib()
        _hip.check(L.psfm_adam_step(_hip.ptr(self.table), _hip.ptr(self.chunks), self.nchunks,
                                    _hip.ptr(self.hparams), _hip.ptr(self.step_count),
                                    _hip.ptr(flat_grad), ctypes.c_float(grad_scale), _hip.ptr(self.master),
                                    _hip.ptr(self.exp_avg), _hip.ptr(self.exp_avg_sq),
                                    _hip.stream(self.device)), "psfm_adam_step")

    def new_flat_grad(self):
        return torch.zeros(self.total, device=self.device, dtype=torch.float32)

    # -------------------------------------------------------------------------------------------
    def master_view(self, p):
        """fp32 master weight of model parameter p, shaped (and strided) like p."""
        i = next(k for k, q in enumerate(self.params) if q is p)
        flat = self.master[self.offsets[i]:self.offsets[i] + p.numel()]
        return flat.as_strided(p.shape, p.stride())
