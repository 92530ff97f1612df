"""Bucketed gradient all-reduce overlapped with the backward pass (DDPTrainer comm='overlap').

The reference averages gradients with Horovod's DistributedOptimizer (mocked in the fork,
packnet_sfm/utils/horovod.py; trainers/horovod_trainer.py:222-284 steps after the full
backward), whose real implementation fuses ready gradients into buffers and all-reduces them
while the backward is still running.  Here the flat fp32 all-reduce buffer of the trainer is cut
into contiguous buckets of consecutive parameters (about `cap_bytes` each); a post-accumulate
hook counts the gradients of each bucket, and when a bucket is complete its gradients are packed
into their slice of the flat buffer (one psfm_grad_pack launch through a per-bucket tensor
table on the fused path) and the slice is all-reduced — on a side stream for RCCL, so the
remaining backward kernels run while the collective is on the links.  `finish()` joins the side
stream (or waits the gloo works) before the optimizer reads the buffer.

Determinism across ranks: collectives must be issued in the same order on every rank, so buckets
are launched in a FIXED order (the completion order observed in the first, learning step); a
bucket completed early waits for its predecessors.  Inside a HIP-graph capture the hooks run
once, at capture time: the packs, the stream fork/join and the RCCL calls become graph nodes and
every replay re-runs them in the captured order.
"""
import ctypes

import numpy as np
import torch
import torch.distributed as dist

from .. import _hip


class GradBuckets:
    def __init__(self, params, offsets, flat, cap_bytes, device, fused=None, order=None):
        """params / offsets: parameters that receive a gradient every step and their element
        offsets in `flat` (increasing); `fused`: the FusedMixedAdam whose table layout `flat`
        follows (None: plain copies); `order`: parameters in the order their gradients became
        ready in the learning step (sets the bucket launch order)."""
        assert all(offsets[i] < offsets[i + 1] for i in range(len(offsets) - 1)), "offsets must increase"
        self.device, self.flat, self.fused = device, flat, fused
        self.buckets = []          # [(first param idx, end idx)]
        cap_el = max(1, int(cap_bytes) // 4)
        i = 0
        while i < len(params):
            j, start = i + 1, offsets[i]
            while j < len(params) and offsets[j] + params[j].numel() - start <= cap_el:
                j += 1
            self.buckets.append((i, j))
            i = j
        self.params, self.offsets = list(params), list(offsets)
        self.presence = None       # agreed once (agree_presence): which params have gradients
        self.bucket_of = {}
        for b, (i, j) in enumerate(self.buckets):
            for k in range(i, j):
                self.bucket_of[id(self.params[k])] = (b, k)
        self.ranges = [(offsets[i], offsets[j - 1] + params[j - 1].numel()) for i, j in self.buckets]
        if order is not None:
            first = {}
            for r, p in enumerate(order):
                b = self.bucket_of.get(id(p), (None,))[0]
                if b is not None:
                    first[b] = max(first.get(b, -1), r)   # a bucket completes with its last gradient
            self.launch_order = sorted(range(len(self.buckets)), key=lambda b: first.get(b, len(order)))
        else:
            self.launch_order = list(range(len(self.buckets)))[::-1]
        self.launch_order = self._agree(self.launch_order, device, self.ranges)
        self.stream = torch.cuda.Stream(device=device) if device.type == "cuda" else None
        self.armed = False
        self.capturing = False
        if fused is not None:
            self._plan_tables()

    @staticmethod
    def _agree(order, device, ranges):
        """Every rank must issue its bucket collectives in ONE order over the SAME bucket cuts, or the
        all-reduces pair up different buckets (a hang for different sizes, silently mixed slices for
        equal ones).  Rank 0's learned order is broadcast and adopted by all ranks (as torch DDP
        broadcasts its rebuilt bucket order); rank 0's cuts (flat element ranges) are broadcast too
        and every rank checks its own against them."""
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return order
        dev = device if dist.get_backend() == "nccl" else torch.device("cpu")
        cuts = [v for r in ranges for v in r]
        t = torch.tensor([len(order)] + list(order) + cuts, dtype=torch.int64, device=dev)
        # plan sizes first (every rank learns a mismatch: all raise together, none waits in a collective)
        n = torch.tensor([t.numel(), -t.numel()], dtype=torch.int64, device=dev)
        dist.all_reduce(n, op=dist.ReduceOp.MAX)
        if int(n[0]) != -int(n[1]):
            raise RuntimeError(f"ranks cut different buckets: plan sizes {-int(n[1])}..{int(n[0])} differ")
        dist.broadcast(t, src=0)
        got = [int(v) for v in t.cpu()]
        agreed, cuts0 = got[1:1 + len(order)], got[1 + len(order):]
        bad = torch.tensor([int(cuts0 != cuts or sorted(agreed) != sorted(order))], dtype=torch.int64, device=dev)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if int(bad):
            raise RuntimeError("ranks cut different buckets: a rank's flat ranges differ from rank 0's")
        return agreed

    # -------------------------------------------------------------------------------------------
    def _plan_tables(self):
        """Per-bucket device tables (psfm_optim_tensor rows) and chunk plans, allocated and
        planned before any capture (only the rows' gradient pointers change later)."""
        from .fused_adam import TENSOR_DT
        L = _hip.lib()
        self.tables, self.chunks, self.nchunks, self._pending = [], [], [], []
        for i, j in self.buckets:
            n = np.asarray([p.numel() for p in self.params[i:j]], np.int64)
            cnt = L.psfm_optim_plan_chunks(len(n), n.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), None, 0)
            _hip.check(min(cnt, 0), "psfm_optim_plan_chunks")
            ch = np.zeros(2 * max(cnt, 1), np.int32)
            rc = L.psfm_optim_plan_chunks(len(n), n.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                          ch.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), cnt)
            _hip.check(min(rc, 0), "psfm_optim_plan_chunks")
            self.chunks.append(torch.from_numpy(ch).to(self.device))
            self.nchunks.append(cnt)
            self.tables.append(torch.zeros((j - i) * TENSOR_DT.itemsize, device=self.device, dtype=torch.uint8))

    def arm(self, capturing=False):
        """Start of a backward: reset the per-bucket counters."""
        self.armed, self.capturing = True, capturing
        self.left = [j - i for i, j in self.buckets]
        self.done = [False] * len(self.buckets)
        self.next = 0
        self.works = []
        self.forked = False

    def on_grad(self, p):
        if not self.armed:
            return
        hit = self.bucket_of.get(id(p))
        if hit is None:
            raise RuntimeError("gradient of a parameter outside the all-reduce buckets (the set of "
                               "parameters receiving gradients changed)")
        b, _ = hit
        self.left[b] -= 1
        if self.left[b] == 0:
            self.done[b] = True
            self._launch_ready()

    def _launch_ready(self):
        while self.next < len(self.launch_order) and self.done[self.launch_order[self.next]]:
            self._launch(self.launch_order[self.next])
            self.next += 1

    def _pack(self, b):
        i, j = self.buckets[b]
        if self.fused is not None:
            from .fused_adam import TENSOR_DT
            rows = self.fused.rows_for(self.params[i:j])
            blob = torch.from_numpy(np.array(rows, dtype=TENSOR_DT).view(np.uint8).copy())
            if self.capturing:
                self._pending.append((b, blob))   # uploaded by finish_capture()
            else:
                self.tables[b][:blob.numel()].copy_(blob)
            L = _hip.lib()
            _hip.check(L.psfm_grad_pack(_hip.ptr(self.tables[b]), _hip.ptr(self.chunks[b]), self.nchunks[b],
                                        _hip.ptr(self.flat), _hip.stream(self.device)), "psfm_grad_pack")
        else:
            for k in range(i, j):
                g, off, p = self.params[k].grad, self.offsets[k], self.params[k]
                if g is None:   # no gradient this step (e.g. a scale dropped): its slice sums zeros
                    self.flat[off:off + p.numel()].zero_()
                else:
                    self.flat[off:off + g.numel()].view_as(g).copy_(g)

    def _launch(self, b):
        self._pack(b)
        a, e = self.ranges[b]
        view = self.flat[a:e]
        if self.stream is not None:
            # the collective waits for this bucket's pack on the side stream; the compute stream
            # runs on into the rest of the backward
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                dist.all_reduce(view, op=dist.ReduceOp.SUM)
            self.forked = True
        else:
            self.works.append(dist.all_reduce(view, op=dist.ReduceOp.SUM, async_op=True))

    def finish(self):
        """End of the backward: launch what is left (a parameter without a gradient this step
        keeps its bucket open until here), then join the collectives."""
        if not self.armed:
            return
        for b in range(len(self.buckets)):
            self.done[b] = True
        self._launch_ready()
        if self.stream is not None:
            if self.forked:
                torch.cuda.current_stream(self.device).wait_stream(self.stream)
        else:
            for w in self.works:
                w.wait()
        self.armed = False

    def finish_capture(self):
        for b, blob in self._pending if self.fused is not None else ():
            self.tables[b][:blob.numel()].copy_(blob)
        if self.fused is not None:
            self._pending = []

    def agree_presence(self):
        """Which parameters have a gradient, agreed across ranks (one small all-reduce of a flag per
        parameter and a host sync).  A parameter with a gradient on ANY rank gets the average on
        every rank (its slice summed zeros where it had none); one with no gradient anywhere stays
        None everywhere (the optimizer skips it, as for a single process)."""
        has = torch.tensor([p.grad is not None for p in self.params], dtype=torch.int32)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            has = has.to(self.device if dist.get_backend() == "nccl" else torch.device("cpu"))
            dist.all_reduce(has, op=dist.ReduceOp.SUM)
        self.presence = [bool(h) for h in has.tolist()]

    def unpack(self, scale):
        """Plain-optimizer path: averaged slices back into the parameters' .grad.  Eager steps agree
        on gradient presence every step (the set may change: a head that stops receiving
        gradients); inside a stream capture a pageable H2D copy, a collective on the capture stream
        and a .tolist() are not allowed, so a captured unpack is device ops only and uses the
        presence agreed by the last eager step (the trainer's warm-up): a graph replays one fixed
        backward, so its set is that step's."""
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            if self.presence is None:
                raise RuntimeError("grad_buckets.unpack: gradient presence must be agreed in an eager step "
                                   "before the capture (agree_presence)")
        else:
            self.agree_presence()
        for p, off, h in zip(self.params, self.offsets, self.presence):
            if not h:
                if p.grad is not None:
                    raise RuntimeError("grad_buckets.unpack: a parameter without a gradient in the agreed set "
                                       "has one now (the set of parameters with gradients must be static)")
                continue
            avg = self.flat[off:off + p.numel()].view(p.shape) * scale
            if p.grad is None:
                p.grad = avg.to(p.dtype)
            else:
                p.grad.copy_(avg.view_as(p.grad))
