"""Fused normalisation / activation layers of the depth and pose networks on HIP
(include/psfm_netops.h, csrc/psfm_netops.hip).

Each helper takes the modules the reference builds (nn.BatchNorm2d, nn.GroupNorm, nn.Conv2d
bias) — parameters, buffers and state_dict layout are unchanged — and on a ROCm device with bf16
NHWC (channels_last) activations runs one fused kernel pair instead of the reference's op chain:

  bn_act(x, bn, relu, residual)   BatchNorm2d (train) [+ identity] [+ ReLU]
                                  (resnet_encoder.py:16-98 BasicBlock / stem / downsample)
  bias_act(x, bias, act)          Conv2d bias add + ReLU / Sigmoid (layers.py:44-51, depth_decoder.py:60)
  gn_act(x, bias, gn, relu)       Conv2d bias + GroupNorm(16) + ReLU (PoseNet.py:15-19)

Anything else (CPU tensors, fp32 activations, eval-mode BatchNorm, momentum=None) runs the same
math as plain torch ops — that is the reference's own path, not a fallback of a HIP kernel:
the photometric loss (losses/_hip_photometric.py) has no such path.
"""
import ctypes

import numpy as np
import torch
import torch.nn.functional as F

from ... import _hip

ACT_NONE, ACT_RELU, ACT_SIGMOID = 0, 1, 2
# Which layer kinds run fused, from the A/B of the ResNetSAN01 + PoseNet step on MI355X
# (profiles/r02/netops_ab): conv bias + ReLU / sigmoid and bias + GroupNorm + ReLU beat the op
# chain (972 -> 1025 img/s together).  BatchNorm: "resident" = the one-launch resident kernels where
# a workgroup holds the layer (psfm_bn_act_resident: ResNet18 layer3 / layer4), MIOpen's BatchNorm
# elsewhere; "all" = every shape the library's fused BatchNorm takes (psfm_bn_act_fused: the same on
# the product library; A/B builds add the two-launch ticket kernels, which lost: profiles/r05/bn);
# False = MIOpen everywhere.  bench.py --fused-nets overrides.
FUSE = {"bias": True, "gn": True, "bn": "resident"}


def _fusable(x, kind):
    return FUSE[kind] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4


def _rows(t):
    """NHWC storage as an [M, C] matrix (copy only if not already channels_last)."""
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


# Forked outputs.  A tensor read by k consumers gets k gradients, which autograd sums with k - 1
# bf16 add kernels (CUDAFunctor_add) before the producer's backward runs.  A fused op asked for
# `nout` outputs returns its result plus nout - 1 views of it (the same memory, no copy): each
# consumer takes its own, autograd hands the producer's backward one gradient per view, and the
# backward kernel sums them in its load (one bf16 rounding per sum, as autograd's add).
FORK = True   # bench.py --no-fork: the plain output handed to every consumer (autograd's adds)


def _fork(y, nout):
    return y if nout == 1 else (y,) + tuple(y.view_as(y) for _ in range(nout - 1))


def _apply_fork(fn, nout, *args):
    """fn.apply(*args, nout) — or, FORK off, the single output handed to nout consumers."""
    if FORK or nout == 1:
        return fn.apply(*args, nout)
    return fork_plain(fn.apply(*args, 1), nout)


def _grads(dys, like):
    """The non-None gradients of a forked output (at least one; zeros if autograd passed none)."""
    gs = [g for g in dys if g is not None]
    return gs if gs else [torch.zeros_like(like)]


def fork_plain(y, nout):
    """The reference op chain's result handed to nout consumers (autograd sums their gradients)."""
    return y if nout == 1 else (y,) * nout


# ----------------------------------------------------------------------------------------------
class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act, nout=1):
        _hip.note_forward(ctx)
        x = _rows(x)
        N, C, H, W = x.shape
        M = N * H * W
        y = torch.empty_like(x, dtype=torch.float32 if act == ACT_SIGMOID else x.dtype,
                             memory_format=torch.channels_last)
        L = _hip.lib()
        _hip.check(L.psfm_bias_act_fwd(_hip.ptr(x), _hip.ptr(bias), int(bias.dtype == torch.bfloat16), M, C, act,
                                       _hip.ptr(y), _hip.stream(x.device)), "psfm_bias_act_fwd")
        ctx.save_for_backward(y)
        ctx.act, ctx.bias_dtype, ctx.x_dtype = act, bias.dtype, x.dtype
        return _fork(y, nout)

    @staticmethod
    def backward(ctx, *dys):
        _hip.capture_guard(ctx)
        (y,) = ctx.saved_tensors
        gs = [_rows(g.to(y.dtype)) for g in _grads(dys, y)]
        while len(gs) > 2:   # (a decoder output has at most two consumers)
            gs = [gs[0] + gs[1]] + gs[2:]
        N, C, H, W = y.shape
        M = N * H * W
        L = _hip.lib()
        dx = torch.empty_like(y, dtype=ctx.x_dtype, memory_format=torch.channels_last)
        db = torch.empty(C, device=y.device, dtype=ctx.bias_dtype)
        ws = torch.empty(L.psfm_netops_ws_floats(M, C), device=y.device, dtype=torch.float32)
        _hip.check(L.psfm_bias_act_bwd_sum(_hip.ptr(gs[0]), _hip.ptr(gs[1] if len(gs) > 1 else None), _hip.ptr(y),
                                           M, C, ctx.act, _hip.ptr(dx), _hip.ptr(db),
                                           int(ctx.bias_dtype == torch.bfloat16), _hip.ptr(ws),
                                           _hip.stream(y.device)), "psfm_bias_act_bwd")
        return dx, db, None, None


def bias_act(x, bias, act, module=None, nout=1):
    """act(x + bias): x = conv output WITHOUT its bias (F.conv2d(..., None)).  Sigmoid outputs are
    fp32 (they feed the fp32 photometric loss).  nout > 1 (ReLU / none): a tuple of nout views for
    nout consumers, whose gradients the backward kernel sums (_fork).  `module` (unused: the
    reductions need no device state) is kept for the call sites."""
    if _fusable(x, "bias") and bias is not None and (nout == 1 or act != ACT_SIGMOID):
        return _apply_fork(_BiasAct, nout, x, bias, act)
    y = x if bias is None else x + bias.to(x.dtype).view(1, -1, 1, 1)
    if act == ACT_RELU:
        y = torch.relu(y)
    elif act == ACT_SIGMOID:
        y = torch.sigmoid(y.float()) if x.is_cuda else torch.sigmoid(y)
    return fork_plain(y, nout)


def conv_nobias(conv, x):
    """The reference Conv2d without its bias term (the bias goes into the fused epilogue)."""
    return F.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)


# ----------------------------------------------------------------------------------------------
class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, momentum, eps, relu, nout=1):
        _hip.note_forward(ctx)
        x = _rows(x)
        N, C, H, W = x.shape
        M = N * H * W
        dev = x.device
        res = _rows(residual.to(x.dtype)) if residual is not None else None
        y = torch.empty_like(x, memory_format=torch.channels_last)
        mean = torch.empty(C, device=dev, dtype=torch.float32)
        invstd = torch.empty(C, device=dev, dtype=torch.float32)
        L = _hip.lib()
        # the form is decided once, here; the backward reuses it (a knob changed in between must not
        # send the backward down another path, or leave it without the workspace it needs)
        resident = bool(L.psfm_bn_act_resident(M, C))
        ws = None if resident else torch.empty(L.psfm_netops_ws_floats(M, C), device=dev, dtype=torch.float32)
        _hip.check(L.psfm_bn_act_fwd(_hip.ptr(x), _hip.ptr(res), _hip.ptr(weight), _hip.ptr(bias),
                                     _hip.ptr(running_mean), _hip.ptr(running_var), ctypes.c_float(momentum),
                                     ctypes.c_float(eps), M, C, int(relu), _hip.ptr(y), _hip.ptr(mean),
                                     _hip.ptr(invstd), _hip.ptr(ws), _hip.stream(dev)), "psfm_bn_act_fwd")
        ctx.save_for_backward(x, y, weight, mean, invstd)
        ctx.relu, ctx.has_res, ctx.resident = relu, residual is not None, resident
        return _fork(y, nout)

    @staticmethod
    def backward(ctx, *dys):
        _hip.capture_guard(ctx)
        x, y, weight, mean, invstd = ctx.saved_tensors
        gs = [_rows(g.to(x.dtype)) for g in _grads(dys, y)]
        N, C, H, W = x.shape
        M = N * H * W
        dev = x.device
        L = _hip.lib()
        resident = ctx.resident
        while len(gs) > 3:   # the kernels sum up to three gradients in their loads
            gs = [gs[0] + gs[1]] + gs[2:]
        dy = gs[0]
        dy1, dy2 = (gs + [None, None])[1:3]
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dres = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_res else None
        dw = torch.empty(C, device=dev, dtype=torch.float32)
        db = torch.empty(C, device=dev, dtype=torch.float32)
        ws = None if resident else torch.empty(L.psfm_netops_ws_floats(M, C), device=dev, dtype=torch.float32)
        _hip.check(L.psfm_bn_act_bwd_sum(_hip.ptr(dy), _hip.ptr(dy1), _hip.ptr(dy2), _hip.ptr(y), _hip.ptr(x),
                                         _hip.ptr(weight), _hip.ptr(mean), _hip.ptr(invstd), M, C, int(ctx.relu),
                                         _hip.ptr(dx), _hip.ptr(dres), _hip.ptr(dw), _hip.ptr(db), _hip.ptr(ws),
                                         _hip.stream(dev)), "psfm_bn_act_bwd")
        return dx, dw.to(weight.dtype), db.to(weight.dtype), dres, None, None, None, None, None, None


class _AddReLU(torch.autograd.Function):
    """relu(a [+ b]) on bf16 (include/psfm_netops.h psfm_add_relu_fwd / psfm_relu_mask_bwd_sum): the
    BasicBlock tail after MIOpen's BatchNorm (and, b = None, the stem's ReLU), one pass each way
    instead of add + relu / the ReLU backward (the add's backward is the identity to both inputs);
    nout > 1 forks the output (_fork) and the mask pass sums its gradients."""

    @staticmethod
    def forward(ctx, a, b, nout=1):
        _hip.note_forward(ctx)
        y = torch.empty_like(a)
        _hip.check(_hip.lib().psfm_add_relu_fwd(_hip.ptr(a), _hip.ptr(b), a.numel(), _hip.ptr(y),
                                                _hip.stream(a.device)), "psfm_add_relu_fwd")
        ctx.save_for_backward(y)
        ctx.has_b = b is not None
        return _fork(y, nout)

    @staticmethod
    def backward(ctx, *dys):
        _hip.capture_guard(ctx)
        (y,) = ctx.saved_tensors
        gs = [g.contiguous(memory_format=_fmt(y)) for g in _grads(dys, y)]
        while len(gs) > 3:
            gs = [gs[0] + gs[1]] + gs[2:]
        dy1, dy2 = (gs + [None, None])[1:3]
        dz = torch.empty_like(y)
        _hip.check(_hip.lib().psfm_relu_mask_bwd_sum(_hip.ptr(gs[0]), _hip.ptr(dy1), _hip.ptr(dy2), _hip.ptr(y),
                                                     y.numel(), _hip.ptr(dz), _hip.stream(y.device)),
                   "psfm_relu_mask_bwd")
        return dz, (dz if ctx.has_b else None), None


def _fmt(t):
    return torch.channels_last if (t.dim() == 4 and not t.is_contiguous()
                                   and t.is_contiguous(memory_format=torch.channels_last)) else torch.contiguous_format


ADD_RELU = True   # the BasicBlock tail on HIP (bench.py --no-add-relu: the op chain)


def add_relu(a, b, nout=1):
    """relu(a + b) (b None: relu(a)): ONE HIP pass each way for bf16 tensors of the same shape and
    layout on a ROCm device (the ResNet BasicBlock's `out += identity; relu(out)`); otherwise the op
    chain.  nout > 1: a tuple for nout consumers (_fork)."""
    if (ADD_RELU and a.is_cuda and a.dtype == torch.bfloat16 and a.numel() % 8 == 0
            and a.is_contiguous(memory_format=_fmt(a))
            and (b is None or (b.dtype == torch.bfloat16 and a.shape == b.shape and a.device == b.device
                               and _fmt(a) == _fmt(b) and b.is_contiguous(memory_format=_fmt(b))))):
        return _apply_fork(_AddReLU, nout, a, b)
    return fork_plain(torch.relu(a if b is None else a + b), nout)


def _bn_fused_shape(x):
    """FUSE["bn"] == "resident": the shapes the one-launch kernels hold (psfm_bn_act_resident); else
    every shape the library's fused BatchNorm takes (psfm_bn_act_fused)."""
    N, C, H, W = x.shape
    L = _hip.lib()
    return bool(L.psfm_bn_act_resident(N * H * W, C) if FUSE["bn"] == "resident" else L.psfm_bn_act_fused(N * H * W, C))


def bn_act(x, bn, relu=True, residual=None, nout=1):
    """act(bn(x) [+ residual]) with the reference's BatchNorm2d module `bn` (torchvision BasicBlock
    conv -> bn -> relu and conv -> bn -> +identity -> relu, resnet_encoder.py:61-98): ONE HIP launch
    each way where FUSE["bn"] takes the shape, else MIOpen's BatchNorm + the add / ReLU passes.
    nout > 1: a tuple of nout views for nout consumers, whose gradients the backward sums (_fork)."""
    if (_fusable(x, "bn") and bn.training and bn.track_running_stats and bn.momentum is not None and bn.affine
            and bn.running_mean is not None and (residual is None or residual.shape == x.shape)
            and _bn_fused_shape(x)):
        if bn.num_batches_tracked is not None:  # the graph trainer keeps these off the step
            bn.num_batches_tracked.add_(1)
        return _apply_fork(_BNAct, nout, x, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var,
                           float(bn.momentum), float(bn.eps), bool(relu))
    y = bn(x)
    if relu and (residual is None or residual.dtype == y.dtype):
        return add_relu(y, residual, nout)
    if residual is not None:
        y = y + residual
    return fork_plain(torch.relu(y) if relu else y, nout)


NET_INPUTS = True   # the nets' bf16 input images in one HIP pass (bench.py --no-net-inputs: ATen's chain)


def _autocast_bf16():
    return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16


def normalize_input(x, sub=0.45, div=0.225):
    """(x - sub) / div, the depth encoder's input normalisation (resnet_encoder.py:89).  Under bf16
    autocast on a ROCm device (where the first convolution casts it to bf16 anyway) ONE HIP pass
    (include/psfm_netops.h psfm_normalize_bf16) returns that bf16 tensor, bit for bit what ATen's sub,
    div (x * fp32 reciprocal) and cast give, in x's layout; otherwise the op chain."""
    if (NET_INPUTS and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and not x.requires_grad
            and _autocast_bf16() and (x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last))
            and x.data_ptr() % 16 == 0):
        y = torch.empty_like(x, dtype=torch.bfloat16)
        if y.stride() == x.stride():
            mul = float(np.float32(1.0) / np.float32(div))
            _hip.check(_hip.lib().psfm_normalize_bf16(_hip.ptr(x), x.numel(), ctypes.c_float(sub), ctypes.c_float(mul),
                                                      _hip.ptr(y), _hip.stream(x.device)), "psfm_normalize_bf16")
            return y
    return (x - sub) / div


def cat_input(images):
    """torch.cat(images, 1), PoseNet's input (target + contexts, PoseNet.py).  Under bf16 autocast on a
    ROCm device with channels_last fp32 images: ONE HIP pass (psfm_cat_channels_bf16) into the bf16
    channels_last tensor the first convolution would cast the concatenation to; otherwise torch.cat."""
    x0 = images[0]
    if (NET_INPUTS and 1 <= len(images) <= 4 and _autocast_bf16() and all(
            t.is_cuda and t.dtype == torch.float32 and t.dim() == 4 and not t.requires_grad
            and t.device == x0.device and t.shape[0] == x0.shape[0] and t.shape[2:] == x0.shape[2:]
            and t.is_contiguous(memory_format=torch.channels_last) for t in images)):
        N, _, H, W = x0.shape
        cs = [int(t.shape[1]) for t in images]
        y = torch.empty((N, sum(cs), H, W), device=x0.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        P, CI = ctypes.c_void_p * len(images), ctypes.c_int * len(images)
        _hip.check(_hip.lib().psfm_cat_channels_bf16(len(images), P(*[t.data_ptr() for t in images]), CI(*cs),
                                                     N * H * W, _hip.ptr(y), _hip.stream(x0.device)),
                   "psfm_cat_channels_bf16")
        return y
    return torch.cat(images, 1)


class _ReLUMaxPool(torch.autograd.Function):
    """The ResNet stem's relu -> MaxPool2d(3, 2, 1) (include/psfm_netops.h psfm_relu_maxpool_fwd/bwd):
    one pass each way for the ReLU, the pooling (uint8 window positions instead of ATen's int64
    indices) and, backward, the pooled output's second consumer's add, the skip's add and the ReLU
    mask.  Outputs: (relu(y) — the decoder skip, pooled [, its fork view])."""

    @staticmethod
    def forward(ctx, y, nout=2):
        _hip.note_forward(ctx)
        N, C, H, W = y.shape
        r = torch.empty_like(y, memory_format=torch.channels_last)
        # allocated channels_last (empty(...).contiguous(channels_last) would launch a copy of garbage)
        p = torch.empty((N, C, H // 2, W // 2), device=y.device, dtype=y.dtype, memory_format=torch.channels_last)
        am = torch.empty((N, C, H // 2, W // 2), device=y.device, dtype=torch.uint8, memory_format=torch.channels_last)
        _hip.check(_hip.lib().psfm_relu_maxpool_fwd(_hip.ptr(y), N, H, W, C, _hip.ptr(r), _hip.ptr(p), _hip.ptr(am),
                                                    _hip.stream(y.device)), "psfm_relu_maxpool_fwd")
        ctx.save_for_backward(r, am)
        return (r,) + _fork(p, nout) if nout > 1 else (r, p)

    @staticmethod
    def backward(ctx, dskip, *dps):
        _hip.capture_guard(ctx)
        r, am = ctx.saved_tensors
        N, C, H, W = r.shape
        gs = [_rows(g.to(r.dtype)) for g in dps if g is not None]
        if not gs:
            gs = [torch.zeros((N, C, H // 2, W // 2), device=r.device, dtype=r.dtype, memory_format=torch.channels_last)]
        while len(gs) > 2:
            gs = [gs[0] + gs[1]] + gs[2:]
        dskip = None if dskip is None else _rows(dskip.to(r.dtype))
        dx = torch.empty_like(r, memory_format=torch.channels_last)
        _hip.check(_hip.lib().psfm_relu_maxpool_bwd(_hip.ptr(gs[0]), _hip.ptr(gs[1] if len(gs) > 1 else None),
                                                    _hip.ptr(dskip), _hip.ptr(r), _hip.ptr(am), N, H, W, C,
                                                    _hip.ptr(dx), _hip.stream(r.device)), "psfm_relu_maxpool_bwd")
        return dx, None


STEM_POOL = True   # the stem's relu + max-pool on HIP (bench.py --no-stem-pool: add_relu + ATen's max-pool)


def _stem_pool_ok(y, pool):
    N, C, H, W = y.shape
    k, s, p = (pool.kernel_size, pool.stride, pool.padding)
    return (STEM_POOL and y.is_cuda and y.dtype == torch.bfloat16 and y.dim() == 4
            and y.is_contiguous(memory_format=torch.channels_last) and H % 2 == 0 and W % 2 == 0 and C % 8 == 0
            and k in (3, (3, 3)) and s in (2, (2, 2)) and p in (1, (1, 1)) and pool.dilation in (1, (1, 1))
            and not pool.ceil_mode and not pool.return_indices)


def bn_relu_maxpool(x, bn, pool, nout=2):
    """The ResNet stem after conv1 (torchvision ResNet through resnet_encoder.py:89-92):
    skip = relu(bn(x)), pooled = pool(skip).  Returns (skip, pooled) or, nout = 2, (skip, pooled,
    pooled's fork view) for layer1's first block (conv1 and identity).  Where the fused BatchNorm
    does not take the stem (MIOpen's BatchNorm runs it: M = N * H * W rows is beyond the resident
    kernels) the ReLU and the pooling run as ONE HIP pass each way (_ReLUMaxPool)."""
    if not (_fusable(x, "bn") and _bn_fused_shape(x)):
        y = bn(x)
        if _stem_pool_ok(y, pool):
            if FORK or nout == 1:
                return _ReLUMaxPool.apply(y, nout)
            skip, h = _ReLUMaxPool.apply(y, 1)
            return (skip,) + fork_plain(h, nout)
        xr, skip = add_relu(y, None, 2)
    else:
        xr, skip = bn_act(x, bn, relu=True, nout=2)
    h = pool(xr)
    return (skip,) + fork_plain(h, nout) if nout > 1 else (skip, h)


# ----------------------------------------------------------------------------------------------
class _GNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, bias, weight, beta, G, eps, act):
        _hip.note_forward(ctx)
        x = _rows(x)
        res = _rows(res.to(x.dtype)) if res is not None else None
        N, C, H, W = x.shape
        HW = H * W
        dev = x.device
        y = torch.empty_like(x, memory_format=torch.channels_last)
        mean = torch.empty(N * G, device=dev, dtype=torch.float32)
        invstd = torch.empty(N * G, device=dev, dtype=torch.float32)
        L = _hip.lib()
        ws = torch.empty(L.psfm_gn_ws_floats(N, HW, C, G), device=dev, dtype=torch.float32)
        bf = int(bias is not None and bias.dtype == torch.bfloat16)
        _hip.check(L.psfm_gn_act_fwd(_hip.ptr(x), _hip.ptr(res), _hip.ptr(bias), bf, _hip.ptr(weight), _hip.ptr(beta),
                                     ctypes.c_float(eps), N, HW, C, G, int(act), _hip.ptr(y), _hip.ptr(mean),
                                     _hip.ptr(invstd), _hip.ptr(ws), _hip.stream(dev)), "psfm_gn_act_fwd")
        ctx.save_for_backward(x, res, bias, weight, beta, mean, invstd)
        ctx.G, ctx.act = G, act
        return y

    @staticmethod
    def backward(ctx, dy):
        _hip.capture_guard(ctx)
        x, res, bias, weight, beta, mean, invstd = ctx.saved_tensors
        dy = _rows(dy.to(x.dtype))
        N, C, H, W = x.shape
        HW, G = H * W, ctx.G
        dev = x.device
        L = _hip.lib()
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dres = torch.empty_like(x, memory_format=torch.channels_last) if res is not None else None
        dbias = torch.empty(C, device=dev, dtype=bias.dtype) if bias is not None else None
        dw = torch.empty(C, device=dev, dtype=torch.float32)
        db = torch.empty(C, device=dev, dtype=torch.float32)
        ws = torch.empty(L.psfm_gn_ws_floats(N, HW, C, G), device=dev, dtype=torch.float32)
        bf = int(bias is not None and bias.dtype == torch.bfloat16)
        _hip.check(L.psfm_gn_act_bwd(_hip.ptr(dy), _hip.ptr(x), _hip.ptr(res), _hip.ptr(bias), bf, _hip.ptr(weight),
                                     _hip.ptr(beta), _hip.ptr(mean), _hip.ptr(invstd), N, HW, C, G, int(ctx.act),
                                     _hip.ptr(dx), _hip.ptr(dres), _hip.ptr(dbias), _hip.ptr(dw), _hip.ptr(db),
                                     _hip.ptr(ws), _hip.stream(dev)), "psfm_gn_act_bwd")
        return dx, dres, dbias, dw.to(weight.dtype), db.to(weight.dtype), None, None, None


ACT_ELU = 3  # PSFM_ACT_ELU (GroupNorm only)
# limits of psfm_gn_act_* (psfm_netops.hip gn_setup): the parameter-gradient pass gives each sample
# 64 / N lanes (N <= 64), the group totals of a sample fit one workgroup (G <= 128), C <= 512
GN_MAX_N, GN_MAX_G, GN_MAX_C = 64, 128, 512


def gn_shape_ok(shape, num_groups):
    """The GroupNorm shapes the HIP kernels take; anything else runs the torch chain."""
    N, C = shape[0], shape[1]
    return (len(shape) == 4 and C % num_groups == 0 and N <= GN_MAX_N and num_groups <= GN_MAX_G
            and C <= GN_MAX_C and (C % 8 == 0 or C <= 256))


def gn_act(x, bias, gn, relu=True, act=None, residual=None):
    """act(groupnorm(x [+ residual] + bias)) with the reference's nn.GroupNorm module `gn`; act is
    ReLU (relu=True, PoseNet) / none, or `act=ACT_ELU` (PackNet Conv2D / ResidualConv).  `bias`
    may be None."""
    act = (ACT_RELU if relu else ACT_NONE) if act is None else act
    if (_fusable(x, "gn") and gn.affine and gn_shape_ok(tuple(x.shape), gn.num_groups)
            and (residual is None or (residual.shape == x.shape and residual.device == x.device))):
        return _GNAct.apply(x, residual, bias, gn.weight, gn.bias, int(gn.num_groups), float(gn.eps), act)
    if residual is not None:
        x = x + residual
    if bias is not None:
        x = x + bias.to(x.dtype).view(1, -1, 1, 1)
    y = gn(x)
    if act == ACT_RELU:
        return torch.relu(y)
    if act == ACT_ELU:
        return F.elu(y)
    return y


# ----------------------------------------------------------------------------------------------
UPCAT = True  # decoder up-stage input on HIP


class _UpCat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, skip):
        _hip.note_forward(ctx)
        N, C1, h, w = x.shape
        C2 = skip.shape[1] if skip is not None else 0
        out = torch.empty((N, C1 + C2, 2 * h, 2 * w), device=x.device, dtype=x.dtype,
                          memory_format=torch.channels_last)
        _hip.check(_hip.lib().psfm_upcat_fwd(_hip.ptr(x), _hip.ptr(skip), N, h, w, C1, C2, _hip.ptr(out),
                                             _hip.stream(x.device)), "psfm_upcat_fwd")
        ctx.dims, ctx.has_skip = (N, C1, C2, h, w), skip is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        _hip.capture_guard(ctx)
        N, C1, C2, h, w = ctx.dims
        dout = _rows(dout)
        dx = torch.empty((N, C1, h, w), device=dout.device, dtype=dout.dtype, memory_format=torch.channels_last)
        dskip = torch.empty((N, C2, 2 * h, 2 * w), device=dout.device, dtype=dout.dtype,
                            memory_format=torch.channels_last) if ctx.has_skip else None
        _hip.check(_hip.lib().psfm_upcat_bwd(_hip.ptr(dout), N, h, w, C1, C2, _hip.ptr(dx), _hip.ptr(dskip),
                                             _hip.stream(dout.device)), "psfm_upcat_bwd")
        return dx, dskip


def _nhwc_bf16(t):
    return t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)


def up_cat(x, skip=None):
    """torch.cat([F.interpolate(x, scale_factor=2, mode='nearest'), skip], 1) — the DepthDecoder
    up-stage input (depth_decoder.py:48-57) — as ONE HIP kernel each way on bf16 channels_last
    activations (include/psfm_netops.h psfm_upcat_*).  Other layouts / dtypes / devices run the
    reference's op chain (upsample with the deterministic block-sum backward, then cat)."""
    from ...utils.image import upsample_nearest
    if (UPCAT and _nhwc_bf16(x) and x.shape[1] % 8 == 0 and
            (skip is None or (_nhwc_bf16(skip) and skip.shape[1] % 8 == 0 and skip.device == x.device
                              and tuple(skip.shape[-2:]) == (2 * x.shape[2], 2 * x.shape[3])
                              and skip.shape[0] == x.shape[0]))):
        return _UpCat.apply(x, skip)
    up = upsample_nearest(x, 2)
    return up if skip is None else torch.cat([up, skip.to(up.dtype)], 1)


class _UpCatBiasReLU(torch.autograd.Function):
    """cat([nearest_up2(relu(x + bias)), skip]): the up-stage's first ConvBlock epilogue folded into
    the up-stage input (include/psfm_netops.h psfm_upcat_bias_relu_*).  The ReLU mask of the
    backward is read from the output itself (its x part holds relu(x + bias) upsampled)."""

    @staticmethod
    def forward(ctx, x, bias, skip):
        _hip.note_forward(ctx)
        N, C1, h, w = x.shape
        C2 = skip.shape[1] if skip is not None else 0
        out = torch.empty((N, C1 + C2, 2 * h, 2 * w), device=x.device, dtype=x.dtype,
                          memory_format=torch.channels_last)
        bf = int(bias.dtype == torch.bfloat16)
        _hip.check(_hip.lib().psfm_upcat_bias_relu_fwd(_hip.ptr(x), _hip.ptr(bias), bf, _hip.ptr(skip), N, h, w, C1,
                                                       C2, _hip.ptr(out), _hip.stream(x.device)),
                   "psfm_upcat_bias_relu_fwd")
        ctx.save_for_backward(out)
        ctx.dims, ctx.has_skip, ctx.bias_dtype = (N, C1, C2, h, w), skip is not None, bias.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        _hip.capture_guard(ctx)
        (out,) = ctx.saved_tensors
        N, C1, C2, h, w = ctx.dims
        dout = _rows(dout)
        L = _hip.lib()
        dx = torch.empty((N, C1, h, w), device=dout.device, dtype=dout.dtype, memory_format=torch.channels_last)
        dskip = torch.empty((N, C2, 2 * h, 2 * w), device=dout.device, dtype=dout.dtype,
                            memory_format=torch.channels_last) if ctx.has_skip else None
        db = torch.empty(C1, device=dout.device, dtype=ctx.bias_dtype)
        ws = torch.empty(max(L.psfm_upcat_ws_floats(N, h, w, C1), 1), device=dout.device, dtype=torch.float32)
        _hip.check(L.psfm_upcat_bias_relu_bwd(_hip.ptr(dout), _hip.ptr(out), N, h, w, C1, C2, _hip.ptr(dx),
                                              _hip.ptr(dskip), _hip.ptr(db), int(ctx.bias_dtype == torch.bfloat16),
                                              _hip.ptr(ws), _hip.stream(dout.device)), "psfm_upcat_bias_relu_bwd")
        return dx, db, dskip


def conv_block_up_cat(block, x, skip=None):
    """cat([upsample(ConvBlock(x)), skip]) — ConvBlock = Conv3x3 + ReLU (layers.py:25-41), the
    DepthDecoder's upconv_i0 followed by its up-stage input (depth_decoder.py:48-57).  On bf16
    channels_last activations: the convolution without its bias, then ONE HIP kernel each way for
    bias + ReLU + upsample + cat (psfm_upcat_bias_relu); otherwise the block and up_cat."""
    c = block.conv
    xin = c.pad(x) if c.pad is not None else x
    bias = c.conv.bias
    if FUSE["bias"] and UPCAT and bias is not None:
        y = conv_nobias(c.conv, xin)
        C1 = y.shape[1]
        if (_nhwc_bf16(y) and C1 % 8 == 0 and 256 % (C1 // 8) == 0 and
                (skip is None or (_nhwc_bf16(skip) and skip.shape[1] % 8 == 0 and skip.device == y.device
                                  and tuple(skip.shape[-2:]) == (2 * y.shape[2], 2 * y.shape[3])
                                  and skip.shape[0] == y.shape[0]))):
            return _UpCatBiasReLU.apply(y, bias, skip)
        return up_cat(bias_act(y, bias, ACT_RELU), skip)
    return up_cat(block(x), skip)

