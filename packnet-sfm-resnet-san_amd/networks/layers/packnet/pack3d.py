"""Fused PackNet pack / unpack 3-D convolution on HIP (include/psfm_pack3d.h,
csrc/psfm_pack3d.hip) — the SURVEY §8f "next" row 1.

  pack_conv3d(x, conv3d, r)    packing(x) -> unsqueeze -> Conv3d(1->d) -> view   (layers01.py:217-223)
  conv3d_unpack(x, conv3d, r)  unsqueeze -> Conv3d(1->d) -> view -> PixelShuffle (layers01.py:276-282)
d = 8 (PackNet01) or 4 (PackNetSAN01, num_3d_feat = 4).

One kernel per direction reads the (virtually packed) volume from x's own layout and writes the
folded / pixel-shuffled result once, channels_last, where ATen runs a permute copy, im2col,
GEMM, col2im and a second copy.  Under autocast the inputs and weights are rounded to the
autocast dtype exactly as nn.Conv3d's autocast does (fp32 accumulation, output in that dtype).
CPU tensors (and ENABLED = False) run the reference op chain itself (the nets are PyTorch)."""
import ctypes

import torch
import torch.nn.functional as F

from .... import _hip

ENABLED = True
PACK, UNPACK = 0, 1


class P3dDesc(ctypes.Structure):
    """psfm_p3d_desc (include/psfm_pack3d.h)."""
    _fields_ = [("mode", ctypes.c_int), ("dtype", ctypes.c_int), ("B", ctypes.c_int), ("C", ctypes.c_int),
                ("Hv", ctypes.c_int), ("Wv", ctypes.c_int), ("r", ctypes.c_int), ("d", ctypes.c_int),
                ("xs", ctypes.c_int64 * 4), ("ys", ctypes.c_int64 * 4)]


def _desc(mode, x, y, r, d):
    B, C, H, W = x.shape
    Hv, Wv = (H // r, W // r) if mode == PACK else (H, W)
    d = P3dDesc(mode=mode, dtype=1 if x.dtype == torch.bfloat16 else 0, B=B, C=C, Hv=Hv, Wv=Wv, r=r, d=d)
    d.xs[:] = list(x.stride())
    d.ys[:] = list(y.stride())
    return d


def _out_shape(mode, x, r, d):
    B, C, H, W = x.shape
    if mode == PACK:
        return (B, d * C * r * r, H // r, W // r)
    return (B, d * C // (r * r), H * r, W * r)


class Pack3dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, mode, r):
        _hip.note_forward(ctx)
        d = w.shape[0]
        y = torch.empty(_out_shape(mode, x, r, d), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        wf = w.detach().float().reshape(d, 27).contiguous()
        bf = b.detach().float().contiguous() if b is not None else None
        desc = _desc(mode, x, y, r, d)
        _hip.check(_hip.lib().psfm_p3d_fwd(ctypes.byref(desc), _hip.ptr(x), _hip.ptr(wf), _hip.ptr(bf), _hip.ptr(y),
                                           _hip.stream(x.device)), "psfm_p3d_fwd")
        ctx.save_for_backward(x, wf)
        ctx.mode, ctx.r, ctx.has_b, ctx.w_dtype = mode, r, b is not None, w.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        _hip.capture_guard(ctx)
        x, wf = ctx.saved_tensors
        gy = gy.contiguous(memory_format=torch.channels_last).to(x.dtype)
        d = wf.shape[0]
        desc = _desc(ctx.mode, x, gy, ctx.r, d)
        need_x, need_w, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        gx = torch.empty_strided(x.shape, x.stride(), device=x.device, dtype=x.dtype) if need_x else None
        gw = torch.empty(d, 27, device=x.device, dtype=torch.float32) if need_w else None
        gb = torch.empty(d, device=x.device, dtype=torch.float32) if (need_b and ctx.has_b) else None
        ws = None
        if gw is not None or gb is not None:
            n = _hip.lib().psfm_p3d_ws_floats(ctypes.byref(desc))
            ws = torch.empty(max(n, 1), device=x.device, dtype=torch.float32)
        _hip.check(_hip.lib().psfm_p3d_bwd(ctypes.byref(desc), _hip.ptr(x), _hip.ptr(wf), _hip.ptr(gy), _hip.ptr(gx),
                                           _hip.ptr(gw), _hip.ptr(gb), _hip.ptr(ws), _hip.stream(x.device)),
                   "psfm_p3d_bwd")
        gw = gw.reshape(d, 1, 3, 3, 3).to(ctx.w_dtype) if gw is not None else None
        gb = gb.to(ctx.w_dtype) if gb is not None else None
        return gx, gw, gb, None, None


def _fusable(x, conv3d):
    return (ENABLED and x.is_cuda and x.dim() == 4 and conv3d.out_channels in (4, 8) and conv3d.in_channels == 1
            and tuple(conv3d.kernel_size) == (3, 3, 3) and tuple(conv3d.padding) == (1, 1, 1)
            and tuple(conv3d.stride) == (1, 1, 1) and x.dtype in (torch.float32, torch.bfloat16))


def _autocast_args(x, conv3d):
    w, b = conv3d.weight, conv3d.bias
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        x = x.to(dt)
        w = w.to(dt)   # nn.Conv3d under autocast multiplies autocast-dtype weights (fp32 accumulate)
        b = b.to(dt) if b is not None else None
    elif x.dtype != w.dtype:
        x = x.to(w.dtype)
    return x, w, b


def pack_conv3d(x, conv3d, r, packing):
    """conv3d(packing(x).unsqueeze(1)) folded to [B, d C r^2, H/r, W/r] (d = 4 or 8 features)."""
    if not _fusable(x, conv3d):
        y = conv3d(packing(x).unsqueeze(1))
        b, c, d, h, w = y.shape
        return y.reshape(b, c * d, h, w)
    x, w, b = _autocast_args(x, conv3d)
    with torch.autocast("cuda", enabled=False):
        return Pack3dFn.apply(x, w, b, PACK, r)


def conv3d_unpack(x, conv3d, r, unpack):
    """PixelShuffle(r)(conv3d(x.unsqueeze(1)) folded) -> [B, d C / r^2, H r, W r]."""
    if not _fusable(x, conv3d):
        y = conv3d(x.unsqueeze(1))
        b, c, d, h, w = y.shape
        return unpack(y.reshape(b, c * d, h, w))
    x, w, b = _autocast_args(x, conv3d)
    with torch.autocast("cuda", enabled=False):
        return Pack3dFn.apply(x, w, b, UNPACK, r)
