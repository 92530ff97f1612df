"""Composed PackNet packing layer on HIP (include/psfm_packconv.h, csrc/psfm_packconv.hip) — the
Conv2D half of the SURVEY §8f row 1.

Reference: packnet_sfm/networks/layers/packnet/layers01.py:239-246 (PackLayerConv3d.forward):
    x = packing(x); x = conv3d(x.unsqueeze(1)); x = x.view(b, d*4C, H/2, W/2); x = self.conv(x)
with self.conv = Conv2D (:10-37) = ConstantPad2d(k//2) -> Conv2d(d*4C -> C, k) -> GroupNorm -> ELU.

Conv3d (3x3x3, 1 -> d, pad 1, bias b3) followed by the k x k Conv2d (weights W2) is one linear
(k+2) x (k+2) convolution over the 4C packed channels P:
    Weff[m, kp', a, b'] = sum_{o, dz, dy, dx} W2[m, o*4C + kp'+1-dz, a-dy, b'-dx] w3[o, dz, dy, dx]
(a 3-D transposed convolution of W2 by w3).  It differs from the reference only where the
reference zero-pads V = conv3d(P) + b3 (ConstantPad2d) and the composition would extend V past
the image: on the frame of output pixels within k//2 of the border.  There
    y = conv(P, Weff) + BT[row class, col class] - E_T - E_B - E_L - E_R + corner terms
where BT sums b3's contribution over the in-image taps, E_T (E_B, E_L, E_R) is a 1-D (k+2)-tap
convolution of P's first row (last row, first / last column) with the composition of the
out-of-image tap row (column) of W2 with w3's inward tap plane, and the corner terms remove what
E_L / E_R count twice with E_T / E_B.  Everything runs on HIP through the C-ABI: psfm_pc_compose
builds the composed tensors in kernel layouts from the module's parameters (each rounded to bf16 as
autocast's Conv3d / Conv2d casts do), psfm_pc_fwd / psfm_pc_bwd do the data-sized work and
psfm_pc_compose_bwd carries the composed weights' gradients back to W2, w3, b3 (fp32: the bf16
rounding passes gradients straight through, where autocast would round them to bf16).  Exactness of
the decomposition (fp64, every gradient, k = 3 / 5, d = 4 / 8) is tested on the CPU against the
reference chain (oracle/packconv_oracle.py, tests/test_packconv.py).
"""
import ctypes

import torch

from .... import _hip

ENABLED = True
c_int, c_int64, c_void_p = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p


class PcDesc(ctypes.Structure):
    """psfm_pc_desc (include/psfm_packconv.h)."""
    _fields_ = [("B", c_int), ("C", c_int), ("H", c_int), ("W", c_int), ("k", c_int), ("d", c_int),
                ("xs", c_int64 * 4), ("ys", c_int64 * 4)]


class PcWeights(ctypes.Structure):
    """psfm_pc_weights."""
    _fields_ = [("wf", c_void_p), ("wb", c_void_p), ("ef", c_void_p * 4), ("eb", c_void_p * 4),
                ("corner", c_void_p), ("bt", c_void_p)]


def _cl_strides(B, C, H, W):
    return [H * W * C, 1, W * C, C]


def supported(x, C, k, d):
    """The library takes this layer (asked through psfm_pc_ws_floats, which applies every limit of
    the kernels — including the corner kernels' LDS bound — and returns -1 outside them)."""
    B, _, H, W = x.shape
    if not (ENABLED and x.is_cuda and k in (3, 5) and d in (4, 8) and H % 2 == 0 and W % 2 == 0):
        return False
    t = PcDesc(B=B, C=C, H=H, W=W, k=k, d=d)
    t.xs[:] = _cl_strides(B, C, H, W)
    t.ys[:] = _cl_strides(B, C, H // 2, W // 2)
    return int(_hip.lib().psfm_pc_ws_floats(ctypes.byref(t))) >= 0


def _sizes(L, t):
    """(workspace floats, weight-buffer bytes) of a descriptor; a negative answer is the library
    refusing the shape, an error here (supported() said yes)."""
    ws, wb = int(L.psfm_pc_ws_floats(ctypes.byref(t))), int(L.psfm_pc_wbuf_bytes(ctypes.byref(t)))
    if ws < 0 or wb < 0:
        raise RuntimeError("psfm_pc: shape refused: " + L.psfm_pc_last_error().decode(errors="replace"))
    return ws, wb


def beneficial(x, C):
    """The composed layer pays for its weight composition (~C^2 work, independent of the image)
    out of the per-pixel savings: measured on every PackNet01 / PackNetSAN01 / DDAD pack layer
    (profiles/r05/packconv/), it wins wherever B (H/2) (W/2) >= 2 C^2 (all C <= 64 layers: PackNet01
    pack1 8.9 -> 2.2 ms fwd+bwd, pack2 1.20 -> 0.67; PackNetSAN01 pack1 2.26 -> 1.13) and loses
    below (C >= 128: the composer dominates)."""
    B, _, H, W = x.shape
    return B * (H // 2) * (W // 2) >= 2 * C * C


def _desc(x, y, k, d):
    B, C, H, W = x.shape
    t = PcDesc(B=B, C=C, H=H, W=W, k=k, d=d)
    t.xs[:] = list(x.stride())
    t.ys[:] = list(y.stride())
    return t


def _param32(p, shape):
    """The parameter as the contiguous fp32 tensor the composer reads (bf16 weights of the
    mixed-precision trainer are widened exactly)."""
    if p.dtype not in (torch.float32, torch.bfloat16) or tuple(p.shape) != tuple(shape) or not p.is_cuda:
        raise RuntimeError(f"packconv: parameter must be an fp32 / bf16 ROCm tensor of shape {tuple(shape)}, "
                           f"got {p.dtype} {tuple(p.shape)} on {p.device}")
    return p.detach().float().contiguous()


class PackConvFn(torch.autograd.Function):
    """y = the Conv2d output (no Conv2d bias) of PackLayerConv3d on bf16 channels_last x, from the
    module's fp32 parameters W2 (Conv2D.conv_base.weight), w3, b3 (conv3d); backward returns dx,
    dW2, dw3, db3."""

    @staticmethod
    def forward(ctx, x, W2, w3, b3, k):
        _hip.note_forward(ctx)
        B, C, H, W = x.shape
        d = w3.shape[0]
        ctx.dtypes = (W2.dtype, w3.dtype, b3.dtype if b3 is not None else None)
        W2 = _param32(W2, (C, 4 * C * d, k, k))
        w3 = _param32(w3, (d, 1, 3, 3, 3))
        b3 = _param32(b3, (d,)) if b3 is not None else None
        y = torch.empty((B, C, H // 2, W // 2), device=x.device, dtype=torch.bfloat16,
                        memory_format=torch.channels_last)
        t = _desc(x, y, k, d)
        L = _hip.lib()
        nws, nwb = _sizes(L, t)
        wbuf = torch.empty(nwb, device=x.device, dtype=torch.uint8)
        ws = torch.empty(max(nws, 1), device=x.device, dtype=torch.float32)
        st = _hip.stream(x.device)
        _hip.check(L.psfm_pc_compose(ctypes.byref(t), _hip.ptr(W2), _hip.ptr(w3), _hip.ptr(b3), _hip.ptr(wbuf), st),
                   "psfm_pc_compose")
        w = PcWeights()
        _hip.check(L.psfm_pc_weights_of(ctypes.byref(t), _hip.ptr(wbuf), ctypes.byref(w)), "psfm_pc_weights_of")
        _hip.check(L.psfm_pc_fwd(ctypes.byref(t), ctypes.byref(w), _hip.ptr(x), _hip.ptr(y), _hip.ptr(ws), st),
                   "psfm_pc_fwd")
        ctx.save_for_backward(x, W2, w3, b3, wbuf)
        ctx.k = k
        return y

    @staticmethod
    def backward(ctx, gy):
        _hip.capture_guard(ctx)
        x, W2, w3, b3, wbuf = ctx.saved_tensors
        k = ctx.k
        B, C, H, W = x.shape
        d = w3.shape[0]
        ke, pk = k + 2, k // 2
        gy = gy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dev = x.device
        f32 = dict(device=dev, dtype=torch.float32)
        need_x, need_w = ctx.needs_input_grad[0], any(ctx.needs_input_grad[1:4])
        t = _desc(x, gy, k, d)
        L = _hip.lib()
        st = _hip.stream(dev)
        w = PcWeights()
        _hip.check(L.psfm_pc_weights_of(ctypes.byref(t), _hip.ptr(wbuf), ctypes.byref(w)), "psfm_pc_weights_of")
        ws = torch.empty(max(_sizes(L, t)[0], 1), **f32)
        dx = torch.empty_like(x, memory_format=torch.channels_last) if need_x else None
        dwm = de = dc = dbt = None
        if need_w:
            dwm = torch.empty(C, ke, ke, 4 * C, **f32)
            de = torch.empty(4, pk, C, ke, 4 * C, **f32)
            dc = torch.empty(4, pk, pk, C, 4 * C, **f32)
            dbt = torch.empty(2 * pk + 1, 2 * pk + 1, C, **f32)
        _hip.check(L.psfm_pc_bwd(ctypes.byref(t), ctypes.byref(w), _hip.ptr(x), _hip.ptr(gy), _hip.ptr(dx),
                                 _hip.ptr(dwm), _hip.ptr(de), _hip.ptr(dc), _hip.ptr(dbt), _hip.ptr(ws), st),
                   "psfm_pc_bwd")
        gW2 = gw3 = gb3 = None
        if need_w:
            gW2, gw3 = torch.empty_like(W2), torch.empty_like(w3)
            gb3 = torch.empty_like(b3) if b3 is not None else None
            _hip.check(L.psfm_pc_compose_bwd(ctypes.byref(t), _hip.ptr(W2), _hip.ptr(w3), _hip.ptr(b3), _hip.ptr(dwm),
                                             _hip.ptr(de), _hip.ptr(dc), _hip.ptr(dbt), _hip.ptr(gW2), _hip.ptr(gw3),
                                             _hip.ptr(gb3), _hip.ptr(ws), st), "psfm_pc_compose_bwd")
            dt = ctx.dtypes
            gW2, gw3 = gW2.to(dt[0]), gw3.to(dt[1])
            gb3 = gb3.to(dt[2]) if gb3 is not None else None
        return dx, gW2, gw3, gb3, None


def pack_conv2d(x, conv3d, conv2d, k):
    """The Conv2d output (without its bias) of PackLayerConv3d, conv2d(pad(view(conv3d(pack(x))))),
    on HIP in bf16 (the autocast dtype of the reference's convolutions)."""
    with torch.autocast("cuda", enabled=False):
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        return PackConvFn.apply(xb, conv2d.weight, conv3d.weight, conv3d.bias, k)
