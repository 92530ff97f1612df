"""Composed PackNet packing layer (include/psfm_packconv.h, networks/layers/packnet/packconv.py):
SURVEY §8f row 1, the Conv2D half.

Reference chain (the oracle, evaluated with torch ops on the reference's own algorithm):
packnet_sfm/networks/layers/packnet/layers01.py:239-246 — packing -> Conv3d(1 -> d, 3x3x3, pad 1)
-> view(b, d*4C, H/2, W/2) -> Conv2D's ConstantPad2d(k//2) + Conv2d (:34-39).

CPU (no GPU needed):
  * the decomposition behind the kernels — main composed (k+2)^2 convolution + bias table - edge
    lines + corner terms, built from `packconv.compose` — equals the chain in float64 for y and for
    every gradient (x, W2, w3, b3), k = 3 / 5, d = 4 / 8, non-square and minimum-size images;
  * the kernel layouts decode back to the composed tensors, and a float64 emulation of the
    kernels' forward (main convolution from the decoded `wf`, edge convolutions from the decoded
    `ef`, the epilogue's class / frame logic) equals the chain.
GPU (-m gpu): the HIP path through the C-ABI against the chain on the same bf16-rounded inputs
(float64 CPU at small shapes, float32 GPU at the benchmarked first-layer shapes), bitwise
determinism, HIP-graph capture, and PackLayerConv3d's composed path vs its round-4 path."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from oracle import packconv_oracle as O
from oracle.packconv_oracle import chain, composed_forward

SHAPES = [(2, 4, 16, 20, 8, 5), (2, 8, 12, 16, 4, 3), (1, 4, 10, 14, 8, 3), (1, 2, 10, 10, 4, 5),
          (2, 3, 14, 22, 4, 5), (1, 2, 6, 6, 8, 3)]


def rand_case(B, C, H, W, d, k, dtype=torch.float64, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, C, H, W, generator=g, dtype=dtype)
    W2 = torch.randn(C, 4 * C * d, k, k, generator=g, dtype=dtype)
    w3 = torch.randn(d, 1, 3, 3, 3, generator=g, dtype=dtype)
    b3 = torch.randn(d, generator=g, dtype=dtype)
    return x, W2, w3, b3


@pytest.mark.parametrize("shape", SHAPES)
def test_decomposition_is_exact_in_float64(shape):
    *_, k = shape
    x, W2, w3, b3 = (t.requires_grad_(True) for t in rand_case(*shape))
    yr = chain(x, W2, w3, b3, k)
    yd = composed_forward(x, W2, w3, b3, k)
    assert ((yd - yr).abs().max() / yr.abs().max()).item() < 1e-12
    gy = torch.randn_like(yr)
    gr = torch.autograd.grad(yr, (x, W2, w3, b3), gy)
    gd = torch.autograd.grad(yd, (x, W2, w3, b3), gy)
    for a, b, n in zip(gd, gr, ("x", "W2", "w3", "b3")):
        assert ((a - b).abs().max() / b.abs().max()).item() < 1e-12, n


def _decode_wf(wf, C, ke):
    return wf.permute(0, 5, 1, 4, 6, 2, 3).reshape(-1, 4 * C, ke, ke)[:C]


def _decode_wb(wb, C, ke):
    # [nb][q][a][b][kq][n][e8] -> [m = (q, kq, e8)][kin = (nb, n)][a][b], taps flipped back
    return wb.permute(1, 4, 6, 0, 5, 2, 3).reshape(C, 4 * C, ke, ke).flip(2, 3)


def _decode_ef(ef, C, pk, ke):
    return ef.permute(0, 4, 1, 3, 5, 2).reshape(-1, 4 * C, ke)[:pk * C]


def _decode_eb(eb, C, pk, ke):
    return eb.permute(1, 3, 5, 0, 4, 2).reshape(pk * C, 4 * C, ke).flip(2)


@pytest.mark.parametrize("C,d,k", [(32, 8, 5), (64, 4, 3), (96, 8, 3)])
def test_kernel_layouts_decode_to_the_composed_weights(C, d, k):
    x, W2, w3, b3 = rand_case(1, C, 12, 12, d, k, dtype=torch.float32)
    Weff, U, Cn, bt = O.compose(W2, w3, b3, k)
    wf, wb, ef, eb, corner, btf = O.kernel_layouts(Weff, U, Cn, bt, C, k)
    pk, ke = k // 2, k + 2
    Wk = O.kin_order(Weff, C, 1).to(torch.bfloat16)
    assert torch.equal(_decode_wf(wf, C, ke), Wk)
    assert torch.equal(_decode_wb(wb, C, ke), Wk)
    Uk = O.kin_order(U, C, 3).reshape(4, pk * C, 4 * C, ke).to(torch.bfloat16)
    for e in range(4):
        assert torch.equal(_decode_ef(ef[e], C, pk, ke), Uk[e])
        assert torch.equal(_decode_eb(eb[e], C, pk, ke), Uk[e])
    assert torch.equal(O.ref_order(corner, C, 4), Cn)
    assert torch.equal(O.ref_order(O.kin_order(Weff, C, 1), C, 1), Weff)
    assert wf.shape == ((C + 63) // 64, 4 * C // 32, ke, ke, 4, 64, 8)
    assert wb.shape == (4 * C // 64, C // 32, ke, ke, 4, 64, 8)
    assert ef[0].shape == ((pk * C + 63) // 64, 4 * C // 32, ke, 4, 64, 8)
    assert eb[0].shape == (4 * C // 64, pk * C // 32, ke, 4, 64, 8)


def emulate_kernels_fwd(x, wf, ef, corner, bt, C, k):
    """float64 emulation of psfm_pc_fwd from the kernel layouts: edge convolutions -> corner
    terms into E_L / E_R -> main convolution + epilogue (bias class table, frame edge terms)."""
    pk, pe, ke = k // 2, k // 2 + 1, k + 2
    B, _, H, W = x.shape
    Ho, Wo = H // 2, W // 2
    Pk = x.reshape(B, C, Ho, 2, Wo, 2).permute(0, 3, 5, 1, 2, 4).reshape(B, 4 * C, Ho, Wo)   # kin = s C + c
    Wk = _decode_wf(wf, C, ke).double()
    lines = [Pk[:, :, 0, :], Pk[:, :, Ho - 1, :], Pk[:, :, :, 0], Pk[:, :, :, Wo - 1]]
    E = [F.conv1d(l_, _decode_ef(ef[e], C, pk, ke).double(), padding=pe).permute(0, 2, 1) for e, l_ in enumerate(lines)]
    corner = corner.double()
    pc = [Pk[:, :, 0, 0], Pk[:, :, Ho - 1, 0], Pk[:, :, 0, Wo - 1], Pk[:, :, Ho - 1, Wo - 1]]
    for cn in range(4):   # k_pc_corner_fwd
        top, left = cn % 2 == 0, cn < 2
        for i in range(pk):
            for j in range(pk):
                Y = pk - 1 - i if top else Ho - 1 - i
                v = pc[cn] @ corner[cn, i, j].T                                     # [B, C]
                E[2 if left else 3][:, Y, j * C:(j + 1) * C] -= v
    y = F.conv2d(Pk, Wk, padding=pe)
    rc = lambda yy, n: yy if yy < pk else (2 * pk - (n - 1 - yy) if yy >= n - pk else pk)
    bt = bt.double()
    for Y in range(Ho):
        for X in range(Wo):
            v = y[:, :, Y, X] + bt[rc(Y, Ho), rc(X, Wo)]
            if Y < pk:
                v = v - E[0][:, X, (pk - 1 - Y) * C:(pk - Y) * C]
            if Y >= Ho - pk:
                v = v - E[1][:, X, (Ho - 1 - Y) * C:(Ho - Y) * C]
            if X < pk:
                v = v - E[2][:, Y, (pk - 1 - X) * C:(pk - X) * C]
            if X >= Wo - pk:
                v = v - E[3][:, Y, (Wo - 1 - X) * C:(Wo - X) * C]
            y[:, :, Y, X] = v
    return y


@pytest.mark.parametrize("shape", [(2, 32, 12, 16, 4, 5), (1, 64, 10, 14, 8, 3)])
def test_emulated_kernel_forward_matches_the_chain(shape):
    B, C, H, W, d, k = shape
    x, W2, w3, b3 = rand_case(*shape, dtype=torch.float64)
    Weff, U, Cn, bt = O.compose(W2, w3, b3, k)
    # the emulation reads bf16-rounded weights (as the kernels do): compare with the chain on the
    # exact weights within the bf16 rounding of the composed weights
    wf, wb, ef, eb, corner, btf = O.kernel_layouts(Weff, U, Cn, bt, C, k)
    y = emulate_kernels_fwd(x, wf, ef, corner, btf, C, k)
    yr = chain(x, W2, w3, b3, k)
    err = ((y - yr).norm() / yr.norm()).item()
    assert err < 5e-3, err
    # and exactly, with fp64 layouts (no bf16 rounding): the layout / epilogue logic itself
    Wk64 = O.kin_order(Weff, C, 1)
    wf64 = O.pad_rows(Wk64, O.cop(C)).reshape(O.cop(C) // 64, 64, C // 8, 4, 8, k + 2, k + 2)
    wf64 = wf64.permute(0, 2, 5, 6, 3, 1, 4)
    pk = k // 2
    Uk = O.kin_order(U, C, 3).reshape(4, pk * C, 4 * C, k + 2)
    ef64 = [O.pad_rows(Uk[e], O.cop(pk * C)).reshape(-1, 64, C // 8, 4, 8, k + 2)
            .permute(0, 2, 5, 3, 1, 4) for e in range(4)]
    y64 = emulate_kernels_fwd(x, wf64, ef64, O.kin_order(Cn, C, 4), bt, C, k)
    assert ((y64 - yr).abs().max() / yr.abs().max()).item() < 1e-12


# ------------------------------------------------------------------------------------------- GPU
def _params(B, C, H, W, d, k, seed=0, bias_scale=0.3):
    g = torch.Generator().manual_seed(seed)
    bf = torch.bfloat16
    x = torch.randn(B, C, H, W, generator=g).to(bf)
    W2 = torch.randn(C, 4 * C * d, k, k, generator=g) / (4 * C * d * k * k) ** 0.5
    w3 = torch.randn(d, 1, 3, 3, 3, generator=g) / 27 ** 0.5
    b3 = bias_scale * torch.randn(d, generator=g)
    gy = torch.randn(B, C, H // 2, W // 2, generator=g).to(bf)
    return x, W2, w3, b3, gy


def _hip_run(x, W2, w3, b3, gy, k):
    from packnet_sfm_amd.networks.layers.packnet import packconv
    cl = torch.channels_last
    xd = x.cuda().contiguous(memory_format=cl).requires_grad_(True)
    Ws = [t.cuda().requires_grad_(True) for t in (W2, w3, b3)]
    y = packconv.PackConvFn.apply(xd, *Ws, k)
    y.backward(gy.cuda().contiguous(memory_format=cl))
    torch.cuda.synchronize()
    return y.detach(), xd.grad, *(t.grad for t in Ws)


def _gpu_case(B, C, H, W, d, k, ref_dev, seed=0):
    """HIP vs the reference chain on the same bf16-rounded operands (the HIP path rounds W2, w3, b3
    to bf16 as autocast does; its weight gradients are those of the rounded weights, in fp32)."""
    x, W2, w3, b3, gy = _params(B, C, H, W, d, k, seed)
    out = _hip_run(x, W2, w3, b3, gy, k)
    dt = torch.float64 if ref_dev == "cpu" else torch.float32
    bfr = lambda t: t.to(torch.bfloat16).to(ref_dev, dt).requires_grad_(True)
    xr, W2r, w3r, b3r = bfr(x), bfr(W2), bfr(w3), bfr(b3)
    yr = chain(xr, W2r, w3r, b3r, k)
    yr.backward(gy.to(ref_dev, dt))
    ref = (yr.detach(), xr.grad, W2r.grad, w3r.grad, b3r.grad)
    return {n: (a.double().cpu(), b.double().cpu()) for n, a, b in zip(("y", "dx", "dW2", "dw3", "db3"), out, ref)}


def _check(res, tol_y=1.5e-2, tol_w=1e-4):
    """y / dx carry the bf16 rounding of the composed weights and of the bf16 output (the
    reference's own bf16 chain rounds V and y): relative L2 error <= 5e-3 and max error <= tol_y
    of max|ref|.  Weight gradients are fp32 end to end (gy and x are exact bf16 values): <= tol_w of
    max|ref| (a float32 reference at the big shapes contributes its own ~1e-6)."""
    out = {}
    for n, (a, b) in res.items():
        mx = ((a - b).abs().max() / b.abs().max()).item()
        l2 = ((a - b).norm() / b.norm()).item()
        out[n] = f"{mx:.1e}/{l2:.1e}"
        if n in ("y", "dx"):
            assert l2 < 5e-3 and mx < tol_y, (n, mx, l2)
        else:
            assert mx < tol_w, (n, mx, l2)
    return out


GPU_SMALL = [(2, 32, 16, 24, 4, 3), (2, 64, 20, 28, 8, 5), (1, 32, 14, 18, 8, 5), (2, 64, 12, 16, 4, 3),
             (1, 96, 16, 144, 8, 3), (3, 128, 10, 12, 8, 3), (1, 32, 10, 10, 4, 5), (2, 64, 6, 6, 8, 3)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", GPU_SMALL)
def test_hip_matches_the_float64_chain(shape):
    print(shape, _check(_gpu_case(*shape, ref_dev="cpu")))


def _windows(B, Ho, Wo, pk):
    """(b, y0, y1, x0, x1) output windows: the four corners, a top-edge and a left-edge window and
    an interior one, in different images (every frame class and the batch indexing)."""
    h, w = 2 * pk + 2, 3 * pk + 4
    ws = [(0, 0, h, 0, w), (1 % B, Ho - h, Ho, Wo - w, Wo), (2 % B, 0, h, Wo - w, Wo), (3 % B, Ho - h, Ho, 0, w),
          (4 % B, 0, h, Wo // 2, Wo // 2 + w), (5 % B, Ho // 2, Ho // 2 + h, 0, w),
          (0, Ho // 2, Ho // 2 + h, Wo // 2, Wo // 2 + w)]
    return ws


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(6, 64, 192, 640, 8, 5), (4, 32, 384, 640, 4, 5), (6, 64, 96, 320, 8, 3),
                                   (6, 128, 48, 160, 8, 3)])
def test_hip_matches_the_float64_chain_at_packnet_layer_shapes(shape):
    """Full-size layers, exact float64 reference without a full-size float64 convolution: dy is
    nonzero only on small output windows (corners, edges, interior), so dx, dW2, dw3 and db3 are
    sums over those windows, which the reference chain computes exactly on crops of x around each
    window (margin pe + 1 packed pixels: no output of a window sees a crop boundary that is not
    the image's).  y is compared on the same windows."""
    B, C, H, W, d, k = shape
    pk, pe = k // 2, k // 2 + 1
    Ho, Wo = H // 2, W // 2
    x, W2, w3, b3, _ = _params(B, C, H, W, d, k)
    g = torch.Generator().manual_seed(1)
    gy = torch.zeros(B, C, Ho, Wo, dtype=torch.bfloat16)
    wins = _windows(B, Ho, Wo, pk)
    for (b, y0, y1, x0, x1) in wins:
        gy[b, :, y0:y1, x0:x1] = torch.randn(C, y1 - y0, x1 - x0, generator=g).to(torch.bfloat16)
    y, dx, dW2, dw3, db3 = (t.double().cpu() for t in _hip_run(x, W2, w3, b3, gy, k))
    bfr = lambda t: t.to(torch.bfloat16).double().requires_grad_(True)
    W2r, w3r, b3r = bfr(W2), bfr(w3), bfr(b3)
    m = pe + 1
    dx_ref = torch.zeros_like(dx)
    covered = torch.zeros(B, 1, H, W, dtype=torch.bool)
    ys, yr_all = [], []
    for (b, y0, y1, x0, x1) in wins:
        cy0, cy1, cx0, cx1 = max(0, y0 - m), min(Ho, y1 + m), max(0, x0 - m), min(Wo, x1 + m)
        xc = x[b:b + 1, :, 2 * cy0:2 * cy1, 2 * cx0:2 * cx1].double().requires_grad_(True)
        yc = chain(xc, W2r, w3r, b3r, k)
        gyc = gy[b:b + 1, :, cy0:cy1, cx0:cx1].double()
        yc.backward(gyc)
        dx_ref[b, :, 2 * cy0:2 * cy1, 2 * cx0:2 * cx1] += xc.grad[0]
        covered[b, :, 2 * cy0:2 * cy1, 2 * cx0:2 * cx1] = True
        ys.append(y[b, :, y0:y1, x0:x1])
        yr_all.append(yc.detach()[0, :, y0 - cy0:y1 - cy0, x0 - cx0:x1 - cx0])
    assert not dx[~covered.expand_as(dx)].any()
    res = {"y": (torch.stack(ys), torch.stack(yr_all)), "dx": (dx, dx_ref), "dW2": (dW2, W2r.grad),
           "dw3": (dw3, w3r.grad), "db3": (db3, b3r.grad)}
    print(shape, _check(res))


@pytest.mark.gpu
@pytest.mark.parametrize("C,d,k", [(32, 4, 5), (64, 8, 3), (96, 8, 5)])
def test_hip_composer_writes_the_oracle_layouts(C, d, k):
    """psfm_pc_compose == oracle.kernel_layouts(oracle.compose(bf16-rounded params)) up to the fp32
    summation order: bf16 weights within one bf16 ulp, fp32 tables within 1e-5."""
    from packnet_sfm_amd import _hip
    from packnet_sfm_amd.networks.layers.packnet import packconv
    _, W2, w3, b3, _ = _params(1, C, 12, 12, d, k)
    bfr = lambda t: t.to(torch.bfloat16).float()
    ref = O.kernel_layouts(*O.compose(bfr(W2), bfr(w3), bfr(b3), k), C, k)
    x = torch.empty(1, C, 12, 12, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t = packconv._desc(x, torch.empty(1, C, 6, 6, device="cuda").contiguous(memory_format=torch.channels_last), k, d)
    L = _hip.lib()
    wbuf = torch.zeros(int(L.psfm_pc_wbuf_bytes(ctypes.byref(t))), device="cuda", dtype=torch.uint8)
    Wd, w3d, b3d = (v.cuda() for v in (W2, w3, b3))
    _hip.check(L.psfm_pc_compose(ctypes.byref(t), _hip.ptr(Wd), _hip.ptr(w3d), _hip.ptr(b3d), _hip.ptr(wbuf),
                                 _hip.stream(x.device)), "psfm_pc_compose")
    w = packconv.PcWeights()
    _hip.check(L.psfm_pc_weights_of(ctypes.byref(t), _hip.ptr(wbuf), ctypes.byref(w)), "psfm_pc_weights_of")
    torch.cuda.synchronize()
    base = wbuf.data_ptr()

    def view(ptr, like):
        off = ptr - base
        n = like.numel() * like.element_size()
        return wbuf[off:off + n].view(like.dtype).view(like.shape).cpu()

    wf, wb, ef, eb, corner, bt = ref
    for got, want in [(view(w.wf, wf), wf), (view(w.wb, wb), wb)] + \
            [(view(w.ef[e], ef[e]), ef[e]) for e in range(4)] + [(view(w.eb[e], eb[e]), eb[e]) for e in range(4)]:
        g, r = got.float(), want.float()
        # one bf16 rounding apart (the fp32 sums run in another order), plus fp32 noise near zero
        assert ((g - r).abs() <= r.abs() * 2 ** -7 + 1e-5 * r.abs().max()).all()
    for got, want in [(view(w.corner, corner), corner), (view(w.bt, bt), bt)]:
        assert ((got - want).abs().max() / want.abs().max()).item() < 1e-5


@pytest.mark.gpu
def test_hip_path_is_bitwise_deterministic_and_graph_capturable():
    from packnet_sfm_amd.networks.layers.packnet import packconv
    x, W2, w3, b3, gy = _params(2, 64, 64, 96, 8, 5)
    a = _hip_run(x, W2, w3, b3, gy, 5)
    b = _hip_run(x, W2, w3, b3, gy, 5)
    for u, v in zip(a, b):
        assert torch.equal(u, v)
    # capture forward + backward into a HIP graph on a side stream and replay it
    cl = torch.channels_last
    xd = x.cuda().contiguous(memory_format=cl).requires_grad_(True)
    Ws = [t.cuda().requires_grad_(True) for t in (W2, w3, b3)]
    gyd = gy.cuda().contiguous(memory_format=cl)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):   # warm-up on the capture stream
            for t in [xd] + Ws:
                t.grad = None
            packconv.PackConvFn.apply(xd, *Ws, 5).backward(gyd)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    for t in [xd] + Ws:
        t.grad = None
    with torch.cuda.graph(g):
        y = packconv.PackConvFn.apply(xd, *Ws, 5)
        y.backward(gyd)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, a[0].cuda())
    for t, r in zip([xd] + Ws, a[1:]):
        assert torch.equal(t.grad, r.cuda())


def _spy_pack_conv(monkeypatch, packconv):
    """Count PackConvFn.apply calls (the composed layer's only entry) while the test runs."""
    calls = []
    orig = packconv.PackConvFn.apply

    def spy(*a):
        calls.append(tuple(a[0].shape))
        return orig(*a)
    monkeypatch.setattr(packconv.PackConvFn, "apply", staticmethod(spy))
    return calls


@pytest.mark.gpu
@pytest.mark.parametrize("C,d,k,B,H,W,force", [(64, 8, 5, 2, 192, 320, False), (32, 4, 5, 2, 64, 96, False),
                                               (128, 8, 3, 6, 96, 320, True)])
def test_pack_layer_composed_path_matches_the_round4_path(monkeypatch, C, d, k, B, H, W, force):
    """PackLayerConv3d under bf16 autocast: the composed HIP path (asserted to run: PackConvFn.apply
    is called exactly once per forward) vs the pack3d + MIOpen Conv2d path with composition off
    (both bf16, the Conv2d bias, GroupNorm + ELU after): outputs and every gradient within the bf16
    noise of the two paths.  Every case satisfies B (H/2) (W/2) >= 2 C^2 (packconv.beneficial);
    `force` bypasses beneficial() where the round-5 policy keeps a C = 128 layer on the old path."""
    from packnet_sfm_amd.networks.layers.packnet import packconv
    from packnet_sfm_amd.networks.layers.packnet.layers01 import PackLayerConv3d
    assert B * (H // 2) * (W // 2) >= 2 * C * C
    if force:
        monkeypatch.setattr(packconv, "beneficial", lambda x, C: True)
    calls = _spy_pack_conv(monkeypatch, packconv)
    torch.manual_seed(0)
    m = PackLayerConv3d(C, k, d=d).cuda()
    with torch.no_grad():
        m.conv3d.bias.normal_(0, 0.3)
        m.conv.conv_base.bias.normal_(0, 0.1)
    x = torch.randn(B, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    gy = torch.randn(B, C, H // 2, W // 2, device="cuda")
    outs = []
    for enabled in (True, False):
        packconv.ENABLED = enabled
        try:
            xd = x.clone().requires_grad_(True)
            m.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                assert m._composed(xd) == enabled
                y = m(xd)
            y.float().backward(gy)
            outs.append([y.detach().float(), xd.grad.float()] + [p.grad.float().clone() for p in m.parameters()])
        finally:
            packconv.ENABLED = True
        assert len(calls) == (1 if enabled else 0), calls
        calls.clear()
    errs = [((a - b).norm() / b.norm()).item() for a, b in zip(*outs)]
    print("composed vs round-4 path, rel L2 (y, dx, dparams):", ["%.2e" % e for e in errs])
    assert max(errs) < 2e-2, errs


@pytest.mark.gpu
def test_packnet01_network_with_composed_pack_layers_matches_the_fp32_chain(monkeypatch):
    """a whole PackNet01 depth net whose pack1 and pack2 take the composed path
    (asserted: two PackConvFn calls per forward) under bf16 autocast, against the SAME weights in
    fp32 with composition off (MIOpen fp32 + the fp32 pack3d kernels: the chain
    test_packnet_layer_gradients_match_reference_gpu_fp32 pins to the reference).  B = 2 at the step
    goldens' 64 x 192 (the MIOpen kernels the network tests already built; the product policy
    packconv.beneficial composes the C = 64 layers from B (H/2)(W/2) >= 8192 on — B = 2, 192 x 640 and
    up — and is bypassed here for them, as the module test does).  A fixed linear loss on the four
    inverse-depth maps; compared: the maps, dL/drgb and the pack1 / pack2 parameter gradients.  The
    composed network must be as close to fp32 as the round-4 bf16 network (composition off) is: its
    relative L2 error at most 1.25x the round-4 path's + 2e-3, and the maps within 2e-2.  The two
    Conv3d bias gradients (8 entries, sums that cancel) move from run to run with MIOpen's
    atomic-accumulating bf16 backward: the round-4 path's own error on pack2.b3 measured 3.0e-2 -
    5.4e-2 over four runs on the same weights (the composed path 3.5e-2 - 4.0e-2), so for them the
    bound is that ratio or 6e-2, whichever is larger."""
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.networks.layers.packnet import packconv
    torch.backends.cudnn.benchmark = False
    monkeypatch.setattr(packconv, "beneficial", lambda x, C: C <= 64)
    calls = _spy_pack_conv(monkeypatch, packconv)
    import golden_util as gu
    from test_networks import _packnet_model
    dev = torch.device("cuda:0")
    depth, _ = _packnet_model()
    depth = depth.to(dev).train()
    g = torch.Generator().manual_seed(11)
    B, H, W = 2, 64, 192
    rgb = gu.smooth_texture(g, B, 3, H, W).to(dev)
    gys = [torch.randn(B, 1, H >> i, W >> i, generator=g).to(dev) for i in range(4)]
    watched = [depth.pack1.conv.conv_base.weight, depth.pack1.conv3d.weight, depth.pack1.conv3d.bias,
               depth.pack2.conv.conv_base.weight, depth.pack2.conv3d.weight, depth.pack2.conv3d.bias]

    def run(bf16, enabled):
        packconv.ENABLED = enabled
        try:
            depth.zero_grad()
            x = rgb.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                inv = depth(x)["inv_depths"]
            loss = sum((i.float() * gy).sum() for i, gy in zip(inv, gys))
            loss.backward()
            torch.cuda.synchronize()
            return [i.detach().float() for i in inv] + [x.grad.float()] + [p.grad.float().clone() for p in watched]
        finally:
            packconv.ENABLED = True

    ref = run(False, False)
    print("fp32 chain done", flush=True)
    assert not calls
    comp = run(True, True)
    assert len(calls) == 2 and calls[0][1:] == (64, H, W) and calls[1][1:] == (64, H // 2, W // 2), calls
    calls.clear()
    old = run(True, False)
    assert not calls
    names = ["inv0", "inv1", "inv2", "inv3", "drgb", "pack1.W2", "pack1.w3", "pack1.b3", "pack2.W2", "pack2.w3",
             "pack2.b3"]
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    rows = [(n, rel(c, r), rel(o, r)) for n, c, o, r in zip(names, comp, old, ref)]
    print("rel L2 vs fp32 (composed, round-4 bf16):", ["%s %.2e %.2e" % t for t in rows])
    for n, ec, eo in rows:
        assert ec <= max(1.25 * eo + 2e-3, 6e-2 if n.endswith("b3") else 0.0), (n, ec, eo)
        if n.startswith("inv"):
            assert ec < 2e-2, (n, ec)


def test_supported_asks_the_library_for_its_limits():
    """packconv.supported() applies every limit of the kernels (it asks psfm_pc_ws_floats),
    including the corner kernels' LDS bound (B pk^2 C + 4 B 64) * 4 <= 64 KB that the round-5 Python
    check missed (k = 5, B = 16, C = 256 and B = 8, C = 512 were accepted there, then refused)."""
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.networks.layers.packnet import packconv

    class X:   # stands in for a bf16 channels_last ROCm tensor (only .shape / .is_cuda are read)
        is_cuda = True

        def __init__(self, *shape):
            self.shape = shape
    assert not packconv.supported(X(16, 256, 64, 64), 256, 5, 8)
    assert not packconv.supported(X(8, 512, 64, 64), 512, 5, 8)
    assert packconv.supported(X(8, 512, 64, 64), 512, 3, 8)
    assert packconv.supported(X(6, 64, 192, 640), 64, 5, 8)
    assert not packconv.supported(X(6, 64, 191, 640), 64, 5, 8)
    assert not packconv.supported(X(2, 48, 64, 64), 48, 5, 8)      # C % 32
