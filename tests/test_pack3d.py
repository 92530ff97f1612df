"""GPU parity of the fused PackNet pack / unpack 3-D convolution (include/psfm_pack3d.h;
reference packnet_sfm/networks/layers/packnet/layers01.py:126-146, :189-282) against the
reference op chain (packing / Conv3d / view / PixelShuffle) evaluated in float64 on the CPU, for
the forward and all three gradients (input, weight, bias).

Tolerances: fp32 storage 1e-5 * max|ref| per element; bf16 storage (inputs rounded to bf16 for
both sides, fp32 accumulation) 1e-2 * max|ref| on the bf16 outputs and input gradient, 2e-3
relative on the fp32-accumulated weight / bias gradients."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import __graft_entry__
    __graft_entry__.build()
    return torch.device("cuda:0")


def _ref(mode, x, w, b, r):
    from packnet_sfm_amd.networks.layers.packnet.layers01 import packing
    conv = nn.Conv3d(1, w.shape[0], 3, 1, 1).double()
    with torch.no_grad():
        conv.weight.copy_(w.double())
        conv.bias.copy_(b.double())
    xd = x.detach().double().requires_grad_(True)
    v = packing(xd, r) if mode == 0 else xd
    y = conv(v.unsqueeze(1))
    B, c, d, h, ww = y.shape
    y = y.reshape(B, c * d, h, ww)
    if mode == 1:
        y = nn.PixelShuffle(r)(y)
    return xd, conv, y


@pytest.mark.parametrize("d", [8, 4])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,cl", [((2, 5, 14, 38), True), ((1, 16, 24, 40), False), ((2, 3, 6, 70), True),
                                      ((1, 40, 10, 36), True), ((2, 16, 22, 70), True)])
def test_matches_reference_chain(dev, mode, dtype, shape, cl, d):
    """d = 8: PackNet01; d = 4: PackNetSAN01 (num_3d_feat = 4).  bf16 channels_last pack layers with
    C % 8 == 0 ((1, 40, 10, 36): one 32-k chunk per tile pass of 5; (2, 16, 22, 70): 2 chunks, partial
    edge tiles) take the matrix-core weight gradient (k_p3d_bwd_w_mfma)."""
    from packnet_sfm_amd.networks.layers.packnet.pack3d import Pack3dFn
    g = torch.Generator().manual_seed(sum(shape) + mode + d)
    B, C, H, W = shape
    if mode == 1:
        C = C * 2  # d*C divisible by r^2 = 4
    x = torch.randn(B, C, H, W, generator=g).to(dtype)
    w = (torch.randn(d, 1, 3, 3, 3, generator=g) * 0.2)
    b = torch.randn(d, generator=g) * 0.1
    xd, conv, yref = _ref(mode, x.float(), w, b, 2)
    gy = torch.randn(yref.shape, generator=g).to(dtype).float()   # the upstream gradient in storage dtype
    (yref * gy.double()).sum().backward()
    xg = x.to(dev)
    if cl:
        xg = xg.contiguous(memory_format=torch.channels_last)
    xg.requires_grad_(True)
    wg = w.to(dev).requires_grad_(True)
    bg = b.to(dev).requires_grad_(True)
    y = Pack3dFn.apply(xg, wg, bg, mode, 2)
    (y.float() * gy.to(dev)).sum().backward()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    for got, ref in ((y, yref), (xg.grad, xd.grad)):
        err = (got.double().cpu() - ref).abs().max().item()
        assert err <= tol * ref.abs().max().item(), (err, ref.abs().max().item())
    wtol = 1e-5 if dtype == torch.float32 else 2e-3
    for got, ref in ((wg.grad, conv.weight.grad), (bg.grad, conv.bias.grad)):
        assert (got.double().cpu() - ref).abs().max().item() <= wtol * ref.abs().max().item()


def test_pack_layers_use_fused_op_and_match_torch(dev):
    """PackLayerConv3d / UnpackLayerConv3d on the device (fused) == the same modules' torch chain"""
    from packnet_sfm_amd.networks.layers.packnet import pack3d
    from packnet_sfm_amd.networks.layers.packnet.layers01 import PackLayerConv3d, UnpackLayerConv3d
    torch.manual_seed(0)
    for mod, shape in ((PackLayerConv3d(16, 3), (2, 16, 16, 32)), (UnpackLayerConv3d(32, 32, 3), (2, 32, 8, 16)),
                       (PackLayerConv3d(32, 5, d=4), (2, 32, 16, 32)),
                       (UnpackLayerConv3d(64, 32, 3, d=4), (2, 64, 8, 16))):
        mod = mod.to(dev)
        x = torch.randn(shape, device=dev)
        pack3d.ENABLED = False
        ref = mod(x)
        pack3d.ENABLED = True
        got = mod(x)
        assert (got - ref).abs().max().item() <= 1e-4 * ref.abs().max().item()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            pack3d.ENABLED = False
            ref16 = mod(x)
            pack3d.ENABLED = True
            got16 = mod(x)
        assert got16.dtype == ref16.dtype
        assert (got16.float() - ref16.float()).abs().max().item() <= 3e-2 * ref16.float().abs().max().item()


@pytest.mark.gpu
def test_decoder_merge_cat_feeds_the_same_bf16_input():
    """layers01.merge_cat under bf16 autocast (PackNet decoder stages): the concatenation of bf16
    features and an fp32 one-channel disparity is written channels_last in bf16 and equals what
    the reference chain hands the next autocast convolution (fp32 cat, then the bf16 cast), with
    the same gradients for every part."""
    import torch
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.networks.layers.packnet.layers01 import merge_cat
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(11)
    a = torch.randn(2, 16, 24, 40, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(2, 8, 24, 40, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    d = torch.rand(2, 1, 24, 40, generator=g).to(dev)
    parts = [t.detach().clone().requires_grad_(True) for t in (a, b, d)]
    refs = [t.detach().clone().requires_grad_(True) for t in (a, b, d)]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = merge_cat(parts)
    yr = torch.cat(refs, 1).to(torch.bfloat16)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y, yr)
    gy = torch.randn(y.shape, generator=g).to(dev, torch.bfloat16)
    y.backward(gy)
    yr.backward(gy)
    for p, r in zip(parts, refs):
        assert p.grad.dtype == r.grad.dtype and torch.equal(p.grad, r.grad)


@pytest.mark.parametrize("mode,d,shape", [(0, 8, (6, 64, 192, 640)), (0, 4, (4, 32, 384, 640)),
                                          (1, 8, (6, 64, 96, 320)), (1, 4, (4, 64, 192, 320))])
def test_real_layer_shapes_match_torch_chain(dev, mode, d, shape):
    """The first pack layer of PackNet01 (d = 8, B = 6, 192x640) / PackNetSAN01 on DDAD (d = 4,
    4 cameras, 384x640) and the last unpack layers, in the production storage (bf16, channels_last:
    the grid-size-dependent XCD-aware dx mapping and the o-in-passes staging at their real sizes)
    against the reference op chain in fp32 on the same device (packing / Conv3d / PixelShuffle,
    layers01.py:213-286) on the same bf16-rounded inputs: outputs and input gradient 1e-2 * max
    (one bf16 rounding), weight / bias gradients 2e-3 relative."""
    from packnet_sfm_amd.networks.layers.packnet.pack3d import Pack3dFn
    from packnet_sfm_amd.networks.layers.packnet.layers01 import packing
    g = torch.Generator(device="cpu").manual_seed(7 + mode + d)
    x = torch.randn(shape, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(d, 1, 3, 3, 3, generator=g) * 0.2).to(dev).to(torch.bfloat16).float()
    b = (torch.randn(d, generator=g) * 0.1).to(dev)
    xg, wg, bg = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    y = Pack3dFn.apply(xg, wg, bg, mode, 2)
    gy = torch.randn(y.shape, generator=g).to(dev, torch.bfloat16)
    y.backward(gy.contiguous(memory_format=torch.channels_last))
    # reference chain in fp32 on the same device
    xr = x.float().contiguous().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    v = packing(xr, 2) if mode == 0 else xr
    yr = torch.nn.functional.conv3d(v.unsqueeze(1), wr, br, 1, 1)
    B_, c, dd, h, ww = yr.shape
    yr = yr.reshape(B_, c * dd, h, ww)
    if mode == 1:
        yr = torch.nn.functional.pixel_shuffle(yr, 2)
    yr.backward(gy.float())
    torch.cuda.synchronize()

    def rel(a, r):
        return float((a.float() - r.float()).abs().max() / r.float().abs().max())
    errs = {"y": rel(y, yr), "dx": rel(xg.grad, xr.grad), "dW": rel(wg.grad, wr.grad), "db": rel(bg.grad, br.grad)}
    print(f"mode {mode} d={d} {shape}: " + ", ".join(f"{k} {v:.2e}" for k, v in errs.items()))
    assert errs["y"] <= 1e-2 and errs["dx"] <= 1e-2, errs
    assert errs["dW"] <= 2e-3 and errs["db"] <= 2e-3, errs


@pytest.mark.parametrize("d", [8, 4])
@pytest.mark.parametrize("mode,shape", [(0, (1, 40, 10, 36)), (0, (2, 16, 22, 70)), (0, (1, 10, 8, 20)), (0, (3, 12, 30, 34)),
                                        (0, (2, 32, 14, 38)),
                                        (1, (1, 40, 10, 36)), (1, (2, 16, 11, 35)), (1, (1, 8, 8, 20)), (1, (3, 48, 6, 34))])
def test_dx_matrix_core_and_valu_forms_match_the_reference(dev, knob, mode, d, shape):
    """dV of bf16 channels_last pack (mode 0) and unpack (mode 1) layers: the matrix-core form
    (k_p3d_bwd_x_mfma: 8-k chunks, weights split into bf16 hi + lo, fp32 shift-sum) and the VALU
    form (knob P3D_DX = 2: the k-pair kernel for pack layers with K % 16 == 0, the generic kernel
    otherwise) both within one bf16 rounding of the float64 reference chain (layers01.py:213-282),
    and within two bf16 ulps of each other.  Pack K = 160 / 64 / 40 / 48 and unpack K = 40 / 16 /
    8 / 48: 2 and 1 chunks per workgroup, partial edge tiles, first / last chunk halos.  (The
    grouped-staging form lost the A/B and is built into variant libraries only.)"""
    from packnet_sfm_amd.networks.layers.packnet.pack3d import Pack3dFn
    g = torch.Generator().manual_seed(sum(shape) + d + 10 * mode)
    x = torch.randn(shape, generator=g).to(torch.bfloat16)
    w = torch.randn(d, 1, 3, 3, 3, generator=g) * 0.2
    b = torch.randn(d, generator=g) * 0.1
    xd, conv, yref = _ref(mode, x.float(), w, b, 2)
    gy = torch.randn(yref.shape, generator=g).to(torch.bfloat16)
    (yref * gy.double()).sum().backward()
    grads = {}
    for form, value in (("mfma", 1), ("cl", 2)):
        knob("P3D_DX", value)
        xg = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        y = Pack3dFn.apply(xg, w.to(dev), b.to(dev), mode, 2)
        y.backward(gy.to(dev).contiguous(memory_format=torch.channels_last))
        grads[form] = xg.grad.double().cpu()
        ref = xd.grad
        err = (grads[form] - ref).abs().max().item()
        assert err <= 1e-2 * ref.abs().max().item(), (form, err, ref.abs().max().item())
    for form in ("mfma",):
        diff = (grads[form] - grads["cl"]).abs()
        assert (diff <= 2 * 2.0 ** -8 * grads["cl"].abs() + 3e-5 * grads["cl"].abs().max()).all(), (form, diff.max().item())


@pytest.mark.parametrize("d", [8, 4])
@pytest.mark.parametrize("shape", [(2, 64, 10, 36), (1, 96, 7, 19), (3, 32, 12, 40), (1, 128, 4, 6)])
def test_unpack_dw_matrix_core_matches_the_reference(dev, knob, d, shape):
    """Weight / bias gradient of bf16 channels_last UNPACK layers (layers01.py:226-282) on the
    matrix cores (k_p3d_bwd_w_mfma<d, UNPACK>: V = x staged as contiguous 8-k runs, pixel-shuffled
    dy staged per sub-pixel and interleaved) and on the VALU kernel (knob P3D_DW = 1): both
    within 2e-3 relative of the float64 reference chain; K = 64 / 96 / 32 / 128 (1 .. 4 chunks of
    32), partial edge tiles."""
    from packnet_sfm_amd.networks.layers.packnet.pack3d import Pack3dFn
    g = torch.Generator().manual_seed(sum(shape) + 3 * d)
    x = torch.randn(shape, generator=g).to(torch.bfloat16)
    w = torch.randn(d, 1, 3, 3, 3, generator=g) * 0.2
    b = torch.randn(d, generator=g) * 0.1
    xd, conv, yref = _ref(1, x.float(), w, b, 2)
    gy = torch.randn(yref.shape, generator=g).to(torch.bfloat16)
    (yref * gy.double()).sum().backward()
    for form, value in (("mfma", 0), ("generic", 1)):
        knob("P3D_DW", value)
        xg = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        wg, bg = w.to(dev).requires_grad_(True), b.to(dev).requires_grad_(True)
        y = Pack3dFn.apply(xg, wg, bg, 1, 2)
        y.backward(gy.to(dev).contiguous(memory_format=torch.channels_last))
        for got, ref in ((wg.grad, conv.weight.grad), (bg.grad, conv.bias.grad)):
            err = (got.double().cpu() - ref).abs().max().item()
            assert err <= 2e-3 * ref.abs().max().item(), (form, err, ref.abs().max().item())


@pytest.mark.parametrize("d", [8, 4])
@pytest.mark.parametrize("mode,shape", [(0, (1, 40, 10, 36)), (0, (2, 16, 22, 70)), (0, (3, 8, 14, 38)),
                                        (1, (2, 64, 10, 36)), (1, (1, 96, 7, 19)), (1, (3, 32, 12, 40))])
def test_forward_matrix_core_and_valu_forms_match_the_reference(dev, knob, mode, d, shape):
    """Forward of bf16 channels_last pack (mode 0) / unpack (mode 1) layers on the matrix cores
    (k_p3d_fwd_mfma: im2col rows of 16 k, weights split into bf16 hi + lo columns summed by a DPP
    rotate, the V tile staged twice for aligned reads) and on the VALU kernels (knob P3D_FWD = 2):
    both within one bf16 rounding of the float64 reference chain (layers01.py:126-282) and within
    two bf16 ulps of each other; K = 160 / 64 / 32 (pack), 64 / 96 / 32 (unpack), partial tiles."""
    from packnet_sfm_amd.networks.layers.packnet.pack3d import Pack3dFn
    g = torch.Generator().manual_seed(sum(shape) + 5 * d + mode)
    x = torch.randn(shape, generator=g).to(torch.bfloat16)
    w = torch.randn(d, 1, 3, 3, 3, generator=g) * 0.2
    b = torch.randn(d, generator=g) * 0.1
    _, _, yref = _ref(mode, x.float(), w, b, 2)
    ys = {}
    for form, value in (("mfma", 1), ("valu", 2)):
        knob("P3D_FWD", value)
        xg = x.to(dev).contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            ys[form] = Pack3dFn.apply(xg, w.to(dev), b.to(dev), mode, 2).double().cpu()
        err = (ys[form] - yref.detach()).abs().max().item()
        assert err <= 1e-2 * yref.abs().max().item(), (form, err)
    diff = (ys["mfma"] - ys["valu"]).abs()
    assert (diff <= 2 * 2.0 ** -8 * ys["valu"].abs() + 3e-5 * ys["valu"].abs().max()).all(), diff.max().item()
