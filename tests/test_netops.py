"""Fused network epilogues (include/psfm_netops.h) against plain PyTorch fp32 references of the
same ops (BatchNorm2d / GroupNorm / bias + ReLU / Sigmoid, forward and backward), and the module
wiring on CPU (the reference op chain).  Tolerances: outputs are bf16 (relative rounding 2^-8),
so activations / input gradients are compared at 2e-2 of the tensor's max magnitude, the fp32
parameter gradients and running statistics at 2e-3 relative."""
import pytest
import torch
import torch.nn as nn

import packnet_sfm_amd  # noqa: F401
from packnet_sfm_amd.networks.layers import fused as FU

gpu = pytest.mark.gpu


def _close(a, b, tol, where=None):
    a, b = a.float(), b.float()
    scale = b.abs().max().clamp(min=1e-6)
    d = (a - b).abs()
    if where is not None:
        d = d[where]
    err = d.max() / scale
    assert err < tol, f"max err {err:.3e} (scale {scale:.3e}) > {tol}"


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _check_conv_bias_grad(db, dx, db_ref, dx_ref, shape, rel):
    """Fused GroupNorm conv-bias gradient vs the fp32 chain: within the bf16 rounding noise of the
    M = N*H*W summands (4 sigma) + rel * max, and as close to the column sum of our own bf16 dx."""
    M = shape[0] * shape[2] * shape[3]
    noise = 4 * M ** 0.5 * 2 ** -8 * dx_ref.float().pow(2).mean().sqrt()
    own = dx.double().sum((0, 2, 3)).float()
    assert (db.float() - db_ref).abs().max() <= noise + rel * db_ref.abs().max()
    assert (db.float() - own).abs().max() <= noise + rel * own.abs().max()


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    import __graft_entry__
    __graft_entry__.build()
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def fused_on():
    """Every fused kind on (the product enables the measured winners, fused.FUSE)."""
    prev = dict(FU.FUSE)
    FU.FUSE.update(bias=True, gn=True, bn="resident")
    yield
    FU.FUSE.update(prev)


@gpu
@pytest.mark.parametrize("shape,act,bias_bf16", [((2, 16, 24, 80), FU.ACT_RELU, True),
                                                   ((2, 64, 12, 40), FU.ACT_RELU, False),
                                                   ((2, 256, 6, 20), FU.ACT_RELU, True),
                                                   ((2, 1, 48, 160), FU.ACT_SIGMOID, True),
                                                   ((2, 16, 48, 160), FU.ACT_SIGMOID, False),
                                                   # full-resolution decoder shapes: 480 workgroups, 30 reduction groups
                                                   ((4, 16, 192, 640), FU.ACT_RELU, True),
                                                   ((4, 1, 192, 640), FU.ACT_SIGMOID, True)])
def test_bias_act_matches_torch(dev, shape, act, bias_bf16):
    g = torch.Generator(device="cpu").manual_seed(1)
    x = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16).requires_grad_(True)
    b = torch.randn(shape[1], generator=g).to(dev, torch.bfloat16 if bias_bf16 else torch.float32).requires_grad_(True)
    owner = nn.Module()
    y = FU.bias_act(x, b, act, owner)
    # reference in fp32 on the same (bf16) values
    xr = x.detach().float().requires_grad_(True)
    br = b.detach().float().requires_grad_(True)
    u = xr + br.view(1, -1, 1, 1)
    yr = torch.relu(u) if act == FU.ACT_RELU else torch.sigmoid(u)
    _close(y, yr, 1e-2)
    assert y.dtype == (torch.float32 if act == FU.ACT_SIGMOID else torch.bfloat16)
    dy = torch.randn(shape, generator=g).to(dev, y.dtype)
    y.backward(_cl(dy))
    yr.backward(dy.float())
    _close(x.grad, xr.grad, 2e-2)
    # bias gradient = column sum of the stored bf16 dx (what autograd sums): tight w.r.t. our dx;
    # against the fp32 reference it carries the bf16 rounding noise of M summands
    own = x.grad.double().sum((0, 2, 3))
    out_tol = 2 ** -8 if bias_bf16 else 1e-6
    assert torch.allclose(b.grad.double(), own, rtol=out_tol, atol=1e-3 * own.abs().max().item() + 1e-6)
    M = shape[0] * shape[2] * shape[3]
    noise = 4 * M ** 0.5 * 2 ** -8 * xr.grad.float().pow(2).mean().sqrt()
    assert (b.grad.float() - br.grad).abs().max() <= noise + (2e-2 if bias_bf16 else 2e-3) * br.grad.abs().max()
    assert b.grad.dtype == b.dtype


@pytest.fixture(params=["resident8192", "resident2048"])
def bn_path(request, knob):
    """bn_act with the resident kernels taking every geometry they have (BN_RES_MAXM 8192: M = N*H*W <=
    8192 rows, C % 8 == 0) and with the product limit (2048); larger layers run MIOpen's BatchNorm + the
    fused (add +) ReLU pass (the library's other fused BatchNorm forms lost and were removed in round 6)."""
    knob("BN_RES_MAXM", 8192 if request.param == "resident8192" else 2048)
    return request.param


@gpu
@pytest.mark.parametrize("shape,relu,residual", [((2, 64, 48, 160), True, False),
                                                  ((4, 64, 96, 320), True, False),  # stem: 480 workgroups
                                                  ((2, 64, 24, 80), True, True),
                                                  ((4, 512, 6, 20), True, True),
                                                  ((2, 128, 12, 40), False, False),
                                                  ((2, 24, 10, 30), True, True),   # 3 channel blocks
                                                  # ResNet18 layer2-4 at B = 4, 192x640 (resident: forward
                                                  # RPT 8 x 960 threads, backward RPT 16 x 512; RPT 2 / 1)
                                                  ((4, 128, 24, 80), True, False),
                                                  ((4, 128, 24, 80), True, True),
                                                  ((4, 256, 12, 40), True, True),
                                                  ((4, 512, 6, 20), False, False),
                                                  ((3, 64, 7, 9), True, True),     # M = 189: a partial wave
                                                  ((2, 8, 64, 64), True, False)])  # M = 8192: the resident limit
def test_bn_act_matches_torch(dev, shape, relu, residual, bn_path):
    g = torch.Generator(device="cpu").manual_seed(2)
    C = shape[1]
    bn = nn.BatchNorm2d(C).to(dev).train()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.1)
    ref = nn.BatchNorm2d(C).to(dev).train()
    ref.load_state_dict(bn.state_dict())
    x = _cl(torch.randn(shape, generator=g) * 2 + 0.3).to(dev, torch.bfloat16).requires_grad_(True)
    r = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16).requires_grad_(True) if residual else None
    y = FU.bn_act(x, bn, relu=relu, residual=r)
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if residual else None
    yr = ref(xr)
    if residual:  # autocast semantics: bn(x) is a bf16 tensor before the add (identity gradient)
        yr = yr + (yr.detach().bfloat16().float() - yr.detach()) + rr
    # elements whose pre-activation sits within bf16 noise of the ReLU kink may take either
    # side in two correct implementations: their input gradient is excluded below
    far = (yr.detach().abs() > 2e-2) if relu else None
    if relu:
        yr = torch.relu(yr)
    _close(y, yr, 2e-2)
    _close(bn.running_mean, ref.running_mean, 2e-3)
    _close(bn.running_var, ref.running_var, 2e-3)
    dy = torch.randn(shape, generator=g).to(dev, torch.bfloat16)
    y.backward(_cl(dy))
    yr.backward(dy.float())
    _close(x.grad, xr.grad, 2e-2, far)
    # layers the resident kernels do not take run MIOpen's bf16 BatchNorm (the reference op chain),
    # whose dgamma / dbeta sit up to ~5e-2 from the fp32 chain at these sizes; the fused kernels' fp32 /
    # fp64 reductions are held to 2e-2
    from packnet_sfm_amd import _hip
    fused = bool(_hip.lib().psfm_bn_act_resident(shape[0] * shape[2] * shape[3], C))
    ptol = 2e-2 if fused else 1e-1
    _close(bn.weight.grad, ref.weight.grad, ptol)
    _close(bn.bias.grad, ref.bias.grad, ptol)
    if residual:
        _close(r.grad, rr.grad, 2e-2, far)


@pytest.fixture(params=["resident", "twopass"])
def gn_path(request, knob):
    """Both GroupNorm implementations: the one-pass resident kernels (default wherever the layer
    fits a workgroup's registers) and the two-pass statistics-rows kernels (knob GN_PATH = 1;
    always used for the large layers)."""
    knob("GN_PATH", 1 if request.param == "twopass" else 0)
    return request.param


# GN shapes: two-pass (large HW), resident both ways at every row-vector count (RPT 1 / 2 / 4 of a
# 256-thread workgroup) and channel block (cpg 1 / 2 / 4 -> 8-channel blocks of 8 / 4 / 2 groups,
# cpg 16 / 32 -> 2 / 4 vector columns), resident forward + two-pass backward (res, RPT 4)
GN_SHAPES = [(4, 16, 96, 320), (4, 64, 24, 80), (4, 256, 3, 10), (2, 32, 5, 7), (6, 16, 24, 80),
             (6, 32, 12, 40), (6, 128, 48, 160), (6, 512, 12, 40), (6, 512, 6, 20), (3, 64, 60, 160),
             (2, 384, 6, 20)]   # 24 channels per group: not a resident geometry, two-pass kernels


@gpu
@pytest.mark.parametrize("shape", GN_SHAPES)
def test_gn_act_matches_torch(dev, shape, gn_path):
    g = torch.Generator(device="cpu").manual_seed(3)
    C = shape[1]
    conv_b = torch.randn(C, generator=g).to(dev, torch.bfloat16).requires_grad_(True)
    gn = nn.GroupNorm(16, C).to(dev)
    with torch.no_grad():
        gn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        gn.bias.copy_(torch.randn(C, generator=g) * 0.1)
    x = _cl(torch.randn(shape, generator=g) + 0.5).to(dev, torch.bfloat16).requires_grad_(True)
    y = FU.gn_act(x, conv_b, gn, relu=True)
    xr = x.detach().float().requires_grad_(True)
    br = conv_b.detach().float().requires_grad_(True)
    wr = gn.weight.detach().clone().requires_grad_(True)
    betar = gn.bias.detach().clone().requires_grad_(True)
    yr = torch.relu(torch.nn.functional.group_norm(xr + br.view(1, -1, 1, 1), 16, wr, betar, gn.eps))
    _close(y, yr, 2e-2)
    dy = torch.randn(shape, generator=g).to(dev, torch.bfloat16)
    y.backward(_cl(dy))
    yr.backward(dy.float())
    _close(x.grad, xr.grad, 2e-2)
    # conv-bias gradient in closed form from the statistics rows (sum_hw dx = k1 S1 - HW k2 - k3 X):
    # the sum of the exact dx; autograd would sum the bf16-rounded dx instead, which differs from
    # it by the rounding noise of M summands — both within that noise of the fp32 reference
    _check_conv_bias_grad(conv_b.grad, x.grad, br.grad, xr.grad, shape, 3e-2)
    _close(gn.weight.grad, wr.grad, 2e-2)
    _close(gn.bias.grad, betar.grad, 2e-2)


@gpu
@pytest.mark.parametrize("shape,residual", [((4, 256, 12, 40), True), ((4, 512, 6, 20), False)])
def test_fused_bn_is_bitwise_deterministic_and_captures(dev, shape, residual):
    """The resident BatchNorm (one launch each way, fixed-order reductions, no atomics): eager calls
    repeat bit for bit, and a HIP-graph capture of forward + backward replays the eager results bit for
    bit, twice (running statistics included)."""
    from packnet_sfm_amd import _hip
    N, C, H, W = shape
    assert _hip.lib().psfm_bn_act_resident(N * H * W, C) == 1
    assert _hip.lib().psfm_bn_act_fused(N * H * W, C) == 1
    g = torch.Generator(device="cpu").manual_seed(11)
    x = _cl(torch.randn(shape, generator=g) + 0.2).to(dev, torch.bfloat16)
    r = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16) if residual else None
    dy = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16)
    bn = nn.BatchNorm2d(C).to(dev).train()
    bn.num_batches_tracked = None   # as the graph trainer keeps it (no host-side counter in the graph)
    state = [bn.running_mean.clone(), bn.running_var.clone()]

    def reset():
        bn.running_mean.copy_(state[0])
        bn.running_var.copy_(state[1])

    def step(xi):
        y = FU.bn_act(xi, bn, relu=True, residual=r)
        dx, dw, db = torch.autograd.grad(y, (xi, bn.weight, bn.bias), dy)
        return [y, dx, dw, db, bn.running_mean.clone(), bn.running_var.clone()]

    outs = []
    for _ in range(2):
        reset()
        outs.append([t.detach().clone() for t in step(x.clone().requires_grad_(True))])
        torch.cuda.synchronize()
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)
    reset()
    xs = x.clone().requires_grad_(True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            cap = step(xs)
    torch.cuda.current_stream().wait_stream(side)
    for _ in range(2):
        reset()
        graph.replay()
        torch.cuda.synchronize()
        for a_, b_ in zip(cap, outs[0]):
            assert torch.equal(a_, b_)


@gpu
def test_bn_policies_route_the_shapes(dev, monkeypatch):
    """FUSE["bn"] == "resident" (the product default): only the layers the resident kernels take (M <=
    2048 rows: ResNet18 layer3 / layer4) run fused, the larger ones and C % 8 != 0 MIOpen's BatchNorm;
    "all" routes the same shapes on the product library (A/B builds add the two-launch form)."""
    calls = []
    orig = FU._BNAct.apply
    monkeypatch.setattr(FU._BNAct, "apply", lambda *a: calls.append(tuple(a[0].shape)) or orig(*a))
    shapes = ((4, 256, 12, 40), (4, 128, 24, 80), (4, 64, 48, 160), (2, 12, 10, 30))
    for policy in ("resident", "all"):   # the same on the product library (no other fused form)
        FU.FUSE["bn"] = policy
        for shape in shapes:
            bn = nn.BatchNorm2d(shape[1]).to(dev).train()
            x = _cl(torch.randn(shape)).to(dev, torch.bfloat16)
            FU.bn_act(x, bn, relu=True)
    assert calls == [(4, 256, 12, 40)] * 2


@gpu
def test_resnet_encoder_fused_matches_unfused(dev):
    """The whole ResNet18 encoder + decoder: fused bf16 epilogues are as close to an fp32 run of
    the reference op chain as the reference's own bf16-autocast run is (same weights)."""
    from packnet_sfm_amd.networks.depth.ResNetSAN01 import ResNetSAN01
    torch.manual_seed(0)
    net = ResNetSAN01(version="18A").to(dev).train().to(memory_format=torch.channels_last)
    x = _cl(torch.rand(2, 3, 96, 320)).to(dev)

    def run(enabled, amp):
        FU.FUSE.update(bias=enabled, gn=enabled, bn="resident" if enabled else False)
        try:
            net.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                sig = net(x)["inv_depths"]
            loss = sum(s.float().mean() for s in sig)
            loss.backward()
            return ([s.detach().float() for s in sig],
                    [net.decoder.convs[("dispconv", 0)].conv.bias.grad.detach().float().clone(),
                     net.encoder.encoder.conv1.weight.grad.detach().float().clone(),
                     net.encoder.encoder.layer4[1].bn2.weight.grad.detach().float().clone()])
        finally:
            FU.FUSE.update(bias=True, gn=True, bn="resident")

    ref = run(False, False)
    fused, plain = run(True, True), run(False, True)

    def err(a, b):
        return float((a - b).abs().max() / b.abs().max().clamp(min=1e-12))

    for k in range(4):
        ef, ep = err(fused[0][k], ref[0][k]), err(plain[0][k], ref[0][k])
        assert ef <= 2.0 * ep + 1e-2, (k, ef, ep)
    for k in range(3):
        ef, ep = err(fused[1][k], ref[1][k]), err(plain[1][k], ref[1][k])
        assert ef <= 2.0 * ep + 2e-2, (k, ef, ep)


def test_gn_shapes_outside_the_kernels_take_the_torch_chain():
    """psfm_gn_act_* reject N > 64, G > 128, C > 512 (psfm_netops.hip gn_setup); gn_act must send those
    shapes to the reference op chain instead of raising."""
    assert FU.gn_shape_ok((64, 64, 8, 8), 16)
    assert not FU.gn_shape_ok((65, 64, 8, 8), 16)
    assert not FU.gn_shape_ok((2, 1024, 8, 8), 16)
    assert not FU.gn_shape_ok((2, 256, 8, 8), 256)
    assert not FU.gn_shape_ok((2, 60, 8, 8), 16)
    torch.manual_seed(0)
    gn = nn.GroupNorm(16, 32)
    x, b = torch.randn(65, 32, 3, 4), torch.randn(32)
    assert torch.equal(FU.gn_act(x, b, gn, True), torch.relu(gn(x + b.view(1, -1, 1, 1))))


def test_cpu_path_is_the_reference_op_chain():
    """On CPU the helpers are exactly the reference's modules (BN -> +res -> ReLU etc.)."""
    torch.manual_seed(0)
    bn = nn.BatchNorm2d(8).train()
    x, r = torch.randn(2, 8, 5, 6), torch.randn(2, 8, 5, 6)
    ref = nn.BatchNorm2d(8).train()
    ref.load_state_dict(bn.state_dict())
    assert torch.equal(FU.bn_act(x, bn, True, r), torch.relu(ref(x) + r))
    gn = nn.GroupNorm(4, 8)
    b = torch.randn(8)
    assert torch.equal(FU.gn_act(x, b, gn, True), torch.relu(gn(x + b.view(1, -1, 1, 1))))
    assert torch.equal(FU.bias_act(x, b, FU.ACT_SIGMOID, nn.Module()), torch.sigmoid(x + b.view(1, -1, 1, 1)))
    # the stem: relu -> MaxPool2d(3, 2, 1), the skip and the pooled output forked for two consumers
    pool = nn.MaxPool2d(3, 2, 1)
    xs = torch.randn(2, 8, 6, 10)
    bn2 = nn.BatchNorm2d(8).train()
    ref2 = nn.BatchNorm2d(8).train()
    ref2.load_state_dict(bn2.state_dict())
    skip, h0, h1 = FU.bn_relu_maxpool(xs, bn2, pool, nout=2)
    rs = torch.relu(ref2(xs))
    assert torch.equal(skip, rs) and torch.equal(h0, pool(rs)) and torch.equal(h1, pool(rs))
    # the nets' input images: the reference's normalisation and concatenation (fp32 on CPU)
    ims = [torch.rand(2, 3, 4, 6) for _ in range(3)]
    assert torch.equal(FU.normalize_input(ims[0], 0.45, 0.225), (ims[0] - 0.45) / 0.225)
    assert torch.equal(FU.cat_input(ims), torch.cat(ims, 1))


@gpu
@pytest.mark.parametrize("N,C1,C2,h,w", [(4, 256, 256, 6, 20), (4, 16, 0, 96, 320), (2, 32, 64, 48, 160),
                                         (1, 8, 24, 3, 5)])
def test_upcat_matches_torch(dev, N, C1, C2, h, w):
    """psfm_upcat vs the reference's op chain cat([F.interpolate(x, 2, 'nearest'), skip]):
    forward and dskip bitwise; dx = the 2x2 block sums of dout, fp32 accumulation with one bf16
    rounding (1 bf16 ulp of the fp32 sum); the kernel actually runs (no op-chain fallback)."""
    torch.manual_seed(1)
    x = _cl(torch.randn(N, C1, h, w)).to(dev).bfloat16().requires_grad_(True)
    skip = _cl(torch.randn(N, C2, 2 * h, 2 * w)).to(dev).bfloat16().requires_grad_(True) if C2 else None
    calls = []
    orig = FU._UpCat.apply
    FU._UpCat.apply = lambda *a: calls.append(1) or orig(*a)
    try:
        out = FU.up_cat(x, skip)
    finally:
        FU._UpCat.apply = orig
    assert calls and out.is_contiguous(memory_format=torch.channels_last)
    up = torch.nn.functional.interpolate(x.detach(), scale_factor=2, mode="nearest")
    ref = up if skip is None else torch.cat([up, skip.detach()], 1)
    assert torch.equal(out, ref)
    dout = _cl(torch.randn(out.shape)).to(dev).bfloat16()
    out.backward(dout)
    blk = dout[:, :C1].float().reshape(N, C1, h, 2, w, 2).sum((3, 5))
    assert (x.grad.float() - blk).abs().max() <= (blk.abs() * 2.0 ** -8).max() + 1e-30
    if skip is not None:
        assert torch.equal(skip.grad, dout[:, C1:])


@gpu
@pytest.mark.parametrize("shape,residual,bias", [((6, 64, 96, 320), True, True), ((6, 32, 48, 160), False, True),
                                                 ((2, 256, 12, 40), True, False), ((2, 32, 5, 7), False, True),
                                                 ((6, 128, 48, 160), True, True), ((6, 256, 24, 80), True, True),
                                                 ((6, 64, 24, 80), True, True), ((6, 512, 6, 20), False, True)])
def test_gn_elu_matches_torch(dev, shape, residual, bias, gn_path):
    """PackNet Conv2D / ResidualConv epilogue: ELU(GroupNorm(16)(x [+ res] + bias)) and its backward
    (dx, dres, dbias, dgamma, dbeta) against the fp32 torch chain (layers01.py:10-61)."""
    g = torch.Generator(device="cpu").manual_seed(5)
    C = shape[1]
    conv_b = torch.randn(C, generator=g).to(dev, torch.bfloat16).requires_grad_(True) if bias else None
    gn = nn.GroupNorm(16, C).to(dev)
    with torch.no_grad():
        gn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        gn.bias.copy_(torch.randn(C, generator=g) * 0.1)
    x = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16).requires_grad_(True)
    r = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16).requires_grad_(True) if residual else None
    y = FU.gn_act(x, conv_b, gn, act=FU.ACT_ELU, residual=r)
    assert y.grad_fn is not None and "GNAct" in type(y.grad_fn).__name__
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if residual else None
    br = conv_b.detach().float().requires_grad_(True) if bias else None
    wr = gn.weight.detach().clone().requires_grad_(True)
    betar = gn.bias.detach().clone().requires_grad_(True)
    s = xr + (rr if residual else 0) + (br.view(1, -1, 1, 1) if bias else 0)
    yr = torch.nn.functional.elu(torch.nn.functional.group_norm(s, 16, wr, betar, gn.eps))
    _close(y, yr, 2e-2)
    dy = torch.randn(shape, generator=g).to(dev, torch.bfloat16)
    y.backward(_cl(dy))
    yr.backward(dy.float())
    _close(x.grad, xr.grad, 2e-2)
    if residual:
        assert torch.equal(r.grad, x.grad)
    if bias:
        _check_conv_bias_grad(conv_b.grad, x.grad, br.grad, xr.grad, shape, 3e-2)
    _close(gn.weight.grad, wr.grad, 2e-2)
    _close(gn.bias.grad, betar.grad, 2e-2)


@gpu
@pytest.mark.parametrize("shape,act,residual", [((2, 64, 24, 80), FU.ACT_ELU, True), ((4, 16, 96, 320), FU.ACT_RELU, False)])
def test_gn_forward_only_captures_into_a_hip_graph(dev, shape, act, residual):
    """The forward-only GroupNorm call (eval / no_grad: PackNet's eval forward) captured into a HIP
    graph, three calls per graph: replays equal the eager calls bit for bit, also after the input
    changed (a stale partial row or a stats pass outside the graph would show).  This is the call
    whose capture once crashed (round-2 commit 2c99221); the reductions now keep no device state
    between launches (no lazily allocated arrival counters)."""
    g = torch.Generator(device="cpu").manual_seed(6)
    C = shape[1]
    gn = nn.GroupNorm(16, C).to(dev)
    with torch.no_grad():
        gn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        gn.bias.copy_(torch.randn(C, generator=g) * 0.1)
    b = torch.randn(C, generator=g).to(dev, torch.bfloat16)
    xs = [_cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16) for _ in range(2)]
    rs = [_cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16) if residual else None for _ in range(2)]
    call = lambda x, r: FU.gn_act(x, b, gn, act=act, residual=r)  # noqa: E731
    with torch.no_grad():
        eager = [call(x, r) for x, r in zip(xs, rs)]
        x_st = xs[0].clone()
        r_st = rs[0].clone() if residual else None
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            call(x_st, r_st)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            outs = [call(x_st, r_st) for _ in range(3)]
        for k in (0, 1):
            x_st.copy_(xs[k])
            if residual:
                r_st.copy_(rs[k])
            graph.replay()
            torch.cuda.synchronize()
            for y in outs:
                assert torch.equal(y, eager[k])


@gpu
def test_gn_and_bias_reductions_are_deterministic(dev):
    """GroupNorm + ELU and bias + ReLU forward / backward repeated: every output and gradient bit
    identical run to run (fixed-order partial-row reductions, no atomics)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    gn = nn.GroupNorm(16, 64).to(dev)
    x = _cl(torch.randn(4, 64, 48, 160, generator=g)).to(dev, torch.bfloat16)
    r = _cl(torch.randn(4, 64, 48, 160, generator=g)).to(dev, torch.bfloat16)
    b = torch.randn(64, generator=g).to(dev, torch.bfloat16)
    dy = _cl(torch.randn(4, 64, 48, 160, generator=g)).to(dev, torch.bfloat16)
    outs = []
    for _ in range(3):
        xi, ri, bi = x.clone().requires_grad_(True), r.clone().requires_grad_(True), b.clone().requires_grad_(True)
        gn.zero_grad(set_to_none=True)
        y = FU.gn_act(xi, bi, gn, act=FU.ACT_ELU, residual=ri)
        z = FU.bias_act(y, bi, FU.ACT_RELU)
        z.backward(dy)
        torch.cuda.synchronize()
        outs.append([t.detach().clone() for t in (y, z, xi.grad, ri.grad, bi.grad, gn.weight.grad, gn.bias.grad)])
    for o in outs[1:]:
        for a_, b_ in zip(o, outs[0]):
            assert torch.equal(a_, b_)


@gpu
@pytest.mark.parametrize("N,C1,C2,h,w,bias_bf16", [(4, 256, 256, 6, 20, True), (4, 16, 0, 96, 320, True),
                                                  (2, 32, 64, 48, 160, False), (1, 128, 64, 3, 5, True)])
def test_conv_block_up_cat_equals_the_unfused_chain(dev, N, C1, C2, h, w, bias_bf16):
    """psfm_upcat_bias_relu (ConvBlock bias + ReLU folded into the up-stage input) == bias_act then
    up_cat: output, dx and dskip bitwise; the bias gradient sums the same bf16 values in another
    order (1e-6 of max)."""
    g = torch.Generator(device="cpu").manual_seed(C1 + h)
    x = _cl(torch.randn(N, C1, h, w, generator=g)).to(dev, torch.bfloat16)
    b = torch.randn(C1, generator=g).to(dev, torch.bfloat16 if bias_bf16 else torch.float32)
    skip = _cl(torch.randn(N, C2, 2 * h, 2 * w, generator=g)).to(dev, torch.bfloat16) if C2 else None
    dout = _cl(torch.randn(N, C1 + C2, 2 * h, 2 * w, generator=g)).to(dev, torch.bfloat16)
    res = []
    for fused in (True, False):
        xi, bi = x.clone().requires_grad_(True), b.clone().requires_grad_(True)
        si = skip.clone().requires_grad_(True) if skip is not None else None
        y = FU._UpCatBiasReLU.apply(xi, bi, si) if fused else FU.up_cat(FU.bias_act(xi, bi, FU.ACT_RELU), si)
        y.backward(dout)
        res.append((y.detach(), xi.grad, bi.grad, si.grad if si is not None else None))
    (yf, dxf, dbf, dsf), (yu, dxu, dbu, dsu) = res
    assert torch.equal(yf, yu) and torch.equal(dxf, dxu)
    assert (dsf is None and dsu is None) or torch.equal(dsf, dsu)
    assert dbf.dtype == b.dtype
    assert (dbf.float() - dbu.float()).abs().max() <= 1e-6 * dbu.float().abs().max() + (2 ** -8 if bias_bf16 else 0) * dbu.float().abs().max()


@gpu
@pytest.mark.parametrize("shape,cl", [((4, 64, 48, 160), True), ((4, 512, 6, 20), True), ((2, 8, 3, 5), False)])
def test_add_relu_equals_the_op_chain_bitwise(dev, shape, cl):
    """The BasicBlock tail relu(bn_out + identity) (psfm_add_relu_fwd / psfm_relu_mask_bwd) equals
    autocast's bf16 add + relu and their backward bit for bit (incl. zeros, -0, inf and NaN outputs)."""
    g = torch.Generator(device="cpu").manual_seed(8)
    mk = lambda: torch.randn(shape, generator=g).to(dev, torch.bfloat16)  # noqa: E731
    a, b = mk(), mk()
    a.view(-1)[:4] = torch.tensor([0.0, -0.0, float("inf"), float("nan")], dtype=torch.bfloat16)
    b.view(-1)[:4] = torch.tensor([0.0, 0.0, 1.0, 1.0], dtype=torch.bfloat16)
    if cl:
        a, b = _cl(a), _cl(b)
    a1, b1 = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
    a2, b2 = a.clone().requires_grad_(True), b.clone().requires_grad_(True)
    calls = []
    orig = FU._AddReLU.apply
    FU._AddReLU.apply = lambda *x: calls.append(1) or orig(*x)
    try:
        y1 = FU.add_relu(a1, b1)
    finally:
        FU._AddReLU.apply = orig
    y2 = torch.relu(a2 + b2)
    assert calls and torch.equal(y1.nan_to_num(), y2.nan_to_num()) and y1.stride() == y2.stride()
    dy = mk()
    dy = _cl(dy) if cl else dy
    y1.backward(dy)
    y2.backward(dy)
    assert torch.equal(a1.grad, a2.grad) and torch.equal(b1.grad, b2.grad)


@gpu
@pytest.mark.parametrize("shape,nout", [((4, 64, 96, 320), 2), ((2, 64, 96, 320), 1), ((3, 24, 10, 14), 2),
                                        ((1, 8, 2, 2), 2)])
def test_stem_relu_maxpool_equals_the_op_chain_bitwise(dev, shape, nout):
    """The stem's relu -> MaxPool2d(3, 2, 1) (psfm_relu_maxpool_fwd/bwd via fused.bn_relu_maxpool's
    HIP branch) equals ATen's relu + max_pool2d and autograd's backward (the pooled output read by
    nout consumers, the skip by one) bit for bit: the pooled max and ties (relu zeros: first in window
    order), NaN propagation, ATen's fp32 window sum in (oh, ow) order, the bf16 adds, the ReLU mask."""
    g = torch.Generator(device="cpu").manual_seed(12)
    y = torch.randn(shape, generator=g).permute(0, 2, 3, 1).contiguous()   # NHWC storage
    y.view(-1)[:5] = torch.tensor([float("nan"), 0.0, -0.0, float("inf"), -float("inf")])
    y.view(-1)[-3 * shape[1]:] = 0.0           # three pixels of ties at zero
    y = y.permute(0, 3, 1, 2).to(dev, torch.bfloat16)
    assert y.is_contiguous(memory_format=torch.channels_last)
    pool = nn.MaxPool2d(3, 2, 1)
    y1, y2 = y.clone().requires_grad_(True), y.clone().requires_grad_(True)
    calls = []
    orig = FU._ReLUMaxPool.apply
    FU._ReLUMaxPool.apply = lambda *a: calls.append(1) or orig(*a)
    try:
        out1 = FU._ReLUMaxPool.apply(y1, nout) if FU._stem_pool_ok(y1, pool) else None
    finally:
        FU._ReLUMaxPool.apply = orig
    assert calls and out1 is not None
    r2 = torch.relu(y2)
    p2 = pool(r2)
    out2 = (r2,) + (p2,) * nout
    assert len(out1) == len(out2)
    for a, b in zip(out1, out2):
        assert torch.equal(a.nan_to_num(), b.nan_to_num())
        assert a.is_contiguous(memory_format=torch.channels_last) == b.is_contiguous(memory_format=torch.channels_last)
    grads = [_cl(torch.randn(o.shape, generator=g)).to(dev, torch.bfloat16) for o in out2]
    torch.autograd.backward(out1, grads)
    torch.autograd.backward(out2, grads)
    assert torch.equal(y1.grad, y2.grad)


@gpu
def test_stem_relu_maxpool_routes_the_resnet_stem(dev):
    """bn_relu_maxpool: MIOpen's BatchNorm + the fused pass where the stem is beyond the resident
    BatchNorm (B = 4, 192 x 640: M = 122880 rows); bench.py --no-stem-pool keeps add_relu + ATen."""
    g = torch.Generator(device="cpu").manual_seed(13)
    bn, pool = nn.BatchNorm2d(64).to(dev).train(), nn.MaxPool2d(3, 2, 1)
    x = _cl(torch.randn((4, 64, 96, 320), generator=g)).to(dev, torch.bfloat16)
    seen = []
    orig = FU._ReLUMaxPool.apply
    FU._ReLUMaxPool.apply = lambda *a: seen.append(1) or orig(*a)
    try:
        skip, h0, h1 = FU.bn_relu_maxpool(x, bn, pool, nout=2)
        FU.STEM_POOL = False
        s2, g0, g1 = FU.bn_relu_maxpool(x, bn, pool, nout=2)
    finally:
        FU._ReLUMaxPool.apply = orig
        FU.STEM_POOL = True
    assert seen == [1]
    assert torch.equal(skip, s2) and torch.equal(h0, g0) and torch.equal(h1, g1)


@gpu
@pytest.mark.parametrize("shape,cl", [((4, 3, 192, 640), True), ((4, 3, 192, 640), False), ((1, 3, 5, 7), True),
                                      ((2, 3, 9, 11), False)])
def test_net_input_normalisation_equals_the_op_chain_bitwise(dev, shape, cl):
    """fused.normalize_input under bf16 autocast (psfm_normalize_bf16) = ATen's (x - 0.45) / 0.225 +
    autocast's bf16 cast, bit for bit and in the same layout (odd sizes: the scalar tail)."""
    g = torch.Generator(device="cpu").manual_seed(14)
    x = torch.rand(shape, generator=g) * 1.2 - 0.1
    x.view(-1)[:3] = torch.tensor([0.45, 0.0, 1.0])
    x = (_cl(x) if cl else x).to(dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = FU.normalize_input(x, 0.45, 0.225)   # bf16 out = the HIP pass (the op chain returns fp32)
        ref = ((x - 0.45) / 0.225).to(torch.bfloat16)
    assert y.dtype == torch.bfloat16 and y.stride() == ref.stride() and y.stride() == x.stride()
    assert torch.equal(y, ref)
    FU.NET_INPUTS = False
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert FU.normalize_input(x, 0.45, 0.225).dtype == torch.float32   # the op chain
    finally:
        FU.NET_INPUTS = True


@gpu
@pytest.mark.parametrize("k,shape", [(3, (4, 3, 192, 640)), (3, (4, 3, 24, 40)), (2, (2, 3, 24, 40)),
                                     (1, (2, 3, 24, 40)), (3, (1, 3, 5, 7))])   # 35 px: a partial block, odd size
def test_pose_input_concatenation_equals_the_op_chain_bitwise(dev, k, shape):
    """fused.cat_input under bf16 autocast (psfm_cat_channels_bf16) = torch.cat of the channels_last
    fp32 images + the bf16 cast, bit for bit, channels_last."""
    g = torch.Generator(device="cpu").manual_seed(15)
    ims = [_cl(torch.rand(shape, generator=g)).to(dev) for _ in range(k)]
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = FU.cat_input(ims)
        ref = torch.cat(ims, 1).to(torch.bfloat16)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    assert ref.is_contiguous(memory_format=torch.channels_last) and torch.equal(y, ref)


@gpu
def test_posenet_forward_unchanged_by_the_fused_inputs(dev):
    """PoseNet's forward under bf16 autocast is bit-identical with and without the fused input pass."""
    from packnet_sfm_amd.networks.pose.PoseNet import PoseNet
    torch.manual_seed(3)
    net = PoseNet(nb_ref_imgs=2, rotation_mode="euler").to(dev).train().to(memory_format=torch.channels_last)
    g = torch.Generator(device="cpu").manual_seed(16)
    ims = [_cl(torch.rand((2, 3, 64, 96), generator=g)).to(dev) for _ in range(3)]
    outs = []
    for flag in (True, False):
        FU.NET_INPUTS = flag
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                outs.append(net(ims[0], ims[1:]).detach().float())
        finally:
            FU.NET_INPUTS = True
    assert torch.equal(outs[0], outs[1])


@gpu
def test_gn_backward_captures_when_its_forward_ran_on_the_capture_stream(dev):
    """tools/gn_bench.py's round-3 capture segfault, resolved (profiles/r04/cap): 20 captured
    torch.autograd.grad calls through psfm_gn_act_bwd at [6, 64, 192, 640] replay bit-exactly when
    the forward ran on the stream the graph captures on.  (With the forward on the default stream
    the autograd engine launches the backward there, outside the capture, and HIP crashes in
    capture_end: tools/diag_gn_capture.py --capture-bwd, a usage error the step graph never makes —
    it captures forward and backward together.)"""
    g = torch.Generator(device="cpu").manual_seed(9)
    shape, C = (6, 64, 192, 640), 64
    gn = nn.GroupNorm(16, C).to(dev)
    b = torch.randn(C, generator=g).to(dev)
    x = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16).requires_grad_(True)
    dy = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16)
    cs = torch.cuda.Stream()
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        y = FU.gn_act(x, b, gn, act=FU.ACT_ELU)
        ref = torch.autograd.grad(y, x, dy, retain_graph=True)[0].clone()
    torch.cuda.current_stream().wait_stream(cs)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=cs):
        for _ in range(19):
            torch.autograd.grad(y, x, dy, retain_graph=True)
        out = torch.autograd.grad(y, x, dy, retain_graph=True)[0]
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)



_CAPTURE_MISUSE = r"""
import sys, torch, torch.nn as nn
sys.path.insert(0, {root!r})
import packnet_sfm_amd
from packnet_sfm_amd.networks.layers import fused as FU
dev = torch.device("cuda", 0)
gn = nn.GroupNorm(16, 64).to(dev)
x = torch.randn(6, 64, 48, 160, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
x.requires_grad_(True)
from packnet_sfm_amd import _hip
_guard = _hip.capture_guard
def _loud_guard(*a):
    try:
        _guard(*a)
    except RuntimeError:
        print("GUARD RAISED", flush=True)
        raise
_hip.capture_guard = _loud_guard
y = FU.gn_act(x, None, gn, act=FU.ACT_ELU)          # forward on the default stream, outside any capture
dy = torch.randn_like(y)
torch.cuda.synchronize()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            z = dy * 2                              # a node of the capture's own (HIP refuses an empty graph)
            torch.autograd.grad(y, x, dy)           # its backward captured: the round-4 segfault sequence
except RuntimeError as e:
    print("REFUSED:", "refusing to begin a HIP-graph capture" in str(e) and "_GNAct" in str(e), flush=True)
else:
    print("NOT REFUSED")
    sys.exit(2)
# the refused capture never began: the eager backward runs, and then a capture on the side stream works
gx, = torch.autograd.grad(y, x, dy)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(side):
    with torch.cuda.graph(g, stream=side):
        z = dy * 2
g.replay()
torch.cuda.synchronize()
assert torch.equal(z, dy * 2)
print("AFTER BACKWARD: captured and replayed", flush=True)
sys.exit(0)
"""


@gpu
def test_bn_backward_follows_the_forward_form_when_the_knob_changes(dev, knob):
    """the BatchNorm backward reuses the forward's decision (resident kernels, no
    workspace) even if BN_RES_MAXM changes between forward and backward; its gradients equal those
    of an unperturbed run bitwise."""
    g = torch.Generator(device="cpu").manual_seed(4)
    shape = (4, 256, 12, 40)
    x0 = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16)
    dy = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16)
    outs = []
    for perturb in (False, True):
        bn = nn.BatchNorm2d(shape[1]).to(dev).train()
        x = x0.clone().requires_grad_(True)
        knob("BN_RES_MAXM", 2048)
        y = FU.bn_act(x, bn, relu=True)
        assert y.grad_fn is not None and "BNAct" in type(y.grad_fn).__name__
        if perturb:
            knob("BN_RES_MAXM", 0)     # the forward's form is no longer the policy for this shape
        y.backward(dy)
        outs.append((x.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@gpu
def test_backward_captured_for_a_forward_on_another_stream_raises(dev):
    """capturing the backward of a fused op whose forward ran outside the capture
    on another stream (the round-4 segfault sequence) is refused by the capture_begin hook BEFORE the
    capture exists (_hip.note_forward / _refuse_stray_backward) — raising from the op's backward came
    too late: the autograd engine had already made the capturing stream wait on the forward's stream,
    and HIP segfaulted in capture_end.  The sequence runs in a child process, which must exit cleanly
    with the refusal; then the backward runs eagerly, the pending set empties, and a capture on the
    same side stream begins and replays."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _CAPTURE_MISUSE.format(root=root)], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, (out.returncode, out.stdout[-2000:], out.stderr[-3000:])
    assert "REFUSED: True" in out.stdout and "GUARD RAISED" not in out.stdout, out.stdout
    assert "AFTER BACKWARD: captured and replayed" in out.stdout, out.stdout


@gpu
@pytest.mark.parametrize("kind", ["add_relu", "relu", "bn_resident", "bias_relu"])
def test_forked_outputs_sum_their_gradients_like_autograd(dev, kind):
    """fused._fork: an op asked for nout outputs returns views of one result; its backward sums the
    views' gradients in the kernel's load.  Two consumers: bitwise what autograd computes when the
    plain output is read twice (its bf16 add = fp32 sum, one rounding); three consumers: within one
    bf16 rounding of it (autograd may accumulate in another order)."""
    g = torch.Generator(device="cpu").manual_seed(12)
    shape = (4, 256, 12, 40)
    a = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16)
    b = _cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16)
    bias = torch.randn(shape[1], generator=g).to(dev, torch.bfloat16)
    dys = [_cl(torch.randn(shape, generator=g)).to(dev, torch.bfloat16) for _ in range(3)]
    bn = nn.BatchNorm2d(shape[1]).to(dev).train()
    bn.num_batches_tracked = None
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()

    def run(nout, ncons):
        bn.running_mean.copy_(rm)
        bn.running_var.copy_(rv)
        ai, bi, wi = a.clone().requires_grad_(True), b.clone().requires_grad_(True), bias.clone().requires_grad_(True)
        if kind == "add_relu":
            out = FU.add_relu(ai, bi, nout=nout)
        elif kind == "relu":
            out = FU.add_relu(ai, None, nout=nout)
        elif kind == "bn_resident":
            out = FU.bn_act(ai, bn, relu=True, residual=bi, nout=nout)
        else:
            out = FU.bias_act(ai, wi, FU.ACT_RELU, nout=nout)
        outs = out if isinstance(out, tuple) else (out,) * ncons
        sum((o.float() * d.float()).sum() for o, d in zip(outs, dys[:ncons])).backward()
        return [t for t in (ai.grad, bi.grad if kind in ("add_relu", "bn_resident") else None,
                            wi.grad if kind == "bias_relu" else None) if t is not None]

    for ncons in (2, 3):
        if kind == "bias_relu" and ncons == 3:
            continue
        fork, plain = run(ncons, ncons), run(1, ncons)
        for f, p in zip(fork, plain):
            if ncons == 2:
                assert torch.equal(f, p), (kind, ncons, float((f.float() - p.float()).abs().max()))
            else:
                _close(f, p, 1e-2)
