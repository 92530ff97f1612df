"""CPU checks of the drop-in boundary: the C-ABI library builds, loads, exports every symbol
include/psfm.h declares, and rejects bad arguments without touching a GPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hip():
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd import _hip
    return _hip


def declared_functions():
    names = set()
    for h in sorted(f for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h")):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(psfm_[a-z_0-9]+)\s*\(", src))
    return sorted(names)


def test_every_declared_symbol_is_exported(hip):
    L = hip.lib()
    decl = declared_functions()
    assert len(decl) >= 12
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(hip.EXPORTED) == decl


def test_packconv_abi_validates_without_a_gpu(hip):
    """psfm_packconv.h: workspace / weight-buffer sizes and descriptor validation are host-only."""
    from packnet_sfm_amd.networks.layers.packnet import packconv
    L = hip.lib()
    t = packconv.PcDesc(B=6, C=64, H=192, W=640, k=5, d=8)
    t.xs[:] = [64 * 192 * 640, 1, 640 * 64, 64]
    t.ys[:] = [64 * 96 * 320, 1, 320 * 64, 64]
    ws, wb = L.psfm_pc_ws_floats(ctypes.byref(t)), L.psfm_pc_wbuf_bytes(ctypes.byref(t))
    assert ws > 6 * 320 * 4 * 256 and wb > 2 * 64 * 256 * 49 * 2
    w = packconv.PcWeights()
    assert L.psfm_pc_weights_of(ctypes.byref(t), ctypes.c_void_p(4096), ctypes.byref(w)) == 0
    assert w.wf == 4096 and w.wb > w.wf and w.bt > w.corner
    for bad in (dict(k=7), dict(d=2), dict(C=48), dict(H=191), dict(H=8, W=8)):
        tb = packconv.PcDesc(**{**dict(B=6, C=64, H=192, W=640, k=5, d=8), **bad})
        tb.xs[:] = list(t.xs)
        tb.ys[:] = list(t.ys)
        assert L.psfm_pc_ws_floats(ctypes.byref(tb)) == -1
        assert hip.lib().psfm_pc_last_error()
    tc = packconv.PcDesc(B=6, C=64, H=192, W=640, k=5, d=8)
    tc.xs[:] = [64 * 192 * 640, 640, 1, 192 * 640]   # NCHW: refused (channels_last only)
    tc.ys[:] = list(t.ys)
    assert L.psfm_pc_ws_floats(ctypes.byref(tc)) == -1


def test_workspace_sizes(hip):
    p = hip.Params(B=4, H=192, W=640, N=2, S=4, scale0=0, n_scales=4, automask=1, reduce_op=0)
    n = [ctypes.c_size_t() for _ in range(9)]
    assert hip.lib().psfm_workspace_floats(ctypes.byref(p), *[ctypes.byref(x) for x in n]) == 0
    tiles = hip.tiles_per_image(192, 640)
    assert tiles == 10 * 48
    assert n[0].value >= 4 * 4 * tiles
    assert n[4].value >= 4 * 2 * 4 * tiles * 12
    assert n[5].value == 4 * 4 * 192 * 640
    assert n[6].value == 2 * 4 * 192 * 640
    assert n[7].value == 4 * 4 * 16   # sigmoid chunk sums of the K12 pre-pass
    assert n[8].value == 4 * 4 * 48 * 2   # context-paired camera records (K12: + M = K_ref R, m = K_ref t)


def test_fused_path_argument_checks(hip):
    """psfm_photometric_fwd_grad: K12 needs grad_fused=1, N <= 2 and SSIM candidates"""
    L = hip.lib()
    inp, ws = hip.Inputs(), hip.Workspace()
    p = hip.Params(B=1, H=8, W=8, N=3, S=1, scale0=0, n_scales=1, automask=1, reduce_op=0, ssim_w=0.85,
                   grad_fused=1)
    inp.tgt = inp.cam = 1
    for j in range(3):
        inp.ctx[j] = 1
    inp.sig[0] = 1
    assert L.psfm_photometric_fwd_grad(ctypes.byref(p), ctypes.byref(inp), ctypes.byref(ws), None, None) == -15
    p.N, p.grad_fused = 2, 0
    assert L.psfm_photometric_fwd_grad(ctypes.byref(p), ctypes.byref(inp), ctypes.byref(ws), None, None) == -15
    p.grad_fused = 1
    assert L.psfm_photometric_fwd_grad(ctypes.byref(p), ctypes.byref(inp), ctypes.byref(ws), None, None) == -12
    assert b"workspace" in L.psfm_last_error()
    assert L.psfm_photometric_grad_finish(ctypes.byref(p), None, None, None, None, None) == -14
    assert L.psfm_pose_grad_reduce_scaled(0, None, None, None, None, 12, None) == -1
    assert L.psfm_pose_from_vec_fwd(None, 1, 1, None, None) == -1
    assert L.psfm_pose_from_vec_bwd(None, 1, 9, None, None, None) == -1
    assert L.psfm_pinhole_cam_records(None, None, None, 12, 1, 1, 1, 1.0, None, None) == -1


def test_round5_netops_argument_checks(hip):
    """The round-5 netops entry points refuse bad shapes / pointers before any launch (host-only):
    the stem pool needs even H, W and C % 8 == 0; the input passes need aligned pointers, 1-4 inputs
    and <= 32 channels."""
    L = hip.lib()
    a = ctypes.c_void_p(4096)
    assert L.psfm_relu_maxpool_fwd(a, 2, 96, 320, 64, None, a, a, None) == -1          # no relu_out
    assert L.psfm_relu_maxpool_fwd(a, 2, 95, 320, 64, a, a, a, None) == -1            # odd H
    assert L.psfm_relu_maxpool_fwd(a, 2, 96, 320, 12, a, a, a, None) == -1            # C % 8
    assert b"relu_maxpool_fwd" in L.psfm_netops_last_error()
    assert L.psfm_relu_maxpool_bwd(a, None, None, a, a, 2, 96, 321, 64, a, None) == -1  # odd W
    assert L.psfm_normalize_bf16(ctypes.c_void_p(4100), 16, 0.45, 1.0, a, None) == -1   # x not 16-byte aligned
    assert L.psfm_normalize_bf16(a, 0, 0.45, 1.0, a, None) == -1
    P, CI = ctypes.c_void_p * 5, ctypes.c_int * 5
    xs, cs = P(*[4096] * 5), CI(*[3] * 5)
    assert L.psfm_cat_channels_bf16(5, xs, cs, 100, a, None) == -1                    # > 4 inputs
    assert L.psfm_cat_channels_bf16(2, xs, CI(*[20] * 5), 100, a, None) == -1         # 40 > 32 channels
    assert L.psfm_cat_channels_bf16(2, xs, cs, 100, ctypes.c_void_p(4098), None) == -1   # y not 4-byte aligned
    assert b"cat_channels_bf16" in L.psfm_netops_last_error()


@pytest.mark.parametrize("field,value,code", [("N", 0, -3), ("N", 5, -3), ("S", 0, -4), ("H", 1, -2),
                                              ("reduce_op", 7, -6)])
def test_bad_arguments_are_rejected(hip, field, value, code):
    p = hip.Params(B=1, H=8, W=8, N=2, S=1, scale0=0, n_scales=1, automask=1, reduce_op=0)
    setattr(p, field, value)
    inp, ws = hip.Inputs(), hip.Workspace()
    rc = hip.lib().psfm_photometric_fwd(ctypes.byref(p), ctypes.byref(inp), ctypes.byref(ws), None)
    assert rc == code
    assert hip.lib().psfm_last_error()


def test_automask_requires_min(hip):
    p = hip.Params(B=1, H=8, W=8, N=2, S=1, scale0=0, n_scales=1, automask=1, reduce_op=1)
    rc = hip.lib().psfm_photometric_fwd(ctypes.byref(p), ctypes.byref(hip.Inputs()),
                                        ctypes.byref(hip.Workspace()), None)
    assert rc == -7
    assert b"min" in hip.lib().psfm_last_error()


def test_product_path_refuses_cpu_tensors(hip):
    import torch
    from packnet_sfm_amd.geometry.pose import Pose
    from packnet_sfm_amd.losses.multiview_photometric_loss import MultiViewPhotometricLoss
    B, H, W = 1, 8, 16
    fn = MultiViewPhotometricLoss(photometric_reduce_op="min", automask_loss=True)
    with pytest.raises(RuntimeError, match="ROCm"):
        fn(torch.rand(B, 3, H, W), [torch.rand(B, 3, H, W)] * 2, [torch.rand(B, 1, H, W)] * 4,
           torch.eye(3).expand(B, 3, 3), torch.eye(3).expand(B, 3, 3),
           [Pose.identity(B)] * 2)


def test_optim_plan_chunks(hip):
    """host-side work split of the fused Adam step (include/psfm_optim.h)"""
    L = hip.lib()
    numel = (ctypes.c_int64 * 4)(1, 1024, 1025, 3000)
    n = L.psfm_optim_plan_chunks(4, numel, None, 0)
    assert n == 1 + 1 + 2 + 3
    buf = (ctypes.c_int32 * (2 * n))()
    assert L.psfm_optim_plan_chunks(4, numel, buf, n) == n
    assert list(buf) == [0, 0, 1, 0, 2, 0, 2, 1024, 3, 0, 3, 1024, 3, 2048]
    assert L.psfm_optim_plan_chunks(4, numel, buf, n - 1) == -3
    assert L.psfm_optim_last_error()
    assert L.psfm_grad_pack(None, None, 1, None, None) == -1
    assert L.psfm_adam_step(None, None, 1, None, None, None, ctypes.c_float(1.0), None, None, None, None) == -1


def test_depth_metrics_argument_checks(hip):
    L = hip.lib()
    p = hip.MetricsParams(B=0, H=4, W=4, min_depth=0.0, max_depth=80.0, crop_garg=1, use_gt_scale=1)
    assert L.psfm_depth_metrics(ctypes.byref(p), None, None, None, None, None) == -1
    assert L.psfm_depth_metrics(ctypes.byref(p), 1, 1, 1, 1, None) == -2
    assert b"B/H/W" in L.psfm_metrics_last_error()


def test_depth_metrics_refuses_cpu_tensors(hip):
    import types
    import torch
    from packnet_sfm_amd.utils.depth import compute_depth_metrics
    cfg = types.SimpleNamespace(min_depth=0.0, max_depth=80.0, crop="garg", scale_output="top-center")
    with pytest.raises(RuntimeError, match="ROCm"):
        compute_depth_metrics(cfg, torch.ones(1, 1, 8, 8), torch.ones(1, 1, 8, 8))


def test_library_carries_the_source_hash():
    """build() compiles the sources' sha256 into the library (psfm_version): the built .so must be
    the one the current sources produce (a stale library would make every GPU result unattributable)."""
    import __graft_entry__ as G
    assert G.library_hash() == G.source_hash(), "libpsfm_hip.so is stale: run __graft_entry__.build()"
    from packnet_sfm_amd import _hip
    assert _hip.lib().psfm_version().decode().endswith("src=" + G.source_hash())


def test_bn_resident_shapes(hip):
    """psfm_bn_act_resident (host-only): the one-launch BatchNorm holds 8-channel blocks of up to
    8192 rows — ResNet18 layer2-4 at B = 4, 192x640 — and nothing wider or larger."""
    L = hip.lib()
    assert hip.knobs()["BN_RES_MAXM"] == (2048, 2048)   # product policy: layer3 / layer4
    for M, C in ((1920, 256), (480, 512), (2048, 8), (1, 8)):
        assert L.psfm_bn_act_resident(M, C) == 1, (M, C)
    for M, C in ((7680, 128), (2049, 8), (30720, 64), (122880, 64), (480, 12), (0, 64)):
        assert L.psfm_bn_act_resident(M, C) == 0, (M, C)
    for M, C in ((1920, 256), (480, 512)):   # the product library's fused BatchNorm = the resident shapes
        assert L.psfm_bn_act_fused(M, C) == 1, (M, C)
    for M, C in ((122880, 64), (30720, 64), (7680, 128), (480, 12), (64, 1024)):
        assert L.psfm_bn_act_fused(M, C) == 0, (M, C)
    prev = hip.set_knob("BN_RES_MAXM", 8192)   # the kernels themselves hold up to 8192 rows
    try:
        assert L.psfm_bn_act_resident(7680, 128) == 1 and L.psfm_bn_act_resident(8192, 8) == 1
        assert L.psfm_bn_act_resident(8193, 8) == 0
    finally:
        hip.set_knob("BN_RES_MAXM", prev)


def test_knobs_are_read_once_and_set_explicitly(hip):
    """include/psfm_knobs.h: every kernel-selection knob has a name, a default and a range; the
    product configuration has no non-default knob; set / restore work; out-of-range values and
    unknown names are refused."""
    k = hip.knobs()
    assert set(k) == {"K12_PRIO", "K12_PARTS", "P3D_FWD", "P3D_DX", "P3D_DW", "GN_PATH", "BN_PATH", "BN_RES_MAXM",
                      "GN_RES_RPT"}
    assert hip.nondefault_knobs() == {}
    prev = hip.set_knob("GN_PATH", 1)
    try:
        assert hip.knobs()["GN_PATH"] == (1, 0) and hip.nondefault_knobs() == {"GN_PATH": 1}
    finally:
        hip.set_knob("GN_PATH", prev)
    assert hip.nondefault_knobs() == {}
    L = hip.lib()
    assert L.psfm_knob_set(b"GN_PATH", 7) == -1 and L.psfm_knob_set(b"NO_SUCH", 0) == -1
    for name, value in (("P3D_DX", 3), ("BN_PATH", 1), ("BN_PATH", 2), ("K12_PRIO", 1)):   # removed forms
        with pytest.raises(ValueError):
            hip.set_knob(name, value)


def test_knob_environment_is_parsed_at_load():
    """PSFM_<NAME> is read when the library loads (names or integers; invalid values keep the
    default, are reported on stderr and listed as rejected) — in a fresh process, since this one
    has loaded the library already."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import torch, packnet_sfm_amd; "
            "from packnet_sfm_amd import _hip; print(sorted(_hip.nondefault_knobs().items()))" % ROOT)
    env = dict(os.environ, PSFM_P3D_FWD="valu", PSFM_K12_PRIO="0", PSFM_GN_PATH="bogus", PSFM_BN_PATH="threepass",
               PSFM_GN_PIPE="0")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == ("[('BN_PATH', 'rejected:threepass'), ('GN_PATH', 'rejected:bogus'), "
                                                   "('K12_PRIO', 0), ('P3D_FWD', 2)]")
    assert "ignoring PSFM_GN_PATH=bogus" in out.stderr and "ignoring PSFM_BN_PATH=threepass" in out.stderr
    assert "PSFM_GN_PIPE is set but that form was removed" in out.stderr
    env = dict(os.environ, PSFM_K12_PRIO="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.strip().splitlines()[-1] == "[('K12_PRIO', 'rejected:1')]", out
