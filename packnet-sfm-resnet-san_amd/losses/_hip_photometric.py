"""torch.autograd.Function over the HIP photometric kernels (K1 forward, K2 backward,
K3 smoothness, finalize / pose reduction) — DESIGN.md §Kernels.

Replaces the autograd graph that the reference builds out of ~1.2k ATen ops per step in
`MultiViewPhotometricLoss.forward` (losses/multiview_photometric_loss.py:331-410).
Gradients flow to the sigmoid depth maps and to the [R|t] pose matrices (the images are
data).
"""
import ctypes

import torch
import torch.nn.functional as F

from .. import _hip
from ..utils.image import NearestScales


# Optional live kernel timing (bench.py roofline): HIP events recorded on the stream the kernels
# are launched on (torch's current stream, which is also what we pass to the C-ABI).
KERNEL_TIMING = {"enabled": False, "events": [], "record": None}

# Training steps use K12 (forward + eager backward in one sweep, psfm_photometric_fwd_grad);
# False selects the unfused K1 forward / K2+K3 backward (tests compare the two).
FUSED_GRAD = True


def _run(name, fn, *args, keep=()):
    """One C-ABI launch; `args` end with the stream.  With KERNEL_TIMING["record"] a list, the
    call (minus its stream) is also recorded for graph replay timing (bench.py); `keep` holds the
    tensors whose raw pointers the call uses alive for that replay."""
    rec = KERNEL_TIMING.get("record")
    if rec is not None:
        rec.append((name, fn, args[:-1], keep))
    if KERNEL_TIMING["enabled"]:
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        rc = fn(*args)
        e.record()
        KERNEL_TIMING["events"].append((name, s, e))
    else:
        rc = fn(*args)
    _hip.check(rc, name)


def graph_replay_times_us(records, device, reps=10, iters=20):
    """Per-name average duration (us) of recorded C-ABI calls, each name's calls captured `reps`
    times into one HIP graph and replayed `iters` times between two HIP events on the replay
    stream (no host launch gaps).  `records` from KERNEL_TIMING["record"]."""
    names = []
    for r in records:
        if r[0] not in names:
            names.append(r[0])
    out = {}
    for name in names:
        sel = [r for r in records if r[0] == name]
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            for _, fn, a, _k in sel:   # warm outside capture
                _hip.check(fn(*a, _hip.stream(device)), name)
        torch.cuda.synchronize(device)
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                for _, fn, a, _k in sel:
                    _hip.check(fn(*a, _hip.stream(device)), name)
        g.replay()
        torch.cuda.synchronize(device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            g.replay()
        e1.record()
        torch.cuda.synchronize(device)
        out[name] = 1000.0 * e0.elapsed_time(e1) / (iters * reps)
        del g
    return out


def kernel_times_ms():
    """Sum of recorded durations per kernel name (synchronises); clears the record."""
    torch.cuda.synchronize()
    out = {}
    for name, s, e in KERNEL_TIMING["events"]:
        t, n = out.get(name, (0.0, 0))
        out[name] = (t + s.elapsed_time(e), n + 1)
    KERNEL_TIMING["events"].clear()
    return out


class _Call:
    """One ABI call: scales that share an image size (one call for the full-res case)."""

    def __init__(self, cfg, scale0, S, image, contexts, sigs, cam, mask, fused=False, cam_model=0, shifts=None):
        B, _, H, W = image.shape
        p = _hip.Params()
        p.B, p.H, p.W, p.N, p.S = B, H, W, len(contexts), S
        p.scale0, p.n_scales = scale0, cfg["n"]
        p.automask, p.reduce_op = int(cfg["automask"]), cfg["reduce_op"]
        p.l1_only = int(cfg["ssim_w"] <= 0.0)
        p.ssim_w, p.C1, p.C2 = cfg["ssim_w"], cfg["C1"], cfg["C2"]
        p.min_depth, p.max_depth = cfg["min_depth"], cfg["max_depth"]
        p.clip_loss, p.smooth_w = cfg["clip"], cfg["smooth_w"]
        p.grad_fused = int(fused)
        p.cam_model = cam_model
        for i, k in enumerate(shifts or ()):
            p.sig_shift[i] = int(k)
        self.params = p
        self.image, self.contexts, self.sigs, self.cam, self.mask = image, contexts, sigs, cam, mask
        inp = _hip.Inputs()
        inp.tgt = image.data_ptr()
        for j, c in enumerate(contexts):
            inp.ctx[j] = c.data_ptr()
        for s, t in enumerate(sigs):
            inp.sig[s] = t.data_ptr()
        inp.cam = cam.data_ptr()
        inp.mask = mask.data_ptr() if mask is not None else None
        self.inputs = inp
        # workspace (caller-owned; sized by the library)
        n = [ctypes.c_size_t() for _ in range(9)]
        _hip.check(_hip.lib().psfm_workspace_floats(ctypes.byref(p), *[ctypes.byref(x) for x in n]),
                   "psfm_workspace_floats")
        sizes = [x.value for x in n[:5]] + [n[6].value, n[7].value, n[8].value]
        total = sum(sizes)
        self.fbuf = torch.empty(total, device=image.device, dtype=torch.float32)
        self.abuf = torch.empty(max(n[5].value, 1), device=image.device, dtype=torch.uint8)
        ws = _hip.Workspace()
        off = 0
        base = self.fbuf.data_ptr()
        for name, sz in zip(("photo_part", "smooth_part", "clip_part", "clip_thr", "pose_part", "unwarp",
                             "sig_part", "cam_pairs"), sizes):
            setattr(ws, name, base + 4 * off if sz else None)
            off += sz
        ws.argmin = self.abuf.data_ptr()
        self.ws = ws


def _fisheye_records(K, ref_K, T, sw, sh, S, N, B, dev):
    """[S,N,B,CAMREC] fisheye records (include/psfm.h): target s, div, ux', uy' | context k0..k6,
    s, div, ux', uy' | T, centres scaled (c + 0.5) s - 0.5 per scale, k / s / div unscaled
    (losses/multiview_photometric_loss.py:166-186)."""
    def cam(c):
        return torch.stack([c["s"].float(), c["div"].float(), (c["ux"].float() + 0.5) * sw - 0.5,
                            (c["uy"].float() + 0.5) * sh - 0.5], -1).reshape(B, 4)
    tgt = cam(K).to(dev)
    ref = torch.cat([ref_K["k"].float().reshape(B, 7).to(dev), cam(ref_K).to(dev)], -1)
    rec = torch.zeros(S, N, B, _hip.CAMREC, device=dev, dtype=torch.float32)
    rec[..., 0:4] = tgt.reshape(1, 1, B, 4)
    rec[..., 4:15] = ref.reshape(1, 1, B, 11)
    rec[..., 18:30] = T.reshape(1, N, B, 12)
    return rec.contiguous()


def _sig_array(ts):
    return (ctypes.c_void_p * _hip.MAX_SCALES)(*([t.data_ptr() for t in ts] + [None] * (_hip.MAX_SCALES - len(ts))))


def _to_size(t, hw, mode):
    if tuple(t.shape[-2:]) == tuple(hw):
        return t
    if mode == "nearest":
        return F.interpolate(t, size=tuple(hw), mode="nearest").contiguous()
    return F.interpolate(t, size=tuple(hw), mode="bilinear", align_corners=True).contiguous()


class PhotometricLossFn(torch.autograd.Function):
    """loss, photometric metric, smoothness metric = f(sigs, T) given images and intrinsics."""

    @staticmethod
    def forward(ctx, cfg, image, mask, K, ref_K, T, n_ctx, *rest):
        _hip.note_forward(ctx)
        ctx.set_materialize_grads(False)   # no zero-filled grads for the metric outputs
        # detached: the per-call records (_Call) live on ctx, and an input with a grad_fn stored
        # there would form a ctx -> tensor -> graph -> ctx cycle that keeps every step's autograd
        # graph (and its AccumulateGrad nodes) alive until the garbage collector runs
        contexts = [c.detach().contiguous() for c in rest[:n_ctx]]
        sigs = [s.detach().contiguous() for s in rest[n_ctx:]]
        image = image.detach().contiguous()
        mask = mask.detach() if mask is not None else None
        _hip.require_device(image, mask, T, *contexts, *sigs)
        dev = image.device
        B, _, H, W = image.shape
        N, n = len(contexts), len(sigs)
        # T: [N,B,3,4] ([R|t]) or [N,B,4,4] (Pose.mat; its bottom row is constant)
        Tc = T.detach().float().contiguous()
        t_stride = 4 * T.shape[-2]

        # group consecutive scales of equal size into one call (full-res: one call for all);
        # stored coarse maps with a nearest 2^k mapping count as full size (cfg["shifts"])
        shifts = cfg.get("shifts")
        size = (lambda i: tuple(cfg["full_hw"])) if shifts else (lambda i: tuple(sigs[i].shape[-2:]))
        groups, s0 = [], 0
        while s0 < n:
            s1 = s0 + 1
            while s1 < n and size(s1) == size(s0) and s1 - s0 < _hip.MAX_SCALES:
                s1 += 1
            groups.append((s0, s1))
            s0 = s1
        # training step: K12 computes the gradient during the forward
        # (needs_input_grad is False everywhere under no_grad / for data-only inputs)
        wants_grad = any(ctx.needs_input_grad[5:])
        fish = isinstance(K, dict)
        fused = FUSED_GRAD and wants_grad and N <= 2 and cfg["ssim_w"] > 0.0
        if fish and (N > 2 or cfg["ssim_w"] <= 0.0 or (wants_grad and not fused)):
            raise NotImplementedError("fisheye (VADAS) cameras: N <= 2 contexts, SSIM candidates, and the K12 "
                                      "gradient path (FUSED_GRAD)")
        calls = []
        L = _hip.lib()
        for (a, b) in groups:
            hw = size(a)
            scale = hw[1] / float(W)  # Camera.scaled(DW/W) (camera.py:84-108)
            if fish:
                Tf = Tc[..., :3, :].reshape(N, B, 12)
                cam = _fisheye_records(K, ref_K, Tf, scale, hw[0] / float(H), b - a, N, B, dev)
            else:
                # Camera.scaled + Kinv + [R|t] records for every scale of the group: one launch
                # (include/psfm_pose.h; the ATen chain was ~15 small kernels on the critical path)
                cam = torch.empty(b - a, N, B, _hip.CAMREC, device=dev, dtype=torch.float32)
                Kc, Krc = K.float().contiguous(), ref_K.float().contiguous()
                _hip.require_device(Kc, Krc)
                _hip.check(L.psfm_pinhole_cam_records(_hip.ptr(Kc), _hip.ptr(Krc), _hip.ptr(Tc), t_stride, B, N,
                                                      b - a, scale, _hip.ptr(cam), _hip.stream(dev)),
                           "psfm_pinhole_cam_records")
            im = _to_size(image, hw, "bilinear")
            cx = [_to_size(c, hw, "bilinear") for c in contexts]
            mk = _to_size(mask, hw, "nearest").contiguous() if mask is not None else None
            calls.append(_Call(cfg, a, b - a, im, cx, sigs[a:b], cam, mk, fused,
                               _hip.CAM_FISHEYE if fish else _hip.CAM_PINHOLE,
                               shifts[a:b] if shifts else None))

        st = _hip.stream(dev)
        for c in calls:
            if cfg["clip"] > 0.0:
                _run("clip_stats", L.psfm_photometric_clip_stats, ctypes.byref(c.params),
                     ctypes.byref(c.inputs), ctypes.byref(c.ws), st, keep=(c,))
            if fused:   # K12's dL/dsig planes at the call's full size (grad_finish maps them to the stored size)
                c.gsig = [torch.empty(B, 1, c.params.H, c.params.W, device=dev, dtype=torch.float32) for _ in c.sigs]
                _run("prepass", L.psfm_photometric_prepass, ctypes.byref(c.params), ctypes.byref(c.inputs),
                     ctypes.byref(c.ws), st, keep=(c,))
                _run("K12_photometric_fwd_grad", L.psfm_photometric_fwd_grad, ctypes.byref(c.params),
                     ctypes.byref(c.inputs), ctypes.byref(c.ws), _sig_array(c.gsig), st, keep=(c,))
                continue
            _run("K1_photometric_fwd", L.psfm_photometric_fwd, ctypes.byref(c.params), ctypes.byref(c.inputs),
                 ctypes.byref(c.ws), st, keep=(c,))
            if cfg["smooth_w"] > 0.0:
                _run("K3_smoothness_fwd", L.psfm_smoothness_fwd, ctypes.byref(c.params),
                     ctypes.byref(c.inputs), ctypes.byref(c.ws), st, keep=(c,))
        smooth_stats = torch.empty(cfg["n"] * B * 4, device=dev, dtype=torch.float32)
        out = torch.empty(3, device=dev, dtype=torch.float32)
        pp = (ctypes.POINTER(_hip.Params) * len(calls))(*[ctypes.pointer(c.params) for c in calls])
        wp = (ctypes.POINTER(_hip.Workspace) * len(calls))(*[ctypes.pointer(c.ws) for c in calls])
        _run("finalize", L.psfm_finalize, len(calls), pp, wp, _hip.ptr(smooth_stats), _hip.ptr(out), st,
             keep=(calls, smooth_stats, out))
        ctx.calls, ctx.smooth_stats, ctx.cfg, ctx.n_ctx, ctx.T_shape = calls, smooth_stats, cfg, N, T.shape
        ctx.t_stride = t_stride
        ctx.fused = fused
        ctx.sig_shapes = [s.shape for s in sigs]
        loss, photo, smooth = out[0:1], out[1].clone(), out[2].clone()
        ctx.mark_non_differentiable(photo, smooth)
        return loss, photo, smooth

    @staticmethod
    def backward(ctx, g_loss, g_photo, g_smooth):
        _hip.capture_guard(ctx)
        calls, cfg = ctx.calls, ctx.cfg
        dev = calls[0].image.device
        gout = (g_loss if g_loss is not None else torch.zeros(1, device=dev)).reshape(1).float().contiguous()
        L = _hip.lib()
        st = _hip.stream(dev)
        N, B = ctx.n_ctx, calls[0].params.B
        pp = (ctypes.POINTER(_hip.Params) * len(calls))(*[ctypes.pointer(c.params) for c in calls])
        wp = (ctypes.POINTER(_hip.Workspace) * len(calls))(*[ctypes.pointer(c.ws) for c in calls])
        gT = torch.empty(N, B, ctx.t_stride, device=dev, dtype=torch.float32)
        if ctx.fused:  # gradient already computed by K12 for dL/dloss = 1: scale + normaliser term
            grads = []
            for c in calls:
                gsig = [torch.empty(t.shape, device=dev, dtype=torch.float32) for t in c.sigs]
                _run("grad_finish", L.psfm_photometric_grad_finish, ctypes.byref(c.params),
                     _hip.ptr(ctx.smooth_stats), _hip.ptr(gout), _sig_array(c.gsig), _sig_array(gsig), st,
                     keep=(c, ctx.smooth_stats, gout, gsig))
                grads.extend(gsig)
            _run("pose_grad_reduce", L.psfm_pose_grad_reduce_scaled, len(calls), pp, wp, _hip.ptr(gout),
                 _hip.ptr(gT), ctx.t_stride, st, keep=(calls, gout, gT))
            return (None, None, None, None, None, gT.reshape(ctx.T_shape), None) + (None,) * N + tuple(grads)
        grads = []
        for c in calls:
            gsig = [torch.empty(sh, device=dev, dtype=torch.float32) for sh in
                    ctx.sig_shapes[c.params.scale0:c.params.scale0 + c.params.S]]
            arr = _sig_array(gsig)
            _run("K2_photometric_bwd", L.psfm_photometric_bwd, ctypes.byref(c.params), ctypes.byref(c.inputs),
                 ctypes.byref(c.ws), _hip.ptr(gout), arr, st, keep=(c, gout, gsig))
            if cfg["smooth_w"] > 0.0:
                _run("K3_smoothness_bwd", L.psfm_smoothness_bwd, ctypes.byref(c.params), ctypes.byref(c.inputs),
                     _hip.ptr(ctx.smooth_stats), _hip.ptr(gout), arr, st, keep=(c, ctx.smooth_stats, gout, gsig))
            grads.extend(gsig)
        _run("pose_grad_reduce", L.psfm_pose_grad_reduce, len(calls), pp, wp, _hip.ptr(gT), ctx.t_stride, st,
             keep=(calls, gT))
        return (None, None, None, None, None, gT.reshape(ctx.T_shape), None) + (None,) * N + tuple(grads)


def photometric_loss_hip(image, contexts, sigs, K, ref_K, T, mask, cfg):
    """Returns (loss[1], metrics.photometric_loss, metrics.smoothness_loss).

    `sigs` a list of maps, or a NearestScales (utils/image.py): the stored maps and their 2^k
    nearest factors go to the kernels as psfm_params.sig_shift, gradients come back at the stored
    size.  The in-kernel mapping serves the K12 training path and the K1 forward path; the unfused
    backward (FUSED_GRAD off, N > 2, L1-only) gets the materialised upsample instead."""
    shifts = None
    if isinstance(sigs, NearestScales):
        wants_grad = torch.is_grad_enabled() and (T.requires_grad or any(s.requires_grad for s in sigs.stored))
        in_kernel = cfg["ssim_w"] > 0.0 and (not wants_grad or (FUSED_GRAD and len(contexts) <= 2))
        if in_kernel:
            shifts = tuple(sigs.shifts)
            cfg = dict(cfg, full_hw=tuple(sigs.shape), shifts=shifts)
        sigs = sigs.stored if in_kernel else sigs.materialize()
    return PhotometricLossFn.apply(cfg, image, mask, K, ref_K, T, len(contexts), *contexts, *sigs)


# -------------------------------------------------------------------------------------------------
class ViewSynthesisFn(torch.autograd.Function):
    """view_synthesis (geometry/camera_utils.py:27-59) on HIP: grads to depth and [R|t].
    `rec` [B, CAMREC-18] = the camera fields of the record (pinhole K^-1 | K, or the fisheye
    target | context parameters); T [B,3,4] target -> context."""

    @staticmethod
    def forward(ctx, ref_image, depth, rec, T, cam_model):
        _hip.note_forward(ctx)
        ref_image, depth = ref_image.contiguous(), depth.contiguous()
        _hip.require_device(ref_image, depth)
        B, _, H, W = ref_image.shape
        pad = torch.zeros(B, _hip.CAMREC - 30, device=depth.device)
        cam = torch.cat([rec.reshape(B, 18).float(), T.detach().reshape(B, 12).float(), pad], -1).contiguous()
        warped = torch.empty_like(ref_image)
        _hip.check(_hip.lib().psfm_view_synthesis_fwd(cam_model, B, H, W, _hip.ptr(ref_image), _hip.ptr(depth),
                                                      _hip.ptr(cam), _hip.ptr(warped),
                                                      _hip.stream(depth.device)), "view_synthesis_fwd")
        ctx.save_for_backward(ref_image, depth, cam)
        ctx.T_shape, ctx.cam_model = T.shape, cam_model
        return warped

    @staticmethod
    def backward(ctx, g):
        _hip.capture_guard(ctx)
        ref_image, depth, cam = ctx.saved_tensors
        B, _, H, W = ref_image.shape
        g = g.contiguous().float()
        gd = torch.empty_like(depth)
        tiles = _hip.tiles_per_image(H, W)
        part = torch.empty(B * tiles * 12, device=depth.device)
        gT = torch.empty(B, 12, device=depth.device)
        _hip.check(_hip.lib().psfm_view_synthesis_bwd(ctx.cam_model, B, H, W, _hip.ptr(ref_image), _hip.ptr(depth),
                                                      _hip.ptr(cam), _hip.ptr(g), _hip.ptr(gd),
                                                      _hip.ptr(part), _hip.ptr(gT),
                                                      _hip.stream(depth.device)), "view_synthesis_bwd")
        return None, gd, None, gT.reshape(ctx.T_shape), None
