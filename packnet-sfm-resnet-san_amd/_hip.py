"""ctypes binding of the HIP C-ABI (include/psfm.h) — the only way the product path
reaches the kernels.  There is deliberately NO fallback: if `libpsfm_hip.so` is missing or
the tensors are not on a ROCm device, the call raises.

The library is loaded after `torch` so that its `libamdhip64.so.7` dependency resolves to the
HIP runtime torch already loaded (one runtime per process: device pointers and streams are
shared with PyTorch-ROCm).
"""
import ctypes
import os
import threading
import weakref

import torch

LIB_NAME = "libpsfm_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
DEFAULT_LIB_PATH = LIB_PATH

MAX_CTX = 4
MAX_SCALES = 4
CAMREC = 32
REDUCE_MIN, REDUCE_MEAN = 0, 1
CAM_PINHOLE, CAM_FISHEYE = 0, 1

c_int, c_float, c_void_p, c_size_t = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t


class Params(ctypes.Structure):
    """psfm_params (include/psfm.h)."""
    _fields_ = [("B", c_int), ("H", c_int), ("W", c_int), ("N", c_int), ("S", c_int),
                ("scale0", c_int), ("n_scales", c_int), ("automask", c_int), ("reduce_op", c_int),
                ("l1_only", c_int), ("ssim_w", c_float), ("C1", c_float), ("C2", c_float),
                ("min_depth", c_float), ("max_depth", c_float), ("clip_loss", c_float),
                ("smooth_w", c_float), ("grad_fused", c_int), ("cam_model", c_int),
                ("sig_shift", c_int * MAX_SCALES)]


class Inputs(ctypes.Structure):
    """psfm_inputs."""
    _fields_ = [("tgt", c_void_p), ("ctx", c_void_p * MAX_CTX), ("sig", c_void_p * MAX_SCALES),
                ("cam", c_void_p), ("mask", c_void_p)]


class Workspace(ctypes.Structure):
    """psfm_workspace."""
    _fields_ = [("photo_part", c_void_p), ("smooth_part", c_void_p), ("clip_part", c_void_p),
                ("clip_thr", c_void_p), ("pose_part", c_void_p), ("argmin", c_void_p),
                ("unwarp", c_void_p), ("sig_part", c_void_p), ("cam_pairs", c_void_p)]


class MetricsParams(ctypes.Structure):
    """psfm_metrics_params (include/psfm_metrics.h)."""
    _fields_ = [("B", c_int), ("H", c_int), ("W", c_int), ("min_depth", c_float), ("max_depth", c_float),
                ("crop_garg", c_int), ("use_gt_scale", c_int)]


class Jitter(ctypes.Structure):
    """psfm_jitter (include/psfm_augment.h)."""
    _fields_ = [("apply", c_int), ("order", c_int * 4), ("factor", c_float * 3), ("hue_shift", c_int),
                ("use_matrix", c_int), ("matrix", c_float * 3)]


class AugmentParams(ctypes.Structure):
    """psfm_augment_params (include/psfm_augment.h)."""
    _fields_ = [("n_samples", c_int), ("n_img", c_int), ("src_h", c_int), ("src_w", c_int),
                ("src_stride", ctypes.c_longlong), ("crop_l", c_int), ("crop_t", c_int), ("crop_r", c_int),
                ("crop_b", c_int), ("out_h", c_int), ("out_w", c_int)]


_lib = None
REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _graft_entry():
    """The repo's __graft_entry__ module (source_hash / library_hash), by path."""
    import importlib.util
    import sys
    mod = sys.modules.get("__graft_entry__")
    if mod is None:
        spec = importlib.util.spec_from_file_location("__graft_entry__", os.path.join(REPO_ROOT, "__graft_entry__.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules["__graft_entry__"] = mod
    return mod


POSE_MAX_CTX = 8  # include/psfm_pose.h PSFM_POSE_MAX_CTX


def lib():
    """Load (once) and return the HIP library; raise loudly if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP extension {LIB_PATH} is not built: run `python -c 'import "
                           f"__graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
    G = _graft_entry()
    have, want = G.library_hash(LIB_PATH), G.source_hash()
    # the product library must be the one the tree's sources build (A/B tools may point LIB_PATH at
    # a variant build under build/variants; only the default path is checked)
    if LIB_PATH == DEFAULT_LIB_PATH and have != want:
        raise RuntimeError(f"{LIB_PATH} was built from sources {have}, the tree holds {want}: rebuild "
                           f"(__graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    P, PP, V = ctypes.POINTER(Params), ctypes.POINTER(ctypes.POINTER(Params)), c_void_p
    WS, WSP, IN = ctypes.POINTER(Workspace), ctypes.POINTER(ctypes.POINTER(Workspace)), ctypes.POINTER(Inputs)
    sz = ctypes.POINTER(c_size_t)
    sig = {
        "psfm_workspace_floats": ([P, sz, sz, sz, sz, sz, sz, sz, sz, sz], c_int),
        "psfm_photometric_clip_stats": ([P, IN, WS, V], c_int),
        "psfm_photometric_fwd": ([P, IN, WS, V], c_int),
        "psfm_smoothness_fwd": ([P, IN, WS, V], c_int),
        "psfm_finalize": ([c_int, PP, WSP, V, V, V], c_int),
        "psfm_photometric_bwd": ([P, IN, WS, V, V, V], c_int),
        "psfm_smoothness_bwd": ([P, IN, V, V, V, V], c_int),
        "psfm_pose_grad_reduce": ([c_int, PP, WSP, V, c_int, V], c_int),
        "psfm_photometric_prepass": ([P, IN, WS, V], c_int),
        "psfm_photometric_fwd_grad": ([P, IN, WS, V, V], c_int),
        "psfm_photometric_grad_finish": ([P, V, V, V, V, V], c_int),
        "psfm_pose_grad_reduce_scaled": ([c_int, PP, WSP, V, V, c_int, V], c_int),
        "psfm_view_synthesis_fwd": ([c_int, c_int, c_int, c_int, V, V, V, V, V], c_int),
        "psfm_view_synthesis_bwd": ([c_int, c_int, c_int, c_int, V, V, V, V, V, V, V, V], c_int),
        "psfm_tiles_per_image": ([c_int, c_int], c_int),
        "psfm_last_error": ([], ctypes.c_char_p),
        "psfm_version": ([], ctypes.c_char_p),
        "psfm_k12_stamps": ([V, c_int, V], c_int),
        # include/psfm_optim.h
        "psfm_optim_plan_chunks": ([c_int, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32), c_int],
                                   c_int),
        "psfm_grad_pack": ([V, V, c_int, V, V], c_int),
        "psfm_adam_step": ([V, V, c_int, V, V, V, c_float, V, V, V, V], c_int),
        "psfm_optim_last_error": ([], ctypes.c_char_p),
        # include/psfm_netops.h
        "psfm_netops_ws_floats": ([c_int, c_int], c_size_t),
        "psfm_gn_ws_floats": ([c_int, c_int, c_int, c_int], c_size_t),
        "psfm_bias_act_fwd": ([V, V, c_int, c_int, c_int, c_int, V, V], c_int),
        "psfm_bias_act_bwd": ([V, V, c_int, c_int, c_int, V, V, c_int, V, V], c_int),
        "psfm_bias_act_bwd_sum": ([V, V, V, c_int, c_int, c_int, V, V, c_int, V, V], c_int),
        "psfm_bn_act_fwd": ([V, V, V, V, V, V, c_float, c_float, c_int, c_int, c_int, V, V, V, V, V], c_int),
        "psfm_bn_act_bwd": ([V, V, V, V, V, V, c_int, c_int, c_int, V, V, V, V, V, V], c_int),
        "psfm_bn_act_resident": ([c_int, c_int], c_int),
        "psfm_bn_act_fused": ([c_int, c_int], c_int),
        "psfm_bn_act_bwd_sum": ([V, V, V, V, V, V, V, V, c_int, c_int, c_int, V, V, V, V, V, V], c_int),
        "psfm_gn_act_fwd": ([V, V, V, c_int, V, V, c_float, c_int, c_int, c_int, c_int, c_int, V, V, V, V, V],
                            c_int),
        "psfm_gn_act_bwd": ([V, V, V, V, c_int, V, V, V, V, c_int, c_int, c_int, c_int, c_int, V, V, V, V, V, V,
                             V], c_int),
        "psfm_netops_last_error": ([], ctypes.c_char_p),
        "psfm_add_relu_fwd": ([V, V, ctypes.c_longlong, V, V], c_int),
        "psfm_relu_mask_bwd": ([V, V, ctypes.c_longlong, V, V], c_int),
        "psfm_relu_mask_bwd_sum": ([V, V, V, V, ctypes.c_longlong, V, V], c_int),
        "psfm_normalize_bf16": ([V, ctypes.c_longlong, c_float, c_float, V, V], c_int),
        "psfm_cat_channels_bf16": ([c_int, V, V, ctypes.c_longlong, V, V], c_int),
        "psfm_relu_maxpool_fwd": ([V, c_int, c_int, c_int, c_int, V, V, V, V], c_int),
        "psfm_relu_maxpool_bwd": ([V, V, V, V, V, c_int, c_int, c_int, c_int, V, V], c_int),
        "psfm_upcat_fwd": ([V, V, c_int, c_int, c_int, c_int, c_int, V, V], c_int),
        "psfm_upcat_bwd": ([V, c_int, c_int, c_int, c_int, c_int, V, V, V], c_int),
        "psfm_upcat_bias_relu_fwd": ([V, V, c_int, V, c_int, c_int, c_int, c_int, c_int, V, V], c_int),
        "psfm_upcat_bias_relu_bwd": ([V, V, c_int, c_int, c_int, c_int, c_int, V, V, V, c_int, V, V], c_int),
        "psfm_upcat_ws_floats": ([c_int, c_int, c_int, c_int], c_size_t),
        # include/psfm_pack3d.h
        "psfm_p3d_fwd": ([V, V, V, V, V, V], c_int),
        "psfm_p3d_ws_floats": ([V], ctypes.c_int64),
        "psfm_p3d_bwd": ([V, V, V, V, V, V, V, V, V], c_int),
        "psfm_p3d_last_error": ([], ctypes.c_char_p),
        # include/psfm_packconv.h
        "psfm_pc_ws_floats": ([V], ctypes.c_int64),
        "psfm_pc_wbuf_bytes": ([V], ctypes.c_int64),
        "psfm_pc_weights_of": ([V, V, V], c_int),
        "psfm_pc_compose": ([V, V, V, V, V, V], c_int),
        "psfm_pc_compose_bwd": ([V, V, V, V, V, V, V, V, V, V, V, V, V], c_int),
        "psfm_pc_fwd": ([V, V, V, V, V, V], c_int),
        "psfm_pc_bwd": ([V, V, V, V, V, V, V, V, V, V, V], c_int),
        "psfm_pc_last_error": ([], ctypes.c_char_p),
        # include/psfm_metrics.h
        "psfm_depth_metrics": ([ctypes.POINTER(MetricsParams), V, V, V, V, V], c_int),
        "psfm_metrics_last_error": ([], ctypes.c_char_p),
        # include/psfm_augment.h
        "psfm_augment_plan": ([ctypes.POINTER(AugmentParams), V], ctypes.c_longlong),
        "psfm_augment_ws_bytes": ([ctypes.POINTER(AugmentParams)], c_size_t),
        "psfm_train_augment": ([ctypes.POINTER(AugmentParams), V, V, V, V, V, V, V], c_int),
        "psfm_gather_frames": ([c_int, V, V, V, V, c_int, c_int, c_int, V, V, V], c_int),
        "psfm_augment_last_error": ([], ctypes.c_char_p),
        # include/psfm_pose.h
        "psfm_pose_from_vec_fwd": ([V, c_int, c_int, V, V], c_int),
        "psfm_pose_from_vec_bwd": ([V, c_int, c_int, V, V, V], c_int),
        "psfm_pinhole_cam_records": ([V, V, V, c_int, c_int, c_int, c_int, c_float, V, V], c_int),
        "psfm_pose_last_error": ([], ctypes.c_char_p),
        # include/psfm_knobs.h
        "psfm_knob_count": ([], c_int),
        "psfm_knob_name": ([c_int], ctypes.c_char_p),
        "psfm_knob_default": ([c_int], c_int),
        "psfm_knob_value": ([c_int], c_int),
        "psfm_knob_set": ([ctypes.c_char_p, c_int], c_int),
        "psfm_knob_rejected": ([c_int], ctypes.c_char_p),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes, fn.restype = args, res
    _lib = L
    return L


EXPORTED = ("psfm_workspace_floats", "psfm_photometric_clip_stats", "psfm_photometric_fwd",
            "psfm_smoothness_fwd", "psfm_finalize", "psfm_photometric_bwd", "psfm_smoothness_bwd",
            "psfm_pose_grad_reduce", "psfm_photometric_prepass", "psfm_photometric_fwd_grad", "psfm_photometric_grad_finish",
            "psfm_pose_grad_reduce_scaled", "psfm_view_synthesis_fwd", "psfm_view_synthesis_bwd",
            "psfm_tiles_per_image", "psfm_last_error", "psfm_version", "psfm_k12_stamps",
            "psfm_optim_plan_chunks", "psfm_grad_pack", "psfm_adam_step", "psfm_optim_last_error",
            "psfm_netops_ws_floats", "psfm_gn_ws_floats", "psfm_bias_act_fwd", "psfm_bias_act_bwd",
            "psfm_bn_act_fwd", "psfm_bn_act_bwd", "psfm_bn_act_resident", "psfm_bn_act_fused", "psfm_gn_act_fwd", "psfm_gn_act_bwd", "psfm_netops_last_error",
            "psfm_add_relu_fwd", "psfm_relu_mask_bwd", "psfm_relu_mask_bwd_sum", "psfm_bias_act_bwd_sum",
            "psfm_bn_act_bwd_sum", "psfm_relu_maxpool_fwd", "psfm_relu_maxpool_bwd",
            "psfm_normalize_bf16", "psfm_cat_channels_bf16",
            "psfm_upcat_fwd", "psfm_upcat_bwd", "psfm_upcat_bias_relu_fwd", "psfm_upcat_bias_relu_bwd",
            "psfm_upcat_ws_floats",
            "psfm_depth_metrics", "psfm_metrics_last_error",
            "psfm_p3d_fwd", "psfm_p3d_ws_floats", "psfm_p3d_bwd", "psfm_p3d_last_error",
            "psfm_pc_ws_floats", "psfm_pc_wbuf_bytes", "psfm_pc_weights_of", "psfm_pc_compose",
            "psfm_pc_compose_bwd", "psfm_pc_fwd", "psfm_pc_bwd", "psfm_pc_last_error",
            "psfm_augment_plan", "psfm_augment_ws_bytes", "psfm_train_augment", "psfm_gather_frames",
            "psfm_augment_last_error",
            "psfm_pose_from_vec_fwd", "psfm_pose_from_vec_bwd", "psfm_pinhole_cam_records", "psfm_pose_last_error",
            "psfm_knob_count", "psfm_knob_name", "psfm_knob_default", "psfm_knob_value", "psfm_knob_set",
            "psfm_knob_rejected")


def knobs():
    """{name: (value, default)} of the library's kernel-selection knobs (include/psfm_knobs.h): read
    once from PSFM_<NAME> when the library loaded, changed only through set_knob."""
    L = lib()
    return {L.psfm_knob_name(i).decode(): (L.psfm_knob_value(i), L.psfm_knob_default(i))
            for i in range(L.psfm_knob_count())}


def nondefault_knobs():
    """The knobs whose value differs from the default ({} on the product configuration), plus
    'rejected:<string>' for every PSFM_<NAME> value the library refused at load."""
    L = lib()
    out = {k: v for k, (v, d) in knobs().items() if v != d}
    for i in range(L.psfm_knob_count()):
        r = L.psfm_knob_rejected(i)
        if r is not None:
            out[L.psfm_knob_name(i).decode()] = "rejected:" + r.decode(errors="replace")
    return out


def set_knob(name, value):
    """Set a knob (A/B tools, tests of a non-default form); returns the previous value."""
    prev = knobs()[name][0]
    if lib().psfm_knob_set(name.encode(), int(value)) != 0:
        raise ValueError(f"knob {name}: value {value} out of range")
    return prev


def check(rc, what):
    if rc != 0:
        if what.startswith(("psfm_optim", "psfm_grad", "psfm_adam")):
            err = lib().psfm_optim_last_error
        elif what.startswith(("psfm_bias_act", "psfm_bn_act", "psfm_gn_act", "psfm_netops", "psfm_upcat",
                              "psfm_add_relu", "psfm_relu_mask")):
            err = lib().psfm_netops_last_error
        elif what.startswith("psfm_depth_metrics"):
            err = lib().psfm_metrics_last_error
        elif what.startswith(("psfm_augment", "psfm_train_augment", "psfm_gather_frames")):
            err = lib().psfm_augment_last_error
        elif what.startswith(("psfm_pose_from_vec", "psfm_pinhole_cam_records")):
            err = lib().psfm_pose_last_error
        elif what.startswith("psfm_p3d"):
            err = lib().psfm_p3d_last_error
        elif what.startswith("psfm_pc_"):
            err = lib().psfm_pc_last_error
        else:
            err = lib().psfm_last_error
        raise RuntimeError(f"{what} failed ({rc}): {err().decode()}")


def require_device(*tensors):
    """The HIP path only runs on ROCm device tensors — no CPU fallback."""
    for t in tensors:
        if t is not None and (not t.is_cuda or t.dtype != torch.float32):
            raise RuntimeError("packnet_sfm_amd photometric path needs float32 tensors on a ROCm "
                               f"(HIP) device; got {t.dtype} on {t.device}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


# HIP-graph captures in progress in this process (any thread: autograd runs CUDA backward nodes on
# its own device threads).  torch.cuda.CUDAGraph.capture_begin / capture_end are wrapped once, at
# import, to count them.
_ACTIVE_CAPTURES = 0
_CAPTURE_STREAMS = []   # the streams the captures in progress began on (innermost last)
_CAPTURE_LOCK = threading.Lock()


def _install_capture_hooks():
    G = torch.cuda.CUDAGraph
    if getattr(G, "_psfm_counted", False):
        return
    begin, end = G.capture_begin, G.capture_end

    def capture_begin(self, *a, **k):
        global _ACTIVE_CAPTURES
        _refuse_stray_backward(torch.cuda.current_stream())
        r = begin(self, *a, **k)
        with _CAPTURE_LOCK:
            _ACTIVE_CAPTURES += 1
            _CAPTURE_STREAMS.append(torch.cuda.current_stream())
        return r

    def capture_end(self, *a, **k):
        global _ACTIVE_CAPTURES
        with _CAPTURE_LOCK:
            _ACTIVE_CAPTURES = max(0, _ACTIVE_CAPTURES - 1)
            if _CAPTURE_STREAMS:
                _CAPTURE_STREAMS.pop()
        return end(self, *a, **k)

    G.capture_begin, G.capture_end, G._psfm_counted = capture_begin, capture_end, True


# Autograd contexts of HIP ops whose forward ran outside any capture and whose backward has not run
# yet (weak: a context leaves the set when its graph is freed).  A capture may not begin on another
# stream while one of them is alive: PyTorch-ROCm runs a node's backward on its forward's stream, so
# capturing that backward makes the capturing stream wait on a stream outside the capture, and HIP
# then segfaults in capture_end — by the time the op's own backward runs, the autograd engine has
# already recorded that wait, so the refusal has to come before the capture exists.
_EAGER_CTX = weakref.WeakSet()


def note_forward(ctx):
    """Called first thing in every HIP op's forward: remember a forward that ran outside any
    capture (with its stream) until its backward runs (capture_guard(ctx))."""
    if not torch.cuda.is_initialized() or torch.cuda.is_current_stream_capturing():
        return
    ctx._psfm_stream = torch.cuda.current_stream().cuda_stream
    with _CAPTURE_LOCK:
        _EAGER_CTX.add(ctx)


def _refuse_stray_backward(cap_stream):
    with _CAPTURE_LOCK:
        stray = [c for c in list(_EAGER_CTX) if getattr(c, "_psfm_stream", None) != cap_stream.cuda_stream]
    if stray:
        names = sorted({type(c).__name__ for c in stray})
        raise RuntimeError(
            f"psfm: refusing to begin a HIP-graph capture on stream {cap_stream.cuda_stream:#x}: {len(stray)} "
            f"HIP op forward(s) ({', '.join(names)}) ran outside any capture on another stream and can still be "
            "backpropagated; a backward captured for them would run on their forward's stream, outside the "
            "capture (HIP segfaults in capture_end).  Run the backward (or free the graph) first, or run the "
            "forward inside the same capture, as DDPTrainer.capture does")


_install_capture_hooks()


def capture_guard(ctx=None):
    """Raise before anything is allocated or launched when this thread is not capturing while a
    HIP-graph capture is in progress — called first thing in every HIP backward: PyTorch-ROCm runs a
    node's backward on its forward's stream, so a backward captured for a forward that ran outside
    the capture would otherwise allocate and launch on a stream the capture does not own, and HIP
    segfaults in capture_end.  `ctx` (the op's autograd context) leaves
    the set of pending eager forwards (note_forward) here.  The capture_begin hook refuses such a
    capture before it starts; this check is the last line for anything it cannot see."""
    if ctx is not None:
        with _CAPTURE_LOCK:
            _EAGER_CTX.discard(ctx)
    if _ACTIVE_CAPTURES and not torch.cuda.is_current_stream_capturing():
        # Refuse — but first join this stream into the capture and straight back (an empty fork), so
        # the capture is still well formed when the error unwinds through torch.cuda.graph: the
        # autograd engine syncs the backward's stream with the caller's (capturing) stream on the way
        # out, and a wait on a stream outside the capture makes HIP's capture_end segfault.
        cur = torch.cuda.current_stream()
        cap = _CAPTURE_STREAMS[-1] if _CAPTURE_STREAMS else None
        if cap is not None and cap.cuda_stream != cur.cuda_stream:
            cur.wait_stream(cap)
            cap.wait_stream(cur)
        raise RuntimeError(
            "psfm: a HIP op would run on a stream outside the HIP-graph capture in progress (stream "
            f"{torch.cuda.current_stream().cuda_stream:#x} is not capturing).  This happens when an op's "
            "backward is captured but its forward ran on another stream (autograd runs the backward on "
            "the forward's stream): run the forward inside the same capture (or on the capture stream), "
            "as DDPTrainer.capture does")


def stream(device):
    """torch's current HIP stream of `device`, for a launch through the C-ABI.  Refuses (Python
    RuntimeError, before anything is launched) to launch on a stream that is NOT capturing while a
    HIP-graph capture is in progress: that is a backward whose forward ran outside the capture
    (PyTorch-ROCm runs a node's backward on its forward's stream) — HIP would otherwise record
    nothing for it and segfault in capture_end."""
    capture_guard()
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def tiles_per_image(H, W):
    return lib().psfm_tiles_per_image(H, W)
