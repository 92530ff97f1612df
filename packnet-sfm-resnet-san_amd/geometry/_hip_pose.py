"""Pose.from_vec on HIP (include/psfm_pose.h): all contexts' [B,6] pose vectors -> [B,4,4]
matrices in one launch, and their gradient in one launch -- instead of the ~50 forward and ~60
backward ATen kernels of euler2mat (sin / cos / stack / bmm / cat, pose_utils.py:8-51) on the
training step's critical path.  fp32 whatever the autocast state (the reference's algebra is
fp32; under bf16 autocast the ATen bmm would round the rotations to bf16)."""
import ctypes

import torch

from .. import _hip


class PoseFromVecFn(torch.autograd.Function):
    """vec [B, N, 6] float32 (device) -> N matrices [B, 4, 4] (one per context)."""

    @staticmethod
    def forward(ctx, vec):
        _hip.note_forward(ctx)
        ctx.set_materialize_grads(False)   # an unused context's matrix gets no zero-filled grad
        B, N = vec.shape[0], vec.shape[1]
        mats = [torch.empty(B, 4, 4, device=vec.device, dtype=torch.float32) for _ in range(N)]
        arr = (ctypes.c_void_p * N)(*[m.data_ptr() for m in mats])
        _hip.check(_hip.lib().psfm_pose_from_vec_fwd(_hip.ptr(vec), B, N, arr, _hip.stream(vec.device)),
                   "psfm_pose_from_vec_fwd")
        ctx.save_for_backward(vec)
        return tuple(mats)

    @staticmethod
    def backward(ctx, *grads):
        _hip.capture_guard(ctx)
        vec, = ctx.saved_tensors
        B, N = vec.shape[0], vec.shape[1]
        gs = [None if g is None else g.float().contiguous() for g in grads]
        arr = (ctypes.c_void_p * N)(*[None if g is None else g.data_ptr() for g in gs])
        gv = torch.empty_like(vec)
        _hip.check(_hip.lib().psfm_pose_from_vec_bwd(_hip.ptr(vec), B, N, arr, _hip.ptr(gv),
                                                     _hip.stream(vec.device)), "psfm_pose_from_vec_bwd")
        return gv


def pose_mats_from_vecs(vec):
    """[B, N, 6] -> list of N [B, 4, 4] matrices (Pose.from_vec, mode 'euler', per context)."""
    if vec.shape[1] > _hip.POSE_MAX_CTX:
        raise ValueError(f"at most {_hip.POSE_MAX_CTX} contexts per pose launch")
    return list(PoseFromVecFn.apply(vec.float().contiguous()))
