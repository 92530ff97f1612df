/*
 * psfm_pose.h — C-ABI of the pose algebra and camera-record set-up around the photometric loss.
 *
 * Replaces, per training step, the ~100 small ATen launches (sin / cos / stack / bmm / cat and
 * their autograd backward) that sit on the step's critical path between the pose net and the
 * loss kernels:
 *   - Pose.from_vec (reference packnet_sfm/geometry/pose.py:39-46) over pose_vec2mat
 *     (pose_utils.py:41-51) and euler2mat (pose_utils.py:8-37), mode 'euler', for all contexts
 *     of a batch in one launch (psfm_pose_from_vec_fwd), and its gradient w.r.t. the pose vector
 *     (psfm_pose_from_vec_bwd);
 *   - the pinhole camera records the loss kernels read (include/psfm.h, psfm_inputs.cam):
 *     Camera.scaled (camera.py:84-108 -> camera_utils.scale_intrinsics :16-22), Camera.Kinv
 *     (camera.py:72-81) and the target->context transform, for all scales and contexts
 *     (psfm_pinhole_cam_records).
 * All arithmetic is fp32 in the reference's op order (no contraction), whatever autocast state
 * the caller is in.  Conventions as include/psfm.h: device pointers, caller-owned buffers,
 * stream-ordered, return 0 / <0 bad argument / >0 hipError_t, message from psfm_pose_last_error().
 */
#ifndef PSFM_POSE_H
#define PSFM_POSE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSFM_POSE_MAX_CTX 8

/* vec [B][N][6] = (tx, ty, tz, rx, ry, rz) per sample and context (the pose net's output).
 * mats[j] -> [B][4][4]: [R | t] over the row (0, 0, 0, 1), R = Rx(rx) Ry(ry) Rz(rz). */
int psfm_pose_from_vec_fwd(const float* vec, int B, int N, float* const* mats, void* stream);

/* grad_mats[j] -> [B][4][4] dL/dmats[j] (NULL: zero; the bottom row is ignored, it is constant)
 * -> grad_vec [B][N][6]. */
int psfm_pose_from_vec_bwd(const float* vec, int B, int N, const float* const* grad_mats,
                           float* grad_vec, void* stream);

/* cam [S][N][B][PSFM_CAMREC] for the pinhole loss: Kinv of K scaled by `scale` | ref_K scaled by
 * `scale` | T[j][b] rows 0..2 (row-major 3x4, read with a stride of t_stride floats per (j, b):
 * 12 for [N][B][3][4], 16 for [N][B][4][4]) | zeros.  K, ref_K: [B][3][3].  The same record is
 * written for every scale s (one group of equal-size scales). */
int psfm_pinhole_cam_records(const float* K, const float* ref_K, const float* T, int t_stride,
                             int B, int N, int S, float scale, float* cam, void* stream);

const char* psfm_pose_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_POSE_H */
