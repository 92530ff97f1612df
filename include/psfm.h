/*
 * psfm.h — C-ABI of the MI355X (gfx950) photometric hot path.
 *
 * The reference has no FFI: its hot path is the Python call chain
 *   MultiViewPhotometricLoss.forward        packnet_sfm/losses/multiview_photometric_loss.py:331-410
 *     warp_ref_image / view_synthesis       :131-195, geometry/camera_utils.py:27-59
 *       Camera.reconstruct / project        geometry/camera.py:111-190
 *       grid_sample(bilinear, zeros, align_corners=True)
 *     calc_photometric_loss (SSIM + L1)     :199-267, SSIM :15-54
 *     reduce_photometric_loss ('min'/'mean', automask)  :269-297, :394-399
 *     calc_smoothness_loss                  :301-327, utils/depth.py:146-198
 * plus its autograd backward.  Each entry point below replaces one stage of that
 * chain (cited per function); a Python `torch.autograd.Function` drives them
 * through ctypes.
 *
 * Conventions
 *   - every pointer is DEVICE memory, fp32, NCHW contiguous unless stated; the caller
 *     owns every buffer (no allocation inside); sizes come from psfm_workspace_floats().
 *   - all work is enqueued on `stream`; no host synchronisation, graph-capturable.
 *   - deterministic: no float atomics; every reduction is two-stage in a fixed order.
 *   - return 0 on success, <0 on a bad argument, or a positive hipError_t; the
 *     message is available from psfm_last_error() (thread-local).
 */
#ifndef PSFM_H
#define PSFM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSFM_MAX_CTX 4     /* context frames per target (reference: back+forward context, default 2) */
#define PSFM_MAX_SCALES 4  /* num_scales (default 4, configs/default_config.py:45) */
#define PSFM_CAMREC 32     /* floats per camera record: Kinv[9] | Kref[9] | T[12] | pad[2] */

enum psfm_reduce_op { PSFM_REDUCE_MIN = 0, PSFM_REDUCE_MEAN = 1 };
/* camera model of a call (psfm_params.cam_model): pinhole K (geometry/camera.py:15-190) or the
 * fork's fisheye VADAS model (geometry/camera.py:194-394, dict intrinsics k[7], s, div, ux, uy) */
enum psfm_cam_model { PSFM_CAM_PINHOLE = 0, PSFM_CAM_FISHEYE = 1 };

/* Hyper-parameters of one photometric call: MultiViewPhotometricLoss.__init__ :92-118.
 * One call processes `S` scales that share the image size H x W (the reference's
 * upsample_depth_maps=True case has all num_scales at full resolution in ONE call;
 * multi-resolution scales are issued as one call per scale with S=1). */
typedef struct psfm_params {
    int B, H, W;            /* batch and image size of this call                      */
    int N;                  /* context frames, 1..PSFM_MAX_CTX                         */
    int S;                  /* scales in this call, 1..PSFM_MAX_SCALES                 */
    int scale0;             /* global index of the first scale (smoothness 1/2^i)      */
    int n_scales;           /* n = total scales (ProgressiveScaling, loss_base.py:31)  */
    int automask;           /* automask_loss                                          */
    int reduce_op;          /* psfm_reduce_op                                         */
    int l1_only;            /* ssim_loss_weight == 0 -> 3-channel L1 candidates :246  */
    float ssim_w, C1, C2;   /* ssim_loss_weight, C1, C2                               */
    float min_depth, max_depth;
    float clip_loss;        /* >0: clamp each candidate map at mean+clip*std :249-253 */
    float smooth_w;         /* smooth_loss_weight                                     */
    int grad_fused;         /* 1 when the forward of this call ran through
                               psfm_photometric_fwd_grad (its partial sums use that kernel's
                               unit grid: psfm_finalize / psfm_photometric_grad_finish read it) */
    int cam_model;          /* psfm_cam_model; fisheye: K1 / K12 paths only, N <= 2          */
    int sig_shift[PSFM_MAX_SCALES]; /* sigmoid map s is stored at (H >> k, W >> k), k = sig_shift[s]:
                               the depth net's coarse output, nearest-upsampled to H x W on the
                               fly (models/model_utils.py:152-196 upsample_output; 2^k x 2^k
                               blocks, exact).  0 = stored at H x W.  k > 0: K12 training path
                               (prepass / fwd_grad / grad_finish, grad_sig then at the coarse
                               size) and the K1 forward / clip-stats path; H, W multiples of 2^k */
} psfm_params;

/* Device inputs of one call. `cam` holds one record per (scale, context, batch):
 *   cam[((s*N + j)*B + b)*PSFM_CAMREC + ...] =
 *   pinhole: [0..8] Kinv(3x3, row-major) of the target camera at that scale (camera.py:72-81),
 *            [9..17] Kref(3x3) of the context camera (scaled, camera_utils.py:16-22),
 *   fisheye: [0..3] target s, div, ux, uy; [4..10] context k0..k6; [11..14] context s, div,
 *            ux, uy (centres scaled per scale as (c + 0.5) s - 0.5, :166-186),
 *   both:    [18..29] T = [R|t] (3x4) target->context (pose.py:39-46). */
typedef struct psfm_inputs {
    const float* tgt;                     /* [B,3,H,W] target image at this size           */
    const float* ctx[PSFM_MAX_CTX];       /* N x [B,3,H,W] context images at this size     */
    const float* sig[PSFM_MAX_SCALES];    /* S x [B,1,H,W] sigmoid depth maps               */
    const float* cam;                     /* [S][N][B][PSFM_CAMREC]                          */
    const float* mask;                    /* [B,1,H,W] or NULL (NULL == all ones)           */
} psfm_inputs;

/* Workspace layout (floats), all caller-allocated, sized by psfm_workspace_floats(). */
typedef struct psfm_workspace {
    float* photo_part;   /* [S][B*tiles]            per-tile photometric partial sums      */
    float* smooth_part;  /* [S][B][tiles][4]        per-tile smoothness partial sums       */
    float* clip_part;    /* [S][2N][B*tiles][2]     per-tile sum/sumsq per candidate map   */
    float* clip_thr;     /* [S][2N]                 clip thresholds (written by finalize)  */
    float* pose_part;    /* [S][N][B][tiles][12]    per-tile dL/dT partials                */
    uint8_t* argmin;     /* [S][B][H][W]            selected candidate per pixel ('min')   */
    float* unwarp;       /* [N][B][H][W]            automask: photometric loss of each
                                                    UN-warped context (scale independent)  */
    float* sig_part;     /* [S][B][16]              chunk sums of each sigmoid map (the
                                                    smoothness normaliser, fwd_grad only)  */
    float* cam_pairs;    /* [S][B][48][2]           the camera records of contexts 0 and 1
                                                    interleaved (written by the prepass), with
                                                    M = K_ref R and m = K_ref t appended: K12
                                                    projects both contexts with packed f32
                                                    pairs, one 8-byte scalar load per entry  */
} psfm_workspace;

/* number of floats (and argmin bytes) the workspace of this call needs */
int psfm_workspace_floats(const psfm_params* p, size_t* photo, size_t* smooth, size_t* clip,
                          size_t* clip_thr, size_t* pose, size_t* argmin_bytes, size_t* unwarp,
                          size_t* sig_part, size_t* cam_pairs);

/* Clip statistics pass (only when clip_loss > 0): per-candidate-map sum / sum of squares
 * (calc_photometric_loss :249-253), then thresholds mean + clip*std (unbiased). */
int psfm_photometric_clip_stats(const psfm_params* p, const psfm_inputs* in,
                                const psfm_workspace* ws, void* stream);

/* K1 forward: lift -> transform -> project -> bilinear gather (view_synthesis), SSIM+L1
 * (calc_photometric_loss), automask candidates, min/mean reduction (reduce_photometric_loss).
 * Writes ws->photo_part, (op 'min') ws->argmin and — fused K3 forward — ws->smooth_part when
 * smooth_w > 0 (psfm_smoothness_fwd is then a no-op; it launches only for l1_only calls).
 * With automask it first runs K0, the un-warped candidates into ws->unwarp (skipped when
 * clip_loss > 0: psfm_photometric_clip_stats, which must precede, already produced them). */
int psfm_photometric_fwd(const psfm_params* p, const psfm_inputs* in,
                         const psfm_workspace* ws, void* stream);

/* K3 forward: edge-aware smoothness partial sums (calc_smoothness, calc_smoothness_loss). */
int psfm_smoothness_fwd(const psfm_params* p, const psfm_inputs* in,
                        const psfm_workspace* ws, void* stream);

/* Final deterministic reduction of up to PSFM_MAX_SCALES calls' partials into
 *   out[0] = loss, out[1] = metrics['photometric_loss'], out[2] = metrics['smoothness_loss'],
 * and per-(scale,batch) smoothness stats [n][B][4] for the backward.
 * calls[i] / ws[i] describe the i-th call (scales calls[i]->scale0 ..+S-1). */
int psfm_finalize(int ncalls, const psfm_params* const* calls, const psfm_workspace* const* ws,
                  float* smooth_stats, float* out, void* stream);

/* K2 backward of the photometric term: dL/dsig for the call's S scales (written, not
 * accumulated) and per-tile dL/dT partials.  grad_out: device scalar dL/dloss. */
int psfm_photometric_bwd(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws,
                         const float* grad_out, float* const* grad_sig, void* stream);

/* K3 backward: ADDS the smoothness gradient into grad_sig. */
int psfm_smoothness_bwd(const psfm_params* p, const psfm_inputs* in, const float* smooth_stats,
                        const float* grad_out, float* const* grad_sig, void* stream);

/* Sum the per-tile dL/dT partials of up to PSFM_MAX_SCALES calls into grad_T [N][B][grad_stride]:
 * grad_stride 12 = dL/d[R|t] as [3][4]; 16 = dL/dT of the full [4][4] pose matrix (bottom row 0:
 * the pose's constant row), so the gradient of Pose.mat needs no ATen slice / pad. */
int psfm_pose_grad_reduce(int ncalls, const psfm_params* const* calls,
                          const psfm_workspace* const* ws, float* grad_T, int grad_stride, void* stream);

/* Pre-pass of the K12 training step: K0 (automask candidates, skipped with clip_loss > 0 where
 * psfm_photometric_clip_stats made them) and the per-(scale, image) chunk sums of each sigmoid
 * map into ws->sig_part (the smoothness normaliser K12 needs).  Must precede
 * psfm_photometric_fwd_grad on the same stream. */
int psfm_photometric_prepass(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws,
                             void* stream);

/* K12 — forward AND eager backward in one sweep (training step).  Replaces
 * psfm_photometric_fwd + psfm_photometric_bwd + psfm_smoothness_bwd when the gradient is
 * wanted: the gradient is linear in dL/dloss, so it is produced here for dL/dloss = 1 and
 * scaled by psfm_photometric_grad_finish.  Writes the forward partials (ws->photo_part,
 * ws->smooth_part; finalize as usual, with p->grad_fused = 1), ws->pose_part (dL/dT for
 * dL/dloss = 1) and grad_sig[s] (S planes [B,1,H,W], written once: the photometric gradient
 * plus the per-pixel smoothness gradient).  One kernel; psfm_photometric_prepass first.
 * N <= 2 (the reference's back+forward context); clip_loss > 0 needs
 * psfm_photometric_clip_stats first, as for psfm_photometric_fwd.  Not for l1_only calls. */
int psfm_photometric_fwd_grad(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws,
                              float* const* grad_sig, void* stream);

/* Completes the K12 gradient of one call after psfm_finalize:
 *   grad_sig[s] = grad_out * (grad_k12[s] + c[s][b]),  c = d/ds of the 1/mean(s) normaliser of
 *   the smoothness term (utils/depth.py:183-185; a per-image constant, needs finalize's sums).
 * grad_k12 = the planes psfm_photometric_fwd_grad wrote (read only; grad_sig may alias them).
 * smooth_stats / grad_out as for psfm_smoothness_bwd. */
int psfm_photometric_grad_finish(const psfm_params* p, const float* smooth_stats, const float* grad_out,
                                 const float* const* grad_k12, float* const* grad_sig, void* stream);

/* Pose gradient for the K12 path: grad_T [N][B][grad_stride] = grad_out * sum of the per-unit
 * partials of up to PSFM_MAX_SCALES calls (fixed order, fp64); grad_stride as above. */
int psfm_pose_grad_reduce_scaled(int ncalls, const psfm_params* const* calls,
                                 const psfm_workspace* const* ws, const float* grad_out,
                                 float* grad_T, int grad_stride, void* stream);

/* Standalone view_synthesis (geometry/camera_utils.py:27-59) for one context:
 * warped[B,3,H,W] = grid_sample(ref, project(reconstruct(depth))).  cam: [B][PSFM_CAMREC] records
 * of `cam_model` (psfm_cam_model; layout as psfm_inputs.cam with N = 1). */
int psfm_view_synthesis_fwd(int cam_model, int B, int H, int W, const float* ref, const float* depth,
                            const float* cam, float* warped, void* stream);
/* its backward: dL/ddepth [B,1,H,W] (written) and dL/dT partials [B][tiles][12], reduced into
 * grad_T [B][12] */
int psfm_view_synthesis_bwd(int cam_model, int B, int H, int W, const float* ref, const float* depth,
                            const float* cam, const float* grad_warped, float* grad_depth,
                            float* pose_part, float* grad_T, void* stream);

/* tiles per image used by every kernel for H x W (for sizing pose_part of view synthesis) */
int psfm_tiles_per_image(int H, int W);

const char* psfm_last_error(void);
/* "psfm-gfx950 <ver> src=<16 hex>": the sha256 of the sources the library was built from */
const char* psfm_version(void);

/* Measurement hook (no reference counterpart): when buf != NULL, every later K12 launch
 * (psfm_photometric_fwd_grad) writes each wave's start / end time on the constant 100 MHz clock
 * (s_memrealtime) to buf[2 L], buf[2 L + 1] for workgroup L < capacity; buf = NULL, capacity = 0
 * turns it off.  A device global, so launches inside an already-captured HIP graph are timed in
 * place.  Synchronises `stream`; not for use during capture. */
int psfm_k12_stamps(unsigned long long* buf, int capacity, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_H */
