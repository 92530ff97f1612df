/*
 * psfm_metrics.h — C-ABI of the MI355X (gfx950) depth-evaluation reduction (the Abs Rel gate).
 *
 * Replaces packnet_sfm/utils/depth.py:258-447 compute_depth_metrics(config, gt, pred,
 * use_gt_scale): per image, the valid mask (min_depth < gt < max_depth, optional Garg crop
 * :330-334), ground-truth median scaling (torch.median = the LOWER median of the valid pixels,
 * :380-383), then abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3 (:414-426), averaged over the
 * batch with images that have no valid pixel contributing 0 (:362-365, :446-447).
 * `scale_depth` (:450-483, 'resize' / 'top-center') stays with the caller (an ATen resample).
 *
 * Conventions as include/psfm.h: device pointers, fp32 [B,1,H,W] contiguous, caller-owned
 * buffers, work on `stream`, no host sync, deterministic (exact integer radix-select histograms,
 * fp64 fixed-order sums), 0 / error code + psfm_metrics_last_error().
 */
#ifndef PSFM_METRICS_H
#define PSFM_METRICS_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct psfm_metrics_params {
    int B, H, W;
    float min_depth, max_depth;  /* config.min_depth / config.max_depth (strict bounds on gt) */
    int crop_garg;               /* config.crop == 'garg' */
    int use_gt_scale;            /* ground-truth median scaling */
} psfm_metrics_params;

/* per_image [B][8] = 7 metrics of each image + its valid-pixel count (as float; 0 -> skipped);
 * out [7] = batch average (abs_rel, sq_rel, rmse, rmse_log, a1, a2, a3). */
int psfm_depth_metrics(const psfm_metrics_params* p, const float* gt, const float* pred, float* per_image,
                       float* out, void* stream);

const char* psfm_metrics_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_METRICS_H */
