/*
 * psfm_augment.h — C-ABI of the MI355X (gfx950) training-sample transform (SURVEY §8f row 2:
 * the host data path).
 *
 * Replaces, per batch instead of per sample on CPU DataLoader workers,
 *   packnet_sfm/datasets/transforms.py:21-50   train_transforms(sample, image_shape,
 *                                              jittering, crop_train_borders)
 *     crop_sample            datasets/augmentations.py:517-540 (PIL Image.crop, :373-389)
 *     resize_sample          datasets/augmentations.py:103-194 (torchvision Resize, LANCZOS)
 *     duplicate_sample       datasets/augmentations.py:250-275 (rgb_original = resized copy)
 *     colorjitter_sample     datasets/augmentations.py:277-320 + random_color_jitter_transform
 *                            :323-370 (brightness / contrast / saturation / hue in a shuffled
 *                            order + optional diagonal colour matrix, Image.convert :300-317)
 *     to_tensor_sample       datasets/augmentations.py:202-247 (ToTensor: uint8 / 255, CHW fp32)
 *   packnet_sfm/datasets/transforms.py:52-77   validation_transforms (crop + resize + ToTensor:
 *                                              call with rgb == NULL)
 * Results are bit-identical to Pillow's 8-bit arithmetic (Resample.c fixed-point LANCZOS with a
 * uint8 intermediate, Blend.c float32 blend, Convert.c L / HSV, Matrix.c) — see
 * oracle/augment_oracle.c.  The random draws (factors, shuffled order, colour matrix) stay on
 * the host in Python's `random`, in the reference's draw order; the kernels get them as
 * psfm_jitter records.  PNG decode stays on the host (PIL, datasets/...:load_image).
 *
 * Conventions as include/psfm.h: device pointers, caller-owned buffers, work enqueued on
 * `stream` (hipStream_t), no host synchronisation, no allocation, deterministic (integer
 * contrast sums), 0 / error code + psfm_augment_last_error().
 */
#ifndef PSFM_AUGMENT_H
#define PSFM_AUGMENT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { PSFM_JIT_BRIGHTNESS = 0, PSFM_JIT_CONTRAST = 1, PSFM_JIT_SATURATION = 2, PSFM_JIT_HUE = 3 };

/* One sample's colour jitter (random_color_jitter_transform's fixed parameters). */
typedef struct psfm_jitter {
    int apply;         /* random.random() < prob (augmentations.py:295); 0: rgb = rgb_original */
    int order[4];      /* PSFM_JIT_* in application order (random.shuffle, :368) */
    float factor[3];   /* brightness, contrast, saturation factors, as Image.blend's float32 alpha */
    int hue_shift;     /* uint8 added to H mod 256: np.array(hue_factor * 255).astype(np.uint8) */
    int use_matrix;    /* parameters[4] > 0 (:299-304) */
    float matrix[3];   /* diagonal of the Image.convert('RGB', matrix) transform, float32 */
} psfm_jitter;

typedef struct psfm_augment_params {
    int n_samples;        /* B: image i belongs to sample i % B (its psfm_jitter record) */
    int n_img;            /* B * (1 + contexts); image i = slot i / B (0 rgb, 1.. contexts) */
    int src_h, src_w;     /* decoded image size, shared by every image of the call */
    long long src_stride; /* bytes between consecutive images (>= src_h * src_w * 3) */
    int crop_l, crop_t, crop_r, crop_b; /* PIL crop box (left, top, right, bottom); may exceed
                                           the image (zero fill); the full image = (0,0,w,h) */
    int out_h, out_w;     /* resize target; equal to the crop size = no resize */
} psfm_augment_params;

/* Resample plan (Pillow precompute_coeffs + normalize_coeffs_8bpc for both directions) — host
 * function.  Returns the plan's int32 count (plan == NULL) or fills `plan` (host memory; the
 * caller copies it to the device once per (crop size, output size)). */
long long psfm_augment_plan(const psfm_augment_params* p, int32_t* plan);

/* Device workspace bytes for one call. */
size_t psfm_augment_ws_bytes(const psfm_augment_params* p);

/* src    : device uint8 [n_img] images, each [src_h][src_w][3] (HWC RGB) at i * src_stride
 * plan   : device int32 psfm_augment_plan(p) output
 * jitter : device psfm_jitter [n_samples] (ignored when rgb == NULL)
 * rgb_original : device fp32 [n_img][3][out_h][out_w]  (crop + resize + ToTensor)
 * rgb          : device fp32 [n_img][3][out_h][out_w] or NULL (+ colour jitter) */
int psfm_train_augment(const psfm_augment_params* p, const uint8_t* src, const int32_t* plan,
                       const psfm_jitter* jitter, void* ws, float* rgb_original, float* rgb, void* stream);

/* Batch gather of the HBM-resident training set (the build's DataLoader stand-in,
 * datasets/synthetic.py ResidentLoader.next_into; the reference collates samples on the host,
 * models/model_wrapper.py:1147-1216 DataLoader + trainers/base_trainer.py:8-39 sample_to_cuda).
 * For each of `ntensor` (<= PSFM_GATHER_MAX) fp32 image stores src[t] [n*cams, 3, H, W] (NCHW), image
 * b < B*cams of the batch is row idx[b / cams] * cams + b % cams; it is written to dst_nchw[t]
 * [B*cams, 3, H, W] (NCHW, or NULL) and dst_nhwc[t] (the same tensor in channels_last storage, or
 * NULL).  intr_src [n*cams][3][3] -> intr_dst [B*cams][3][3] the same way (both NULL to skip).
 * idx: device int64 [B].  HW = H*W a multiple of 4, buffers 16-byte aligned.  One launch. */
#define PSFM_GATHER_MAX 4
int psfm_gather_frames(int ntensor, const float* const* src, float* const* dst_nchw, float* const* dst_nhwc,
                       const int64_t* idx, int B, int cams, int HW, const float* intr_src, float* intr_dst,
                       void* stream);

const char* psfm_augment_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_AUGMENT_H */
