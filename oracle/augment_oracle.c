/*
 * ORACLE — test infrastructure only (never linked into the product path).
 *
 * Plain-C restatement of the reference's host data path for one training sample
 * (packnet_sfm/datasets/transforms.py:21-50 train_transforms):
 *   crop_sample (augmentations.py:517-540, PIL Image.crop: zero fill outside the image)
 *   -> resize_sample (augmentations.py:103-194: torchvision Resize(LANCZOS) on a PIL image
 *      = Pillow Image.resize(size, LANCZOS))
 *   -> duplicate_sample (augmentations.py:250-275)
 *   -> colorjitter_sample (augmentations.py:277-320 + random_color_jitter_transform :323-370:
 *      torchvision.transforms.functional adjust_brightness / adjust_contrast / adjust_saturation
 *      / adjust_hue on PIL images, in a shuffled order, then the optional Image.convert('RGB',
 *      matrix) colour transform)
 *   -> to_tensor_sample (augmentations.py:202-247: ToTensor = uint8 / 255 as fp32, CHW).
 *
 * The arithmetic lives in third-party code absent from /root/reference: torchvision (absent
 * from this image; its published PIL functional: ImageEnhance.Brightness/Contrast/Color
 * .enhance, and HSV split / uint8 hue shift / merge for hue) and Pillow (present here, 12.2.0;
 * the reference's docker installs pillow-simd, whose SIMD resampler may round differently by
 * 1 LSB).  Restated algorithms (Pillow C sources, by function name):
 *   Resample.c precompute_coeffs + normalize_coeffs_8bpc + ImagingResampleHorizontal_8bpc /
 *     ImagingResampleVertical_8bpc + ImagingResampleInner (horizontal pass first, into a uint8
 *     intermediate holding only the rows the vertical pass reads; PRECISION_BITS = 22)
 *   Blend.c ImagingBlend (float32 alpha; out = (UINT8)(in1 + alpha * (in2 - in1)), clipped)
 *   Convert.c rgb2l (L24 >> 16), rgb2hsv_row, hsv2rgb
 *   ImageStat mean -> int(mean + 0.5) (ImageEnhance.Contrast)
 *   Matrix.c ImagingConvertMatrix (3-band: float dot + 0.5, CLIPF)
 * Pinned against Pillow itself by tests/golden/augment_*.npz (tools/gen_augment_goldens.py runs
 * Pillow in the build container; tests/test_augment_oracle.py).
 *
 * Images are HWC uint8 RGB, row-major, tightly packed (the layout PIL decodes to and
 * np.array(PIL image) returns).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PRECISION_BITS 22

/* the jitter record: same field meaning as psfm_jitter in include/psfm_augment.h */
typedef struct {
    int apply;
    int order[4]; /* 0 brightness, 1 contrast, 2 saturation, 3 hue */
    float factor[3];
    int hue_shift;
    int use_matrix;
    float matrix[3];
} oracle_jitter;

/* Resample.c lanczos_filter / sinc_filter (support 3) */
static double sinc_filter(double x) {
    if (x == 0.0) return 1.0;
    x = x * M_PI;
    return sin(x) / x;
}
static double lanczos_filter(double x) {
    if (-3.0 <= x && x < 3.0) return sinc_filter(x) * sinc_filter(x / 3);
    return 0.0;
}

/* Resample.c precompute_coeffs + normalize_coeffs_8bpc for box (0, in_size).  Returns ksize;
 * bounds [out][2] = (first tap, tap count); coeffs [out][ksize] fixed point (22 bits).  Call with
 * coeffs == NULL to get ksize only. */
int oracle_resample_plan(int in_size, int out_size, int* bounds, int32_t* coeffs) {
    double scale = (double)in_size / out_size, filterscale = scale < 1.0 ? 1.0 : scale;
    double support = 3.0 * filterscale;
    int ksize = (int)ceil(support) * 2 + 1;
    if (!coeffs) return ksize;
    double* k = (double*)malloc(sizeof(double) * ksize);
    for (int xx = 0; xx < out_size; xx++) {
        double center = (xx + 0.5) * scale, ww = 0.0, ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        int x;
        for (x = 0; x < xmax; x++) {
            double w = lanczos_filter((x + xmin - center + 0.5) * ss);
            k[x] = w;
            ww += w;
        }
        for (x = 0; x < xmax; x++)
            if (ww != 0.0) k[x] /= ww;
        for (; x < ksize; x++) k[x] = 0;
        for (x = 0; x < ksize; x++)
            coeffs[xx * ksize + x] = k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << PRECISION_BITS))
                                              : (int32_t)(0.5 + k[x] * (1 << PRECISION_BITS));
        bounds[2 * xx] = xmin;
        bounds[2 * xx + 1] = xmax;
    }
    free(k);
    return ksize;
}

static uint8_t clip8(int32_t v) {
    v >>= PRECISION_BITS;
    return v < 0 ? 0 : v > 255 ? 255 : (uint8_t)v;
}

/* Image.resize((W, H), LANCZOS) of an RGB image (Resample.c ImagingResampleInner). */
void oracle_resize_lanczos(const uint8_t* src, int h, int w, uint8_t* dst, int H, int W) {
    if (h == H && w == W) {
        memcpy(dst, src, (size_t)h * w * 3);
        return;
    }
    int kh = oracle_resample_plan(w, W, NULL, NULL), kv = oracle_resample_plan(h, H, NULL, NULL);
    int* bh = (int*)malloc(sizeof(int) * 2 * W);
    int* bv = (int*)malloc(sizeof(int) * 2 * H);
    int32_t* ch = (int32_t*)malloc(sizeof(int32_t) * W * kh);
    int32_t* cv = (int32_t*)malloc(sizeof(int32_t) * H * kv);
    oracle_resample_plan(w, W, bh, ch);
    oracle_resample_plan(h, H, bv, cv);
    int need_h = W != w, need_v = H != h;
    const uint8_t* in = src;
    int in_rows = h, in_w = w;
    uint8_t* tmp = NULL;
    if (need_h) {
        int y0 = bv[0], y1 = bv[2 * H - 2] + bv[2 * H - 1];
        if (!need_v) { y0 = 0; y1 = h; }
        tmp = (uint8_t*)malloc((size_t)(y1 - y0) * W * 3);
        for (int y = y0; y < y1; y++)
            for (int xx = 0; xx < W; xx++) {
                int xmin = bh[2 * xx], xmax = bh[2 * xx + 1];
                const int32_t* k = ch + xx * kh;
                for (int c = 0; c < 3; c++) {
                    int32_t ss = 1 << (PRECISION_BITS - 1);
                    for (int x = 0; x < xmax; x++) ss += src[((size_t)y * w + x + xmin) * 3 + c] * k[x];
                    tmp[((size_t)(y - y0) * W + xx) * 3 + c] = clip8(ss);
                }
            }
        if (need_v)
            for (int i = 0; i < H; i++) bv[2 * i] -= y0;
        in = tmp;
        in_rows = y1 - y0;
        in_w = W;
    }
    if (need_v) {
        for (int yy = 0; yy < H; yy++) {
            int ymin = bv[2 * yy], ymax = bv[2 * yy + 1];
            const int32_t* k = cv + yy * kv;
            for (int xx = 0; xx < W; xx++)
                for (int c = 0; c < 3; c++) {
                    int32_t ss = 1 << (PRECISION_BITS - 1);
                    for (int y = 0; y < ymax; y++) ss += in[((size_t)(y + ymin) * in_w + xx) * 3 + c] * k[y];
                    dst[((size_t)yy * W + xx) * 3 + c] = clip8(ss);
                }
        }
    } else {
        memcpy(dst, in, (size_t)in_rows * in_w * 3);
    }
    (void)in_rows;
    free(tmp);
    free(bh); free(bv); free(ch); free(cv);
}

/* Blend.c ImagingBlend for one byte (x86-64 float arithmetic, no contraction). */
static uint8_t blend(int a, int b, float alpha) {
    volatile float d = alpha * (float)(b - a);
    float t = (float)a + d;
    if (t <= 0.0f) return 0;
    if (t >= 255.0f) return 255;
    return (uint8_t)t;
}

/* Convert.c rgb2l */
static int rgb2l(int r, int g, int b) { return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16; }

static int clip8i(int v) { return v <= 0 ? 0 : v >= 255 ? 255 : v; }

/* Convert.c rgb2hsv_row */
static void rgb2hsv(const uint8_t* in, uint8_t* out) {
    uint8_t r = in[0], g = in[1], b = in[2];
    uint8_t maxc = r > g ? (r > b ? r : b) : (g > b ? g : b);
    uint8_t minc = r < g ? (r < b ? r : b) : (g < b ? g : b);
    if (minc == maxc) {
        out[0] = 0; out[1] = 0; out[2] = maxc;
        return;
    }
    float cr = (float)(maxc - minc);
    float s = cr / (float)maxc;
    float rc = ((float)(maxc - r)) / cr, gc = ((float)(maxc - g)) / cr, bc = ((float)(maxc - b)) / cr;
    float h;
    if (r == maxc) h = bc - gc;
    else if (g == maxc) h = 2.0 + rc - bc;
    else h = 4.0 + gc - rc;
    h = fmod((h / 6.0 + 1.0), 1.0);
    out[0] = (uint8_t)clip8i((int)(h * 255.0));
    out[1] = (uint8_t)clip8i((int)(s * 255.0));
    out[2] = maxc;
}

/* Convert.c hsv2rgb */
static void hsv2rgb(const uint8_t* in, uint8_t* out) {
    uint8_t h = in[0], s = in[1], v = in[2];
    if (s == 0) {
        out[0] = out[1] = out[2] = v;
        return;
    }
    int i = (int)floor((float)h * 6.0 / 255.0);
    float f = (float)h * 6.0 / 255.0 - (float)i;
    float fs = ((float)s) / 255.0;
    int p = (int)round((float)v * (1.0 - fs));
    int q = (int)round((float)v * (1.0 - fs * f));
    int t = (int)round((float)v * (1.0 - fs * (1.0 - f)));
    uint8_t up = (uint8_t)clip8i(p), uq = (uint8_t)clip8i(q), ut = (uint8_t)clip8i(t);
    switch (i % 6) {
        case 0: out[0] = v; out[1] = ut; out[2] = up; break;
        case 1: out[0] = uq; out[1] = v; out[2] = up; break;
        case 2: out[0] = up; out[1] = v; out[2] = ut; break;
        case 3: out[0] = up; out[1] = uq; out[2] = v; break;
        case 4: out[0] = ut; out[1] = up; out[2] = v; break;
        case 5: out[0] = v; out[1] = up; out[2] = uq; break;
    }
}

/* Matrix.c CLIPF */
static uint8_t clipf(float v) { return v <= 0.0 ? 0 : v >= 255.0f ? 255 : (uint8_t)v; }

/* one adjust_* op over a whole image, in place */
static void apply_op(uint8_t* img, size_t n, int op, const oracle_jitter* j) {
    if (op == 0) { /* ImageEnhance.Brightness: blend(black, img, f) */
        for (size_t i = 0; i < 3 * n; i++) img[i] = blend(0, img[i], j->factor[0]);
    } else if (op == 1) { /* ImageEnhance.Contrast: blend(mean(L), img, f) */
        uint64_t sum = 0;
        for (size_t i = 0; i < n; i++) sum += rgb2l(img[3 * i], img[3 * i + 1], img[3 * i + 2]);
        int mean = (int)((double)sum / (double)n + 0.5);
        for (size_t i = 0; i < 3 * n; i++) img[i] = blend(mean, img[i], j->factor[1]);
    } else if (op == 2) { /* ImageEnhance.Color: blend(L(img), img, f) */
        for (size_t i = 0; i < n; i++) {
            int l = rgb2l(img[3 * i], img[3 * i + 1], img[3 * i + 2]);
            for (int c = 0; c < 3; c++) img[3 * i + c] = blend(l, img[3 * i + c], j->factor[2]);
        }
    } else { /* adjust_hue: HSV, h += shift (uint8 wrap), back to RGB */
        for (size_t i = 0; i < n; i++) {
            uint8_t hsv[3];
            rgb2hsv(img + 3 * i, hsv);
            hsv[0] = (uint8_t)(hsv[0] + j->hue_shift);
            hsv2rgb(hsv, img + 3 * i);
        }
    }
}

/* colorjitter_sample's per-image work (augmentations.py:303-317), in place. */
void oracle_color_jitter(uint8_t* img, int h, int w, const oracle_jitter* j) {
    if (!j->apply) return;
    size_t n = (size_t)h * w;
    for (int k = 0; k < 4; k++) apply_op(img, n, j->order[k], j);
    if (j->use_matrix)
        for (size_t i = 0; i < n; i++)
            for (int c = 0; c < 3; c++) {
                /* diagonal matrix: the zero terms add exact zeros; "+ 0.5" is a double literal */
                float v = (float)((double)(j->matrix[c] * (float)img[3 * i + c]) + 0.5);
                img[3 * i + c] = clipf(v);
            }
}

/* ToTensor: CHW fp32 = uint8 / 255 (torchvision ToTensor on a uint8 array) */
void oracle_to_tensor(const uint8_t* img, int h, int w, float* out) {
    size_t n = (size_t)h * w;
    for (size_t i = 0; i < n; i++)
        for (int c = 0; c < 3; c++) out[c * n + i] = (float)img[3 * i + c] / 255.0f;
}
