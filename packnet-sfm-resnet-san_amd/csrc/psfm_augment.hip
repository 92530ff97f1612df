// psfm_augment.hip — training-sample transform on gfx950: crop -> LANCZOS resize -> duplicate
// -> colour jitter -> ToTensor for a whole batch (include/psfm_augment.h).
//
// Byte / integer work, HBM bound: no MFMA.  Three launches per call:
//   k_resize_h  one workgroup per intermediate row: the source row segment is staged in LDS
//               with dword loads (zero fill outside the image = PIL crop), then the horizontal
//               Pillow fixed-point LANCZOS pass writes the uint8 intermediate, planar
//               [img][c][row][W] (only the rows the vertical pass reads, like
//               ImagingResampleInner).
//   k_resize_v  thread per output pixel: vertical pass (coalesced byte rows from L2), writes
//               rgb_original (fp32 = u8 / 255) and, when jittering, the resized uint8 planes
//               plus per-workgroup integer sums of L(prefix ops) — the ImageEnhance.Contrast
//               mean of the image as it is when contrast runs in the shuffled order.
//   k_jitter    thread per pixel: the four ops in the sample's order (exact integer mean from
//               the partial sums), the colour matrix, ToTensor into rgb.
// Every step reproduces Pillow's arithmetic bit for bit (oracle/augment_oracle.c): integer
// MACs with the host-computed coefficients, float32 blends without contraction, the double
// precision HSV conversion, IEEE division for ToTensor.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>
#include <vector>

#include "../../include/psfm_augment.h"

namespace {

constexpr int PREC = 22;  // Resample.c PRECISION_BITS (8-bit images)
constexpr int NT = 256;
constexpr int PLAN_HDR = 8;  // kh, kv, rows_tmp, off_bh, off_ch, off_bv, off_cv, y0
constexpr int MAX_CROP_W = 16384;

thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// ---------------------------------------------------------------------------------------------
// host: Pillow's resample plan (Resample.c precompute_coeffs / normalize_coeffs_8bpc)
// ---------------------------------------------------------------------------------------------
double sinc_filter(double x) {
    if (x == 0.0) return 1.0;
    x = x * M_PI;
    return std::sin(x) / x;
}
double lanczos_filter(double x) {
    if (-3.0 <= x && x < 3.0) return sinc_filter(x) * sinc_filter(x / 3);
    return 0.0;
}

int plan_ksize(int in, int out) {
    if (in == out) return 1;  // no pass in Pillow; the identity plan reproduces the copy
    const double scale = (double)in / out, fs = scale < 1.0 ? 1.0 : scale;
    return (int)std::ceil(3.0 * fs) * 2 + 1;
}

// bounds [out][2] (first tap, count), coeffs [out][ksize]; either may be null
void plan_dir(int in, int out, int32_t* bounds, int32_t* coeffs) {
    const int ks = plan_ksize(in, out);
    if (in == out) {
        for (int i = 0; i < out; ++i) {
            if (bounds) { bounds[2 * i] = i; bounds[2 * i + 1] = 1; }
            if (coeffs) coeffs[i] = 1 << PREC;
        }
        return;
    }
    const double scale = (double)in / out, fs = scale < 1.0 ? 1.0 : scale, support = 3.0 * fs;
    double k[512];
    for (int xx = 0; xx < out; ++xx) {
        const double center = (xx + 0.5) * scale, ss = 1.0 / fs;
        double ww = 0.0;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in) xmax = in;
        xmax -= xmin;
        int x;
        for (x = 0; x < xmax; ++x) {
            const double w = lanczos_filter((x + xmin - center + 0.5) * ss);
            k[x] = w;
            ww += w;
        }
        for (x = 0; x < xmax; ++x)
            if (ww != 0.0) k[x] /= ww;
        for (; x < ks; ++x) k[x] = 0;
        if (coeffs)
            for (x = 0; x < ks; ++x)
                coeffs[xx * ks + x] = k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << PREC))
                                                : (int32_t)(0.5 + k[x] * (1 << PREC));
        if (bounds) { bounds[2 * xx] = xmin; bounds[2 * xx + 1] = xmax; }
    }
}

struct Dims {
    int crop_w, crop_h, kh, kv, y0, rows_tmp;
    long long off_bh, off_ch, off_bv, off_cv, total;
};

int dims(const psfm_augment_params* p, Dims& d) {
    d.crop_w = p->crop_r - p->crop_l;
    d.crop_h = p->crop_b - p->crop_t;
    if (d.crop_w < 1 || d.crop_h < 1) return fail(-2, "empty crop box");
    if (d.crop_w > MAX_CROP_W) return fail(-2, "crop wider than 16384 px");
    if (p->out_h < 1 || p->out_w < 1) return fail(-2, "bad output size");
    if ((double)d.crop_w / p->out_w > 80.0 || (double)d.crop_h / p->out_h > 80.0)
        return fail(-2, "downscale factor above 80 (filter support beyond the plan buffer)");
    d.kh = plan_ksize(d.crop_w, p->out_w);
    d.kv = plan_ksize(d.crop_h, p->out_h);
    int32_t b_first[2], b_last[2];
    // vertical bounds of the first / last output row decide the intermediate's rows
    {
        std::vector<int32_t> bv(2 * (size_t)p->out_h);
        plan_dir(d.crop_h, p->out_h, bv.data(), nullptr);
        b_first[0] = bv[0];
        b_last[0] = bv[2 * (p->out_h - 1)];
        b_last[1] = bv[2 * (p->out_h - 1) + 1];
    }
    (void)b_first[1];
    d.y0 = b_first[0];
    d.rows_tmp = b_last[0] + b_last[1] - d.y0;
    d.off_bh = PLAN_HDR;
    d.off_ch = d.off_bh + 2LL * p->out_w;
    d.off_bv = d.off_ch + (long long)d.kh * p->out_w;
    d.off_cv = d.off_bv + 2LL * p->out_h;
    d.total = d.off_cv + (long long)d.kv * p->out_h;
    return 0;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct WsLayout {
    size_t tmp, resized, part, total;
};
WsLayout ws_layout(const psfm_augment_params* p, const Dims& d) {
    WsLayout w;
    const size_t hw = (size_t)p->out_h * p->out_w;
    const size_t nblk = (hw + NT - 1) / NT;
    w.tmp = 0;
    w.resized = align256((size_t)p->n_img * 3 * d.rows_tmp * p->out_w);
    w.part = w.resized + align256((size_t)p->n_img * 3 * hw);
    w.total = w.part + align256((size_t)p->n_img * nblk * sizeof(uint32_t));
    return w;
}

// ---------------------------------------------------------------------------------------------
// device: Pillow's 8-bit pixel arithmetic
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int clip8_fixed(int32_t v) {
    v >>= PREC;
    return v < 0 ? 0 : v > 255 ? 255 : v;
}

// Blend.c: (UINT8)(in1 + alpha * (in2 - in1)) in float32, clipped (no FMA: x86-64 Pillow)
__device__ __forceinline__ int blend(int a, int b, float alpha) {
#pragma clang fp contract(off)
    const float t = (float)a + alpha * (float)(b - a);
    return t <= 0.0f ? 0 : t >= 255.0f ? 255 : (int)t;
}

__device__ __forceinline__ int rgb2l(int r, int g, int b) {
    return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16;
}
__device__ __forceinline__ int clip8i(int v) { return v <= 0 ? 0 : v >= 255 ? 255 : v; }

// Convert.c rgb2hsv_row -> h += shift (uint8) -> hsv2rgb
__device__ __noinline__ void hue_shift(int& R, int& G, int& B, int shift) {
#pragma clang fp contract(off)
    const int r = R, g = G, b = B;
    const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
    int uh = 0, us = 0;
    const int uv = maxc;
    if (minc != maxc) {
        const float cr = (float)(maxc - minc);
        const float s = cr / (float)maxc;
        const float rc = ((float)(maxc - r)) / cr, gc = ((float)(maxc - g)) / cr, bc = ((float)(maxc - b)) / cr;
        float h;
        if (r == maxc) h = bc - gc;
        else if (g == maxc) h = (float)(2.0 + rc - bc);
        else h = (float)(4.0 + gc - rc);
        h = (float)fmod(((double)h / 6.0 + 1.0), 1.0);
        uh = clip8i((int)((double)h * 255.0));
        us = clip8i((int)((double)s * 255.0));
    }
    const int h = (uh + shift) & 255, s = us, v = uv;
    if (s == 0) {
        R = G = B = v;
        return;
    }
    const int i = (int)floor((double)(float)h * 6.0 / 255.0);
    const float f = (float)((double)(float)h * 6.0 / 255.0 - (double)(float)i);
    const float fs = (float)((double)(float)s / 255.0);
    const int p = clip8i((int)round((double)(float)v * (1.0 - (double)fs)));
    const int q = clip8i((int)round((double)(float)v * (1.0 - (double)(fs * f))));
    const int t = clip8i((int)round((double)(float)v * (1.0 - (double)fs * (1.0 - (double)f))));
    switch (i % 6) {
        case 0: R = v; G = t; B = p; break;
        case 1: R = q; G = v; B = p; break;
        case 2: R = p; G = v; B = t; break;
        case 3: R = p; G = q; B = v; break;
        case 4: R = t; G = p; B = v; break;
        default: R = v; G = p; B = q; break;
    }
}

__device__ __forceinline__ void apply_op(int op, int& r, int& g, int& b, const psfm_jitter& j, int mean) {
    if (op == PSFM_JIT_BRIGHTNESS) {  // ImageEnhance.Brightness: blend(black, img, f)
        r = blend(0, r, j.factor[0]); g = blend(0, g, j.factor[0]); b = blend(0, b, j.factor[0]);
    } else if (op == PSFM_JIT_CONTRAST) {  // ImageEnhance.Contrast: blend(mean L, img, f)
        r = blend(mean, r, j.factor[1]); g = blend(mean, g, j.factor[1]); b = blend(mean, b, j.factor[1]);
    } else if (op == PSFM_JIT_SATURATION) {  // ImageEnhance.Color: blend(L, img, f)
        const int l = rgb2l(r, g, b);
        r = blend(l, r, j.factor[2]); g = blend(l, g, j.factor[2]); b = blend(l, b, j.factor[2]);
    } else {
        hue_shift(r, g, b, j.hue_shift);
    }
}

// Matrix.c ImagingConvertMatrix, diagonal 3x4 matrix: float dot, "+ 0.5" in double, CLIPF
__device__ __forceinline__ int matrix_ch(float m, int u) {
#pragma clang fp contract(off)
    const float v = (float)((double)(m * (float)u) + 0.5);
    return v <= 0.0f ? 0 : v >= 255.0f ? 255 : (int)v;
}

__device__ __forceinline__ float to_float(int u) { return (float)u / 255.0f; }  // ToTensor

struct Geo {
    int n_samples, src_h, src_w, crop_l, crop_t, out_h, out_w, crop_w;
    long long src_stride;
    int kh, kv, y0, rows_tmp, seg0, seg_len;
    int off_bh, off_ch, off_bv, off_cv;
};

// ---------------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) k_resize_h(Geo g, const uint8_t* __restrict__ src,
                                                 const int32_t* __restrict__ plan, uint8_t* __restrict__ tmp) {
    extern __shared__ uint8_t seg[];  // [seg_len * 3] bytes of the source row segment
    const int r = blockIdx.x, img = blockIdx.y, tid = threadIdx.x;
    const int sy = g.crop_t + g.y0 + r;  // source row
    const int nbytes = 3 * g.seg_len;
    const int sx0 = g.crop_l + g.seg0;  // source column of seg[0]
    // bytes [lo, hi) of the segment lie inside the image; the rest is PIL's zero fill
    int lo = 0, hi = 0;
    if (sy >= 0 && sy < g.src_h) {
        lo = 3 * max(0, -sx0);
        hi = 3 * min(g.seg_len, g.src_w - sx0);
        if (hi < lo) hi = lo;
    }
    const uint8_t* row = src + img * g.src_stride + (long long)sy * g.src_w * 3 + 3LL * sx0;
    // dword loads of the aligned words covering [lo, hi) (never outside the containing words)
    const uintptr_t base = (uintptr_t)row;
    const long long w0 = (long long)((base + lo) >> 2);
    const long long w1 = hi > lo ? (long long)((base + hi - 1) >> 2) + 1 : w0;
    for (long long w = w0 + tid; w < w1; w += NT) {
        const uint32_t v = *(const uint32_t*)(uintptr_t)(w << 2);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long long o = (w << 2) + k - (long long)base;
            if (o >= lo && o < hi) seg[o] = (uint8_t)(v >> (8 * k));
        }
    }
    for (int o = tid; o < nbytes; o += NT)
        if (o < lo || o >= hi) seg[o] = 0;
    __syncthreads();
    const int32_t* bh = plan + g.off_bh;
    const int32_t* ch = plan + g.off_ch;
    const size_t plane = (size_t)g.rows_tmp * g.out_w;
    uint8_t* out = tmp + (size_t)img * 3 * plane + (size_t)r * g.out_w;
    for (int x = tid; x < g.out_w; x += NT) {
        const int xmin = bh[2 * x] - g.seg0, xn = bh[2 * x + 1];
        const int32_t* k = ch + (size_t)x * g.kh;
        int32_t s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
        const uint8_t* px = seg + 3 * xmin;
        for (int t = 0; t < xn; ++t) {
            const int32_t c = k[t];
            s0 += px[3 * t] * c;
            s1 += px[3 * t + 1] * c;
            s2 += px[3 * t + 2] * c;
        }
        out[x] = (uint8_t)clip8_fixed(s0);
        out[plane + x] = (uint8_t)clip8_fixed(s1);
        out[2 * plane + x] = (uint8_t)clip8_fixed(s2);
    }
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) red[wv] = v;
    __syncthreads();
    uint32_t s = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < NT / 64; ++i) s += red[i];
    return s;
}

__global__ void __launch_bounds__(NT) k_resize_v(Geo g, const int32_t* __restrict__ plan,
                                                 const uint8_t* __restrict__ tmp, const psfm_jitter* __restrict__ jit,
                                                 float* __restrict__ orig, uint8_t* __restrict__ resized,
                                                 uint32_t* __restrict__ part) {
    __shared__ uint32_t red[NT / 64];
    const int img = blockIdx.y, tid = threadIdx.x;
    const int hw = g.out_h * g.out_w;
    const int pidx = blockIdx.x * NT + tid;
    const bool live = pidx < hw;
    int v[3] = {0, 0, 0};
    if (live) {
        const int y = pidx / g.out_w, x = pidx - y * g.out_w;
        const int ymin = plan[g.off_bv + 2 * y], yn = plan[g.off_bv + 2 * y + 1];
        const int32_t* k = plan + g.off_cv + (size_t)y * g.kv;
        const size_t plane = (size_t)g.rows_tmp * g.out_w;
        const uint8_t* col = tmp + (size_t)img * 3 * plane + (size_t)ymin * g.out_w + x;
        int32_t s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
        for (int t = 0; t < yn; ++t) {
            const int32_t c = k[t];
            const uint8_t* q = col + (size_t)t * g.out_w;
            s0 += q[0] * c;
            s1 += q[plane] * c;
            s2 += q[2 * plane] * c;
        }
        v[0] = clip8_fixed(s0); v[1] = clip8_fixed(s1); v[2] = clip8_fixed(s2);
        float* o = orig + (size_t)img * 3 * hw + pidx;
        o[0] = to_float(v[0]);
        o[hw] = to_float(v[1]);
        o[2 * (size_t)hw] = to_float(v[2]);
    }
    if (!resized) return;  // no jitter requested (uniform)
    if (live) {
        uint8_t* q = resized + (size_t)img * 3 * hw + pidx;
        q[0] = (uint8_t)v[0]; q[hw] = (uint8_t)v[1]; q[2 * (size_t)hw] = (uint8_t)v[2];
    }
    // L of the image as ImageEnhance.Contrast sees it: the ops before contrast applied first
    const psfm_jitter j = jit[img % g.n_samples];
    if (!j.apply) return;  // uniform per workgroup
    uint32_t l = 0;
    if (live) {
        int r = v[0], gg = v[1], b = v[2];
        for (int k = 0; k < 4 && j.order[k] != PSFM_JIT_CONTRAST; ++k) apply_op(j.order[k], r, gg, b, j, 0);
        l = (uint32_t)rgb2l(r, gg, b);
    }
    const uint32_t s = block_sum(l, red);
    if (tid == 0) part[(size_t)img * gridDim.x + blockIdx.x] = s;
}

__global__ void __launch_bounds__(NT) k_jitter(Geo g, const psfm_jitter* __restrict__ jit,
                                               const uint8_t* __restrict__ resized, const uint32_t* __restrict__ part,
                                               float* __restrict__ rgb) {
    __shared__ uint32_t red[NT / 64];
    __shared__ int s_mean;
    const int img = blockIdx.y, tid = threadIdx.x;
    const int hw = g.out_h * g.out_w;
    const int nblk = gridDim.x;
    const psfm_jitter j = jit[img % g.n_samples];
    int mean = 0;
    if (j.apply) {
        // the whole image's L sum (exact integers; each partial <= 256 * 255)
        uint32_t s = 0;
        for (int i = tid; i < nblk; i += NT) s += part[(size_t)img * nblk + i];
        const uint32_t tot = block_sum(s, red);
        if (tid == 0) {
            // int(sum / n + 0.5) == floor((2 sum + n) / 2n) exactly (ImageStat mean, Contrast)
            const unsigned long long n = (unsigned long long)hw;
            s_mean = (int)((2ULL * tot + n) / (2ULL * n));
        }
        __syncthreads();
        mean = s_mean;
    }
    const int pidx = blockIdx.x * NT + tid;
    if (pidx >= hw) return;
    const uint8_t* q = resized + (size_t)img * 3 * hw + pidx;
    int r = q[0], gg = q[hw], b = q[2 * (size_t)hw];
    if (j.apply) {
        for (int k = 0; k < 4; ++k) apply_op(j.order[k], r, gg, b, j, mean);
        if (j.use_matrix) {
            r = matrix_ch(j.matrix[0], r);
            gg = matrix_ch(j.matrix[1], gg);
            b = matrix_ch(j.matrix[2], b);
        }
    }
    float* o = rgb + (size_t)img * 3 * hw + pidx;
    o[0] = to_float(r);
    o[hw] = to_float(gg);
    o[2 * (size_t)hw] = to_float(b);
}

}  // namespace

extern "C" {

long long psfm_augment_plan(const psfm_augment_params* p, int32_t* plan) {
    if (!p) return fail(-1, "null params");
    Dims d;
    if (int e = dims(p, d)) return e;
    if (!plan) return d.total;
    plan[0] = d.kh; plan[1] = d.kv; plan[2] = d.rows_tmp;
    plan[3] = (int32_t)d.off_bh; plan[4] = (int32_t)d.off_ch; plan[5] = (int32_t)d.off_bv;
    plan[6] = (int32_t)d.off_cv; plan[7] = d.y0;
    plan_dir(d.crop_w, p->out_w, plan + d.off_bh, plan + d.off_ch);
    plan_dir(d.crop_h, p->out_h, plan + d.off_bv, plan + d.off_cv);
    // the vertical pass reads the intermediate, which starts at crop row y0
    for (int i = 0; i < p->out_h; ++i) plan[d.off_bv + 2 * i] -= d.y0;
    return d.total;
}

size_t psfm_augment_ws_bytes(const psfm_augment_params* p) {
    if (!p) return 0;
    Dims d;
    if (dims(p, d)) return 0;
    return ws_layout(p, d).total;
}

int psfm_train_augment(const psfm_augment_params* p, const uint8_t* src, const int32_t* plan,
                       const psfm_jitter* jitter, void* ws, float* rgb_original, float* rgb, void* stream) {
    if (!p || !src || !plan || !ws || !rgb_original) return fail(-1, "null augment argument");
    if (rgb && !jitter) return fail(-1, "rgb requested without jitter records");
    if (p->n_samples < 1 || p->n_img < 1 || p->n_img % p->n_samples) return fail(-2, "n_img must be a multiple of n_samples");
    if (p->src_h < 1 || p->src_w < 1 || p->src_stride < 3LL * p->src_h * p->src_w) return fail(-2, "bad source size / stride");
    Dims d;
    if (int e = dims(p, d)) return e;
    if ((long long)p->out_h * p->out_w > (1LL << 28)) return fail(-2, "output too large");
    const WsLayout wl = ws_layout(p, d);
    Geo g;
    g.n_samples = p->n_samples; g.src_h = p->src_h; g.src_w = p->src_w; g.crop_l = p->crop_l; g.crop_t = p->crop_t;
    g.out_h = p->out_h; g.out_w = p->out_w; g.crop_w = d.crop_w; g.src_stride = p->src_stride;
    g.kh = d.kh; g.kv = d.kv; g.y0 = d.y0; g.rows_tmp = d.rows_tmp;
    g.off_bh = (int)d.off_bh; g.off_ch = (int)d.off_ch; g.off_bv = (int)d.off_bv; g.off_cv = (int)d.off_cv;
    // the source columns the horizontal pass reads (host copy of the first / last bounds)
    {
        int32_t b0[2], bl[2];
        std::vector<int32_t> bh(2 * (size_t)p->out_w);
        plan_dir(d.crop_w, p->out_w, bh.data(), nullptr);
        b0[0] = bh[0];
        bl[0] = bh[2 * (p->out_w - 1)];
        bl[1] = bh[2 * (p->out_w - 1) + 1];
        g.seg0 = b0[0];
        g.seg_len = bl[0] + bl[1] - b0[0];
    }
    hipStream_t st = (hipStream_t)stream;
    uint8_t* base = (uint8_t*)ws;
    uint8_t* tmp = base + wl.tmp;
    uint8_t* resized = rgb ? base + wl.resized : nullptr;
    uint32_t* part = (uint32_t*)(base + wl.part);
    const int hw = p->out_h * p->out_w;
    const int nblk = (hw + NT - 1) / NT;
    const size_t lds = (size_t)((3 * g.seg_len + 3) & ~3);
    hipLaunchKernelGGL(k_resize_h, dim3(d.rows_tmp, p->n_img), dim3(NT), lds, st, g, src, plan, tmp);
    hipLaunchKernelGGL(k_resize_v, dim3(nblk, p->n_img), dim3(NT), 0, st, g, plan, (const uint8_t*)tmp, jitter,
                       rgb_original, resized, part);
    if (rgb)
        hipLaunchKernelGGL(k_jitter, dim3(nblk, p->n_img), dim3(NT), 0, st, g, jitter, (const uint8_t*)resized,
                           (const uint32_t*)part, rgb);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail((int)e, std::string("launch: ") + hipGetErrorString(e));
    return 0;
}

const char* psfm_augment_last_error(void) { return g_err.c_str(); }

}  // extern "C"
