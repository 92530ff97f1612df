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

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/psfm_augment.h"

namespace {

constexpr int PREC = 22;  // Resample.c PRECISION_BITS (8-bit images)
constexpr int NT = 256;
constexpr int KM = 16;  // fixed-trip (predicated) tap loops up to KM taps
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

// bounds [out][2] (first tap, count), coeffs [out][ksize] (or [ksize][out] when tap_major: the
// horizontal pass reads one tap of 64 consecutive outputs per wave instruction); either may be null
void plan_dir(int in, int out, int32_t* bounds, int32_t* coeffs, bool tap_major = false) {
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
                coeffs[tap_major ? (size_t)x * out + xx : (size_t)xx * ks + x] = k[x] < 0 ? (int32_t)(-0.5 + k[x] * (1 << PREC))
                                                : (int32_t)(0.5 + k[x] * (1 << PREC));
        if (bounds) { bounds[2 * xx] = xmin; bounds[2 * xx + 1] = xmax; }
    }
}

// Per-byte tables, computed on the host with the reference's expressions (IEEE double / float:
// bit-identical to evaluating them on the device):
//   u2f[u] = u / 255.0f                                   ToTensor
//   i[h] = floor(h * 6.0 / 255.0), f[h] = (float)(h * 6.0 / 255.0 - i), fs[s] = (float)(s / 255.0)
//                                                         Convert.c hsv2rgb
//   rcp[n] = 1.0 / n    (float)(a * rcp[n]) == a / (float)n exactly for 0 <= a <= n <= 255: the
//                       double product is within 2^-52 of a / n, which is either a float or at
//                       least 2^-32 (relative) away from every float rounding boundary
struct Tables {
    double rcp[256];
    float u2f[256], f[256], fs[256];
    int i[256];
};
constexpr int TAB_INTS = (int)(sizeof(Tables) / 4);

void fill_tables(Tables* t) {
    for (int v = 0; v < 256; ++v) {
        const double x = (double)(float)v * 6.0 / 255.0;
        const int i = (int)std::floor(x);
        t->i[v] = i;
        t->f[v] = (float)(x - (double)(float)i);
        t->fs[v] = (float)((double)(float)v / 255.0);
        t->rcp[v] = v ? 1.0 / (double)v : 0.0;
        t->u2f[v] = (float)v / 255.0f;
    }
}

struct Dims {
    int crop_w, crop_h, kh, kv, y0, rows_tmp;
    long long off_bh, off_ch, off_bv, off_cv, off_tab, total;
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
    d.off_tab = (d.off_cv + (long long)d.kv * p->out_h + 3) & ~3LL;  // 16-byte aligned
    d.total = d.off_tab + TAB_INTS;
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
// Taps are pixel (0..255) x coefficient (22-bit signed fixed point): both fit the signed 24-bit
// multiplier (v_mad_i32_i24, full rate), not the quarter-rate v_mul_lo_u32 the compiler picks for
// a plain 32-bit product.
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

// hsv2rgb's per-byte quantities (Convert.c), computed once per workgroup with the reference's
// double expressions: i(h) = floor(h * 6.0 / 255.0), f(h) = (float)(h * 6.0 / 255.0 - i),
// fs(s) = (float)(s / 255.0).
// Copy of the per-byte tables the host appended to the plan (psfm_augment_plan: fill_tables),
// staged in LDS once per workgroup with 16-byte loads.
__device__ __forceinline__ void load_tables(Tables& t, const int32_t* __restrict__ src) {
    const uint4* s4 = (const uint4*)src;
    uint4* d4 = (uint4*)&t;
    for (int k = threadIdx.x; k < (int)(sizeof(Tables) / 16); k += blockDim.x) d4[k] = s4[k];
}

// Convert.c rgb2hsv_row -> h += shift (uint8) -> hsv2rgb
__device__ __forceinline__ void hue_shift(int& R, int& G, int& B, int shift, const Tables& T) {
#pragma clang fp contract(off)
    const int r = R, g = G, b = B;
    const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
    int uh = 0, us = 0;
    const int uv = maxc;
    if (minc != maxc) {
        // The float quotients of small integers a / n (a <= n <= 255) are computed as
        // (float)((double)a * (1.0 / n)): the double product is within 2^-52 of a / n, and a / n
        // is either a float itself or at least 2^-32 (relative) from every float rounding
        // boundary, so the conversion rounds to the IEEE float quotient.  (Exhaustively checked
        // against Pillow over all 2^24 colours, tests/test_augment.py.)
        const int cr = maxc - minc;
        const double rc = T.rcp[cr];
        const float s = (float)((double)cr * T.rcp[maxc]);
        // h = bc - gc (float) | 2.0 + rc - bc | 4.0 + gc - rc (double): one select, one formula
        // ((0.0 + bc) - gc in double is exact, so its float rounding is the float subtraction)
        int base, an, bn;
        if (r == maxc) { base = 0; an = maxc - b; bn = maxc - g; }
        else if (g == maxc) { base = 2; an = maxc - r; bn = maxc - b; }
        else { base = 4; an = maxc - g; bn = maxc - r; }
        const float qa = (float)((double)an * rc), qb = (float)((double)bn * rc);
        float h = (float)(((double)base + (double)qa) - (double)qb);
        // fmod(h / 6.0 + 1.0, 1.0) with h in [-1, 5]: the argument lies in [5/6, 11/6), where
        // fmod is the exact subtraction of 1 (Sterbenz) — no libm loop
        double y = (double)h / 6.0 + 1.0;
        if (y >= 1.0) y -= 1.0;
        h = (float)y;
        uh = clip8i((int)((double)h * 255.0));
        us = clip8i((int)((double)s * 255.0));
    }
    const int h = (uh + shift) & 255, s = us, v = uv;
    if (s == 0) {
        R = G = B = v;
        return;
    }
    const int i = T.i[h];
    const float f = T.f[h], fs = T.fs[s];
    const double dv = (double)(float)v;
    const int p = clip8i((int)round(dv * (1.0 - (double)fs)));
    const int q = clip8i((int)round(dv * (1.0 - (double)(fs * f))));
    const int t = clip8i((int)round(dv * (1.0 - (double)fs * (1.0 - (double)f))));
    switch (i % 6) {
        case 0: R = v; G = t; B = p; break;
        case 1: R = q; G = v; B = p; break;
        case 2: R = p; G = v; B = t; break;
        case 3: R = p; G = q; B = v; break;
        case 4: R = t; G = p; B = v; break;
        default: R = v; G = p; B = q; break;
    }
}

template <int V>
__device__ __forceinline__ void apply_op_v(int op, int (&c)[3][V], const psfm_jitter& j, int mean, const Tables& T) {
    if (op == PSFM_JIT_HUE) {
#pragma unroll
        for (int e = 0; e < V; ++e) hue_shift(c[0][e], c[1][e], c[2][e], j.hue_shift, T);
    } else if (op == PSFM_JIT_SATURATION) {
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const int l = rgb2l(c[0][e], c[1][e], c[2][e]);
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) c[ch][e] = blend(l, c[ch][e], j.factor[2]);
        }
    } else {
        const int a = op == PSFM_JIT_CONTRAST ? mean : 0;
        const float f = op == PSFM_JIT_CONTRAST ? j.factor[1] : j.factor[0];
#pragma unroll
        for (int e = 0; e < V; ++e)
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) c[ch][e] = blend(a, c[ch][e], f);
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
    int off_bh, off_ch, off_bv, off_cv, off_tab;
};

// ---------------------------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------------------------
// One workgroup (a multiple of 64 threads, up to 1024: one output column per thread at KITTI
// width) per intermediate row.
__global__ void __launch_bounds__(1024) k_resize_h(Geo g, const uint8_t* __restrict__ src,
                                                   const int32_t* __restrict__ plan, uint8_t* __restrict__ tmp) {
    extern __shared__ uint8_t seg[];  // [seg_len * 3] bytes of the source row segment
    const int r = blockIdx.x, img = blockIdx.y, tid = threadIdx.x, nt = blockDim.x;
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
    const long long wb = (long long)(base >> 2);  // word holding seg[0] (seg is 4-byte aligned)
    const int shift = (int)(base & 3);
    for (long long w = w0 + tid; w < w1; w += nt) {
        const uint32_t v = *(const uint32_t*)(uintptr_t)(w << 2);
        const long long o0 = ((w - wb) << 2) - shift;  // segment offset of the word's byte 0
        if (o0 >= lo && o0 + 3 < hi) {
            // whole word inside [lo, hi): four byte writes at consecutive LDS addresses
            seg[o0] = (uint8_t)v; seg[o0 + 1] = (uint8_t)(v >> 8);
            seg[o0 + 2] = (uint8_t)(v >> 16); seg[o0 + 3] = (uint8_t)(v >> 24);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const long long o = o0 + k;
                if (o >= lo && o < hi) seg[o] = (uint8_t)(v >> (8 * k));
            }
        }
    }
    for (int o = tid; o < lo; o += nt) seg[o] = 0;
    for (int o = hi + tid; o < nbytes; o += nt) seg[o] = 0;
    __syncthreads();
    const int32_t* bh = plan + g.off_bh;
    const int32_t* ch = plan + g.off_ch;  // [out_w][kh]
    const size_t plane = (size_t)g.rows_tmp * g.out_w;
    uint8_t* out = tmp + (size_t)img * 3 * plane + (size_t)r * g.out_w;
    for (int x = tid; x < g.out_w; x += nt) {
        const int xmin = bh[2 * x] - g.seg0, xn = bh[2 * x + 1];
        int32_t s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
        const uint8_t* px = seg + 3 * xmin;  // byte reads: no unpacking VALU
        const int32_t* k = ch + (size_t)x * g.kh;
#pragma unroll 4
        for (int t = 0; t < xn; ++t) {
            const int32_t c = k[t];
            s0 += __mul24((int)px[3 * t], c);
            s1 += __mul24((int)px[3 * t + 1], c);
            s2 += __mul24((int)px[3 * t + 2], c);
        }
        out[x] = (uint8_t)clip8_fixed(s0);
        out[plane + x] = (uint8_t)clip8_fixed(s1);
        out[2 * plane + x] = (uint8_t)clip8_fixed(s2);
    }
}

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) red[wv] = v;
    __syncthreads();
    T s = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < NT / 64; ++i) s += red[i];
    return s;
}

template <int V> struct Vec;
template <> struct Vec<1> { typedef uint8_t u8; typedef float f32; };
template <> struct Vec<4> { typedef uint32_t u8; typedef float4 f32; };

__device__ __forceinline__ void unpack(uint8_t v, int* o) { o[0] = v; }
__device__ __forceinline__ void unpack(uint32_t v, int* o) {
    o[0] = v & 255; o[1] = (v >> 8) & 255; o[2] = (v >> 16) & 255; o[3] = v >> 24;
}
__device__ __forceinline__ void pack(const int* o, uint8_t& v) { v = (uint8_t)o[0]; }
__device__ __forceinline__ void pack(const int* o, uint32_t& v) {
    v = (uint32_t)o[0] | ((uint32_t)o[1] << 8) | ((uint32_t)o[2] << 16) | ((uint32_t)o[3] << 24);
}
// ToTensor through a 256-entry LDS table of the IEEE quotients u / 255.0f (u * (1/255) is not
// exact for 126 of the 256 bytes)
__device__ __forceinline__ void tofloat(const int* o, float& v, const float* t) { v = t[o[0]]; }
__device__ __forceinline__ void tofloat(const int* o, float4& v, const float* t) {
    v = make_float4(t[o[0]], t[o[1]], t[o[2]], t[o[3]]);
}

// V consecutive output pixels of one row per thread (V = 4 when out_w % 4 == 0: dword byte
// loads, float4 stores).  Vertical pass, rgb_original, and (jittering) the resized bytes + the
// contrast prefix's L sums.
template <int V>
__global__ void __launch_bounds__(NT) k_resize_v(Geo g, const int32_t* __restrict__ plan,
                                                 const uint8_t* __restrict__ tmp, const psfm_jitter* __restrict__ jit,
                                                 float* __restrict__ orig, uint8_t* __restrict__ resized,
                                                 uint32_t* __restrict__ part) {
    typedef typename Vec<V>::u8 U8;
    typedef typename Vec<V>::f32 F32;
    __shared__ uint32_t red[NT / 64];
    __shared__ Tables T;       // hue tables: staged only when hue runs before contrast
    __shared__ float u2f[256];  // ToTensor quotients, computed in place (no memory dependency)
    const int img = blockIdx.y, tid = threadIdx.x;
    const int hw = g.out_h * g.out_w;
    const int pidx = (blockIdx.x * NT + tid) * V;
    const bool live = pidx < hw;
    int v[3][V];
    int32_t s[3][V];
    if (live) {
        const int y = pidx / g.out_w, x = pidx - y * g.out_w;
        const int ymin = plan[g.off_bv + 2 * y], yn = plan[g.off_bv + 2 * y + 1];
        const int32_t* k = plan + g.off_cv + (size_t)y * g.kv;
        const size_t plane = (size_t)g.rows_tmp * g.out_w;
        const uint8_t* col = tmp + (size_t)img * 3 * plane + (size_t)ymin * g.out_w + x;
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int e = 0; e < V; ++e) s[c][e] = 1 << (PREC - 1);
        if (g.kv <= KM) {
            // every tap's loads issued at once (predicated, fixed trip count)
            U8 raw[KM][3];
#pragma unroll
            for (int t = 0; t < KM; ++t)
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    raw[t][c] = t < yn ? *(const U8*)(col + (size_t)t * g.out_w + c * plane) : (U8)0;
#pragma unroll
            for (int t = 0; t < KM; ++t) {
                const int32_t cf = t < yn ? k[t] : 0;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    int u[V];
                    unpack(raw[t][c], u);
#pragma unroll
                    for (int e = 0; e < V; ++e) s[c][e] += __mul24(u[e], cf);
                }
            }
        } else {
            for (int t = 0; t < yn; ++t) {
                const int32_t cf = k[t];
                const uint8_t* q = col + (size_t)t * g.out_w;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    int u[V];
                    unpack(*(const U8*)(q + c * plane), u);
#pragma unroll
                    for (int e = 0; e < V; ++e) s[c][e] += __mul24(u[e], cf);
                }
            }
        }
    }
    for (int u = tid; u < 256; u += NT) u2f[u] = to_float(u);
    __syncthreads();
    if (live) {
        float* o = orig + (size_t)img * 3 * hw + pidx;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
#pragma unroll
            for (int e = 0; e < V; ++e) v[c][e] = clip8_fixed(s[c][e]);
            F32 f;
            tofloat(v[c], f, u2f);
            *(F32*)(o + (size_t)c * hw) = f;
        }
    }
    if (!resized) return;  // no jitter requested (uniform)
    // the ops before contrast (in the sample's shuffled order) run here, once: `resized` holds
    // the image as ImageEnhance.Contrast receives it, and the workgroup's sum of its L values
    const psfm_jitter j = jit[img % g.n_samples];
    bool hue_first = false;
    if (j.apply)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (j.order[k] == PSFM_JIT_CONTRAST) break;
            hue_first |= j.order[k] == PSFM_JIT_HUE;
        }
    if (hue_first) {  // uniform per workgroup
        load_tables(T, plan + g.off_tab);
        __syncthreads();
    }
    uint32_t l = 0;
    if (live) {
        if (j.apply)
            for (int k = 0; k < 4 && j.order[k] != PSFM_JIT_CONTRAST; ++k) apply_op_v<V>(j.order[k], v, j, 0, T);
        uint8_t* q = resized + (size_t)img * 3 * hw + pidx;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            U8 w;
            pack(v[c], w);
            *(U8*)(q + (size_t)c * hw) = w;
        }
#pragma unroll
        for (int e = 0; e < V; ++e) l += (uint32_t)rgb2l(v[0][e], v[1][e], v[2][e]);
    }
    if (!j.apply) return;  // uniform per workgroup
    const uint32_t tot = block_sum(l, red);
    if (tid == 0) part[(size_t)img * gridDim.x + blockIdx.x] = tot;
}

template <int V>
__global__ void __launch_bounds__(NT) k_jitter(Geo g, const int32_t* __restrict__ plan, const psfm_jitter* __restrict__ jit,
                                               const uint8_t* __restrict__ resized, const uint32_t* __restrict__ part,
                                               float* __restrict__ rgb) {
    typedef typename Vec<V>::u8 U8;
    typedef typename Vec<V>::f32 F32;
    __shared__ unsigned long long red[NT / 64];
    __shared__ int s_mean;
    __shared__ Tables T;
    const int img = blockIdx.y, tid = threadIdx.x;
    const int hw = g.out_h * g.out_w;
    const int nblk = gridDim.x;
    const psfm_jitter j = jit[img % g.n_samples];
    load_tables(T, plan + g.off_tab);
    int mean = 0;
    if (j.apply) {
        // the whole image's L sum (exact integers; each partial <= NT * V * 255)
        unsigned long long s = 0;
        for (int i = tid; i < nblk; i += NT) s += part[(size_t)img * nblk + i];
        const unsigned long long tot = block_sum(s, red);
        if (tid == 0) {
            // int(sum / n + 0.5) == floor((2 sum + n) / 2n) exactly (ImageStat mean, Contrast)
            const unsigned long long n = (unsigned long long)hw;
            s_mean = (int)((2ULL * tot + n) / (2ULL * n));
        }
    }
    __syncthreads();  // u2f, hue tables, s_mean
    if (j.apply) mean = s_mean;
    const int pidx = (blockIdx.x * NT + tid) * V;
    if (pidx >= hw) return;
    const uint8_t* q = resized + (size_t)img * 3 * hw + pidx;
    int c3[3][V];
#pragma unroll
    for (int c = 0; c < 3; ++c) unpack(*(const U8*)(q + (size_t)c * hw), c3[c]);
    if (j.apply) {
        // from contrast on: the ops before it already ran in k_resize_v (constant indices only:
        // a dynamically indexed record would live in scratch)
        bool after = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            after |= j.order[k] == PSFM_JIT_CONTRAST;
            if (after) apply_op_v<V>(j.order[k], c3, j, mean, T);
        }
        if (j.use_matrix)
#pragma unroll
            for (int e = 0; e < V; ++e)
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) c3[ch][e] = matrix_ch(j.matrix[ch], c3[ch][e]);
    }
    float* o = rgb + (size_t)img * 3 * hw + pidx;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        F32 f;
        tofloat(c3[c], f, T.u2f);
        *(F32*)(o + (size_t)c * hw) = f;
    }
}

// ------------------------------------------------------------------------------------------
// ResidentLoader batch gather (datasets/synthetic.py; the training-sample batch of one step from
// the HBM-resident dataset): every image store of a batch in ONE launch, written in both layouts the
// step consumes (NCHW for the loss kernels, channels_last for the nets), plus the intrinsics rows —
// instead of an index_select (+ layout copy) per tensor.  Thread = 4 pixels of one (store, image):
// 3 float4 plane loads, 3 float4 NCHW stores, 3 float4 NHWC stores (4 pixels x 3 channels).
// ------------------------------------------------------------------------------------------
struct GatherArgs {
    const float* src[PSFM_GATHER_MAX];
    float* nchw[PSFM_GATHER_MAX];
    float* nhwc[PSFM_GATHER_MAX];
    const int64_t* idx;
    const float* intr_src;
    float* intr_dst;
    int ntensor, B, cams, HW, q;  // q = HW / 4 pixel quads per image
};

__global__ __launch_bounds__(256) void k_gather_frames(GatherArgs a) {
    const int t = blockIdx.y, b = blockIdx.z;
    const int quad = blockIdx.x * blockDim.x + threadIdx.x;
    // row of image b: sample idx[b / cams], camera b % cams (flatten_cameras order)
    const int64_t row = a.idx[b / a.cams] * a.cams + (b % a.cams);
    if (t == 0 && blockIdx.x == 0 && a.intr_dst && threadIdx.x < 9)
        a.intr_dst[(size_t)b * 9 + threadIdx.x] = a.intr_src[(size_t)row * 9 + threadIdx.x];
    if (quad >= a.q) return;
    const float* s = a.src[t] + (size_t)row * 3 * a.HW + (size_t)quad * 4;
    float4 v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = *reinterpret_cast<const float4*>(s + (size_t)c * a.HW);
    if (a.nchw[t]) {
        float* d = a.nchw[t] + (size_t)b * 3 * a.HW + (size_t)quad * 4;
#pragma unroll
        for (int c = 0; c < 3; ++c) *reinterpret_cast<float4*>(d + (size_t)c * a.HW) = v[c];
    }
    if (a.nhwc[t]) {
        float4* d = reinterpret_cast<float4*>(a.nhwc[t] + ((size_t)b * a.HW + (size_t)quad * 4) * 3);
        d[0] = make_float4(v[0].x, v[1].x, v[2].x, v[0].y);
        d[1] = make_float4(v[1].y, v[2].y, v[0].z, v[1].z);
        d[2] = make_float4(v[2].z, v[0].w, v[1].w, v[2].w);
    }
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
    fill_tables((Tables*)(plan + d.off_tab));
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
    g.off_tab = (int)d.off_tab;
    // the source columns the horizontal pass reads (host copy of the first / last bounds)
    {
        std::vector<int32_t> bh(2 * (size_t)p->out_w);
        plan_dir(d.crop_w, p->out_w, bh.data(), nullptr);
        g.seg0 = bh[0];
        g.seg_len = bh[2 * (p->out_w - 1)] + bh[2 * (p->out_w - 1) + 1] - bh[0];
    }
    hipStream_t st = (hipStream_t)stream;
    uint8_t* base = (uint8_t*)ws;
    uint8_t* tmp = base + wl.tmp;
    uint8_t* resized = rgb ? base + wl.resized : nullptr;
    uint32_t* part = (uint32_t*)(base + wl.part);
    const int hw = p->out_h * p->out_w;
    int vec = p->out_w % 4 == 0 ? 4 : 1;  // 4-pixel groups never straddle a row
    const int nblk = (hw / vec + NT - 1) / NT;
    const size_t lds = (size_t)((3 * g.seg_len + 3) & ~3);
    int nth = NT;
    hipLaunchKernelGGL(k_resize_h, dim3(d.rows_tmp, p->n_img), dim3(nth), lds, st, g, src, plan, tmp);
    if (vec == 4) {
        hipLaunchKernelGGL(k_resize_v<4>, dim3(nblk, p->n_img), dim3(NT), 0, st, g, plan, (const uint8_t*)tmp, jitter,
                           rgb_original, resized, part);
        if (rgb)
            hipLaunchKernelGGL(k_jitter<4>, dim3(nblk, p->n_img), dim3(NT), 0, st, g, plan, jitter, (const uint8_t*)resized,
                               (const uint32_t*)part, rgb);
    } else {
        hipLaunchKernelGGL(k_resize_v<1>, dim3(nblk, p->n_img), dim3(NT), 0, st, g, plan, (const uint8_t*)tmp, jitter,
                           rgb_original, resized, part);
        if (rgb)
            hipLaunchKernelGGL(k_jitter<1>, dim3(nblk, p->n_img), dim3(NT), 0, st, g, plan, jitter, (const uint8_t*)resized,
                               (const uint32_t*)part, rgb);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail((int)e, std::string("launch: ") + hipGetErrorString(e));
    return 0;
}

int psfm_gather_frames(int ntensor, const float* const* src, float* const* dst_nchw, float* const* dst_nhwc,
                       const int64_t* idx, int B, int cams, int HW, const float* intr_src, float* intr_dst,
                       void* stream) {
    if (ntensor < 1 || ntensor > PSFM_GATHER_MAX || !src || !dst_nchw || !dst_nhwc || !idx || B < 1 || cams < 1 ||
        HW < 4 || HW % 4 || (!intr_src) != (!intr_dst))
        return fail(-1, "gather_frames: bad arguments (1..PSFM_GATHER_MAX stores, HW a multiple of 4)");
    GatherArgs a{};
    for (int t = 0; t < ntensor; ++t) {
        if (!src[t] || (!dst_nchw[t] && !dst_nhwc[t])) return fail(-1, "gather_frames: null store / destination");
        const uintptr_t al = (uintptr_t)src[t] | (uintptr_t)dst_nchw[t] | (uintptr_t)dst_nhwc[t];
        if (al & 15) return fail(-2, "gather_frames: 16-byte aligned buffers required");
        a.src[t] = src[t], a.nchw[t] = dst_nchw[t], a.nhwc[t] = dst_nhwc[t];
    }
    a.idx = idx, a.intr_src = intr_src, a.intr_dst = intr_dst;
    a.ntensor = ntensor, a.B = B, a.cams = cams, a.HW = HW, a.q = HW / 4;
    const dim3 grid((a.q + 255) / 256, ntensor, B * cams);   // one z per image of the batch
    hipLaunchKernelGGL(k_gather_frames, grid, dim3(256), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail((int)e, hipGetErrorString(e));
    return 0;
}

const char* psfm_augment_last_error(void) { return g_err.c_str(); }

}  // extern "C"
