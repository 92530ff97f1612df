// psfm_common.h — device helpers shared by the photometric kernels (gfx950 / CDNA4).
//
// Numerics follow the reference op chain exactly where the order of fp32 operations is
// observable at 1e-4 (projection, normalise/unnormalise round trip, bilinear weights,
// SSIM); see DESIGN.md "Numerics".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/psfm.h"

namespace psfm {

// Tile of output pixels owned by one 256-thread workgroup: 64 columns (one wave per row,
// fully coalesced 256-B row segments) x 4 rows.
constexpr int TX = 64;
constexpr int TY = 4;
constexpr int NT = TX * TY;
constexpr int NWAVE = NT / 64;
constexpr int MAXN = PSFM_MAX_CTX;
constexpr int MAXS = PSFM_MAX_SCALES;

__host__ __device__ inline int tiles_x(int W) { return (W + TX - 1) / TX; }
__host__ __device__ inline int tiles_y(int H) { return (H + TY - 1) / TY; }
__host__ __device__ inline int tiles_img(int H, int W) { return tiles_x(W) * tiles_y(H); }

// ReflectionPad2d(1) index map (SSIM :34), clamped so that halo cells that no real output
// reads (partial tiles) still address valid memory.
__device__ __forceinline__ int reflect1(int i, int n) {
    i = i < 0 ? -i : i;
    i = i >= n ? 2 * n - 2 - i : i;
    return min(max(i, 0), n - 1);
}

struct CamRec {
    float Ki[9];  // K^-1 of the target camera at this scale (camera.py:72-81)
    float Kr[9];  // K of the context camera at this scale
    float T[12];  // [R|t] target -> context (pose.py:39-46), row-major 3x4
};

__device__ __forceinline__ void load_cam(const float* __restrict__ p, CamRec& c) {
#pragma unroll
    for (int i = 0; i < 9; ++i) c.Ki[i] = p[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) c.Kr[i] = p[9 + i];
#pragma unroll
    for (int i = 0; i < 12; ++i) c.T[i] = p[18 + i];
}

// Wave-uniform camera record kept in SGPRs (the record address is uniform; readfirstlane
// tells the compiler the values are too, so they leave the VGPR budget).
__device__ __forceinline__ float sgpr(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ void load_cam_uniform(const float* __restrict__ p, CamRec& c) {
#pragma unroll
    for (int i = 0; i < 9; ++i) c.Ki[i] = sgpr(p[i]);
#pragma unroll
    for (int i = 0; i < 9; ++i) c.Kr[i] = sgpr(p[9 + i]);
#pragma unroll
    for (int i = 0; i < 12; ++i) c.T[i] = sgpr(p[18 + i]);
}

// fp32 reciprocal / quotient from v_rcp_f32 (1 ulp) refined by one Newton step, then one
// residual correction of the quotient: the correctly rounded IEEE result except in rare
// double-rounding cases (then 1 ulp), for the finite, normal operands of this path (|b| in
// [1e-8, 1e12]).  3 / +3 VALU instead of the ~10-instruction v_div_scale/fmas/fixup sequence.
__device__ __forceinline__ float rcp_nr(float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
}
__device__ __forceinline__ float div_nr(float a, float b, float rb /* rcp_nr(b) */) {
    const float q = a * rb;
    return __builtin_fmaf(__builtin_fmaf(-q, b, a), rb, q);
}

// sigmoid -> depth (post_process_depth.py:101-106) -> inv (:369) -> warp depth (depth.py:120)
struct DepthChain {
    float lo, rng;
    __device__ __forceinline__ float warp_depth(float s, float& d1, float& inv) const {
        d1 = rcp_nr(lo + rng * s + 1e-8f);
        inv = rcp_nr(d1 + 1e-8f);
        return rcp_nr(fmaxf(inv, 1e-6f));
    }
    // d(warp depth)/ds with torch's reciprocal-backward form (-out^2) at every 1/x
    __device__ __forceinline__ float dwarp_ds(float d, float d1, float inv) const {
        if (!(inv >= 1e-6f)) return 0.0f;  // clamp(min) passes where x >= min
        return -(d * d) * (inv * inv) * (d1 * d1) * rng;
    }
};

// Projection of pixel (u,v) with depth d: X = d K^-1 [u v 1]^T (camera.py:131-139),
// c = R X + t (pose.py:80-86), p = K_ref c (camera.py:165-167), normalised and
// unnormalised as project() + grid_sample(align_corners=True) do (camera.py:172-176).
struct Proj {
    float xn0, xn1, xn2;  // K^-1 [u v 1]
    float X0, X1, X2;     // lifted point
    float p0, p1, p2;     // K_ref (R X + t)
    float z, iz;          // clamp(p2, 1e-5) and its reciprocal
    float ix, iy;         // sampling position in pixels
};

// Lifted ray / point of one pixel (Camera.reconstruct): shared by every context of a target.
struct Lift {
    float xn0, xn1, xn2, X0, X1, X2;
};
__device__ __forceinline__ Lift lift(const float (&Ki)[9], float u, float v, float d) {
    Lift l;
    l.xn0 = Ki[0] * u + Ki[1] * v + Ki[2];
    l.xn1 = Ki[3] * u + Ki[4] * v + Ki[5];
    l.xn2 = Ki[6] * u + Ki[7] * v + Ki[8];
    l.X0 = l.xn0 * d;
    l.X1 = l.xn1 * d;
    l.X2 = l.xn2 * d;
    return l;
}

// Normalise to [-1,1] and back (Camera.project :172-176 then grid_sample's align_corners
// unnormalisation): ((2 (p/z) / (S-1) - 1) + 1) / 2 * (S-1), each rounding kept.
__device__ __forceinline__ float norm_roundtrip(float pz, float sm1, float rsm1 /* rcp_nr(sm1) */) {
    const float n = div_nr(2.0f * pz, sm1, rsm1) - 1.0f;
    return ((n + 1.0f) * 0.5f) * sm1;
}

// Transform + project one lifted point into one context camera (T = [R|t], Kr).
__device__ __forceinline__ void project_lifted(const float (&T)[12], const float (&Kr)[9], const Lift& l,
                                               float wm1, float rwm1, float hm1, float rhm1, Proj& r) {
    r.xn0 = l.xn0; r.xn1 = l.xn1; r.xn2 = l.xn2;
    r.X0 = l.X0; r.X1 = l.X1; r.X2 = l.X2;
    const float c0 = T[0] * r.X0 + T[1] * r.X1 + T[2] * r.X2 + T[3];
    const float c1 = T[4] * r.X0 + T[5] * r.X1 + T[6] * r.X2 + T[7];
    const float c2 = T[8] * r.X0 + T[9] * r.X1 + T[10] * r.X2 + T[11];
    r.p0 = Kr[0] * c0 + Kr[1] * c1 + Kr[2] * c2;
    r.p1 = Kr[3] * c0 + Kr[4] * c1 + Kr[5] * c2;
    r.p2 = Kr[6] * c0 + Kr[7] * c1 + Kr[8] * c2;
    r.z = fmaxf(r.p2, 1e-5f);
    r.iz = rcp_nr(r.z);
    r.ix = norm_roundtrip(div_nr(r.p0, r.z, r.iz), wm1, rwm1);
    r.iy = norm_roundtrip(div_nr(r.p1, r.z, r.iz), hm1, rhm1);
}

__device__ __forceinline__ void project(const CamRec& c, float u, float v, float d, int H, int W,
                                        Proj& r) {
    const float wm1 = (float)(W - 1), hm1 = (float)(H - 1);
    project_lifted(c.T, c.Kr, lift(c.Ki, u, v, d), wm1, rcp_nr(wm1), hm1, rcp_nr(hm1), r);
}

// Bilinear taps of grid_sample(padding_mode='zeros'): per-tap zero when out of bounds.
struct Taps {
    int x0, y0;
    float fx0, fy0;
    bool ok;  // any tap can be in bounds (also guards int conversion of huge coordinates)
};

__device__ __forceinline__ Taps make_taps(float ix, float iy, int H, int W) {
    Taps t;
    // some tap may be in bounds iff ix in [-1, W) (and y alike); the wider open interval
    // also keeps the float->int conversion below well defined (and rejects NaN)
    t.ok = (ix > -2.0f) && (ix < (float)W + 1.0f) && (iy > -2.0f) && (iy < (float)H + 1.0f);
    t.fx0 = floorf(ix);
    t.fy0 = floorf(iy);
    t.x0 = t.ok ? (int)t.fx0 : 0;
    t.y0 = t.ok ? (int)t.fy0 : 0;
    return t;
}

// Load at a 32-bit BYTE offset from a wave-uniform base: lets the compiler use the
// global_load saddr form (SGPR base + VGPR offset), no per-load 64-bit address arithmetic.
__device__ __forceinline__ float ldg(const float* __restrict__ base, uint32_t byte_off) {
    return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + byte_off);
}

// Branch-free tap setup: out-of-bounds taps read a clamped (valid) address and get weight 0,
// so all 12 loads of a bilinear sample issue back to back (no exec-masked branches, one wait) —
// the per-tap zero padding of grid_sample(padding_mode='zeros') is unchanged: tap*0 == 0 for
// the finite images of this path, and the weighted sum starts from 0 as ATen's does.
struct TapAddr {
    uint32_t nw, ne, sw, se;  // BYTE offsets within one channel plane
    bool vnw, vne, vsw, vse;
    bool xw, xe, yn, ys;      // column x0 / x0+1, row y0 / y0+1 in bounds (tap valid = row && column)
    float ax, bx, ay, by;  // (x0+1-ix), (ix-x0), (y0+1-iy), (iy-y0)
};

__device__ __forceinline__ TapAddr tap_addr(float ix, float iy, int H, int W) {
    const Taps t = make_taps(ix, iy, H, W);
    TapAddr a;
    const int x0 = t.x0, y0 = t.y0;
    const bool xw = t.ok && (unsigned)x0 < (unsigned)W, xe = t.ok && (unsigned)(x0 + 1) < (unsigned)W;
    const bool yn = t.ok && (unsigned)y0 < (unsigned)H, ys = t.ok && (unsigned)(y0 + 1) < (unsigned)H;
    const int cx0 = min(max(x0, 0), W - 1), cx1 = min(max(x0 + 1, 0), W - 1);
    const int cy0 = min(max(y0, 0), H - 1), cy1 = min(max(y0 + 1, 0), H - 1);
    a.nw = (uint32_t)(cy0 * W + cx0) * 4u;
    a.ne = a.nw + (uint32_t)(cx1 - cx0) * 4u;
    a.sw = (uint32_t)(cy1 * W + cx0) * 4u;
    a.se = a.sw + (uint32_t)(cx1 - cx0) * 4u;
    a.xw = xw;
    a.xe = xe;
    a.yn = yn;
    a.ys = ys;
    a.vnw = yn && xw;
    a.vne = yn && xe;
    a.vsw = ys && xw;
    a.vse = ys && xe;
    a.ax = (t.fx0 + 1.0f) - ix;
    a.bx = ix - t.fx0;
    a.ay = (t.fy0 + 1.0f) - iy;
    a.by = iy - t.fy0;
    return a;
}

// warped[c] = sum_tap w_tap * img[c](tap)  (ATen grid_sampler_2d bilinear, nw,ne,sw,se order)
__device__ __forceinline__ void bilinear3(const float* __restrict__ img, int H, int W, float ix,
                                          float iy, float out[3]) {
    const TapAddr t = tap_addr(ix, iy, H, W);
    const uint32_t pb = (uint32_t)(H * W) * 4u;
    float v[3][4];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        v[c][0] = ldg(img, c * pb + t.nw);
        v[c][1] = ldg(img, c * pb + t.ne);
        v[c][2] = ldg(img, c * pb + t.sw);
        v[c][3] = ldg(img, c * pb + t.se);
    }
    const float wnw = t.vnw ? t.ax * t.ay : 0.0f, wne = t.vne ? t.bx * t.ay : 0.0f;
    const float wsw = t.vsw ? t.ax * t.by : 0.0f, wse = t.vse ? t.bx * t.by : 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float acc = v[c][0] * wnw;
        acc += v[c][1] * wne;
        acc += v[c][2] * wsw;
        acc += v[c][3] * wse;
        out[c] = acc;
    }
}

// Adjoint of bilinear3 w.r.t. the sampling position (the images carry no gradient:
// they are data).  Returns d/d(ix), d/d(iy).
__device__ __forceinline__ void bilinear3_grad_pos(const float* __restrict__ img, int H, int W,
                                                   float ix, float iy, const float g[3],
                                                   float& gix, float& giy) {
    gix = giy = 0.0f;
    const Taps t = make_taps(ix, iy, H, W);
    if (!t.ok) return;
    const float ixe = t.fx0 + 1.0f, iys = t.fy0 + 1.0f;
    const bool xw = t.x0 >= 0 && t.x0 < W, xe = t.x0 + 1 >= 0 && t.x0 + 1 < W;
    const bool yn = t.y0 >= 0 && t.y0 < H, ys = t.y0 + 1 >= 0 && t.y0 + 1 < H;
    const size_t plane = (size_t)H * W;
    const size_t base = (size_t)t.y0 * W + t.x0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float* p = img + c * plane;
        const float go = g[c];
        if (yn && xw) {
            const float v = p[base];
            gix -= v * (iys - iy) * go;
            giy -= v * (ixe - ix) * go;
        }
        if (yn && xe) {
            const float v = p[base + 1];
            gix += v * (iys - iy) * go;
            giy -= v * (ix - t.fx0) * go;
        }
        if (ys && xw) {
            const float v = p[base + W];
            gix -= v * (iy - t.fy0) * go;
            giy += v * (ixe - ix) * go;
        }
        if (ys && xe) {
            const float v = p[base + W + 1];
            gix += v * (iy - t.fy0) * go;
            giy += v * (ix - t.fx0) * go;
        }
    }
}

// Adjoint of project() for one pixel: from (gix, giy) to dL/dd and dL/dT (12, accumulated).
// Gradient-only arithmetic: 1/z via v_rcp_f32 (the forward values keep IEEE division).
__device__ __forceinline__ float project_grad(const CamRec& c, const Proj& r, float d, float gix,
                                              float giy, int H, int W, float gT[12]) {
    // ix = ((2u/(W-1) - 1 + 1)/2)(W-1) with u = p0/z  ->  d ix/du = 1 (and likewise for v)
    (void)H;
    (void)W;
    const float iz = r.iz;
    const float gu = gix, gv = giy;
    const float gp0 = gu * iz;
    const float gp1 = gv * iz;
    const float gp2 = (r.p2 >= 1e-5f) ? -(gu * r.p0 + gv * r.p1) * (iz * iz) : 0.0f;
    // c = K_ref^-1 p  -> gc = K_ref^T gp
    const float gc0 = c.Kr[0] * gp0 + c.Kr[3] * gp1 + c.Kr[6] * gp2;
    const float gc1 = c.Kr[1] * gp0 + c.Kr[4] * gp1 + c.Kr[7] * gp2;
    const float gc2 = c.Kr[2] * gp0 + c.Kr[5] * gp1 + c.Kr[8] * gp2;
    gT[0] += gc0 * r.X0; gT[1] += gc0 * r.X1; gT[2] += gc0 * r.X2; gT[3] += gc0;
    gT[4] += gc1 * r.X0; gT[5] += gc1 * r.X1; gT[6] += gc1 * r.X2; gT[7] += gc1;
    gT[8] += gc2 * r.X0; gT[9] += gc2 * r.X1; gT[10] += gc2 * r.X2; gT[11] += gc2;
    // X = d xn, c = R X + t -> dL/dd = (R^T gc) . xn
    const float gX0 = c.T[0] * gc0 + c.T[4] * gc1 + c.T[8] * gc2;
    const float gX1 = c.T[1] * gc0 + c.T[5] * gc1 + c.T[9] * gc2;
    const float gX2 = c.T[2] * gc0 + c.T[6] * gc1 + c.T[10] * gc2;
    (void)d;
    return gX0 * r.xn0 + gX1 * r.xn1 + gX2 * r.xn2;
}

// ---- deterministic block reductions (wave butterfly, then waves in fixed order) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Reduces K values per thread over the 256-thread block; result valid in thread 0.
template <int K>
__device__ __forceinline__ void block_sum(float (&v)[K], float* red /* LDS [NWAVE*K] */) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) red[wave * K + k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float s = 0.0f;
            for (int w = 0; w < NWAVE; ++w) s += red[w * K + k];
            v[k] = s;
        }
    }
    __syncthreads();
}

}  // namespace psfm
