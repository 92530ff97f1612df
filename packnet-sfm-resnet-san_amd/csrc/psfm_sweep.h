// psfm_sweep.h — v2 photometric kernels: row-sweep with register sliding windows (gfx950).
//
// One wave owns a stripe of 64 consecutive columns (lane = column) of one image and sweeps a band
// of RB output rows top to bottom.  Every row of warped / target values is computed ONCE per
// stripe (no 2-D halo re-warping), the 3x3 SSIM windows come from three rows held in registers
// (vertical) and cross-lane DPP shifts (horizontal: v_add_f32_dpp wave_shr:1 / wave_shl:1), so
// the inner loop has no LDS traffic and (K1) no barriers.  All DPP reads happen with every lane
// active; lane-dependent work only after them.
//
//  K1 (forward, one wave per (stripe, band, batch, scale)): lanes = columns c0-1..c0+62, the 62
//     inner lanes are outputs.  Per row: warp every context (bilinear gathers), load the
//     un-warped contexts and the target; then for the row above: SSIM+L1 of every candidate,
//     clip / mask / min+argmin (or mean), and the edge-aware smoothness terms (fused K3 fwd).
//  K2 (backward, one workgroup = N waves, wave j = context j, per (stripe, band, batch, scale)):
//     lanes = columns c0-2..c0+61, the 60 inner lanes are outputs.  Per row: warp (value and
//     d/dix, d/diy of the bilinear sample); SSIM adjoint coefficients of the row above; the
//     reflect-weighted 3x3 gather of those coefficients for the row two above, then the bilinear
//     and projection adjoint.  The N contexts' dL/dsig of a pixel are summed in context order
//     through a 2-row LDS ring (one barrier per row): deterministic.
// Reference: losses/multiview_photometric_loss.py:15-54, :199-297, :301-327 (see psfm.h).
#pragma once
#include <type_traits>

#include "psfm_camera.h"
#include "psfm_common.h"

namespace psfm {
namespace sweep {

constexpr int K1RB = 13;  // output rows per K1 band (4m+1: 4-slot pipeline)
constexpr int K2RB = 24;  // output rows per K2 band
constexpr int K1W = 62;           // output columns per K1 stripe (halo 1)
constexpr int K2W = 60;           // output columns per K2 stripe (halo 2)

__host__ __device__ inline int k1_stripes(int W) { return (W + K1W - 1) / K1W; }
__host__ __device__ inline int k2_stripes(int W) { return (W + K2W - 1) / K2W; }
__host__ __device__ inline int k1_units(int H, int W) { return k1_stripes(W) * ((H + K1RB - 1) / K1RB); }
__host__ __device__ inline int k2_units(int H, int W) { return k2_stripes(W) * ((H + K2RB - 1) / K2RB); }

// Which (unit, batch, scale) this workgroup sweeps.  Grid = (units, B, S).  The linear block id
// is re-dealt so that the blocks one XCD receives (round-robin dealing: blocks i and i+8 share an
// XCD) form one contiguous run of (b, s, unit) -> one image's context frames stay in that XCD's
// L2 (speed only: any placement is correct).
struct WorkItem {
    int unit, b, s;
};
__device__ __forceinline__ WorkItem work_item() {
    const int units = gridDim.x, B = gridDim.y, S = gridDim.z;
    const int T = units * B * S;
    const int L = blockIdx.x + units * (blockIdx.y + B * blockIdx.z);
    const int xcd = L & 7, i = L >> 3, q = T >> 3, r = T & 7;
    const int w = xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
    const int bs = w / units;
    return WorkItem{w - bs * units, bs / S, bs % S};
}
// The same dealing with each image's units cut into P contiguous parts (bands: unit = band x
// stripes + stripe) and the run ordered (b, part, s, unit): an XCD's run then holds one part of an
// image for ALL scales instead of all units for some scales — the scales share the image's
// target and context frames, and a part's rows are what that XCD's L2 must hold (K12 at 384 x 640:
// one image's three frames are 8.8 MB against a 4 MB L2).  P = 1 is work_item().
__device__ __forceinline__ WorkItem work_item_parts(int P) {
    const int units = gridDim.x, B = gridDim.y, S = gridDim.z;
    const int T = units * B * S;
    const int L = blockIdx.x + units * (blockIdx.y + B * blockIdx.z);
    const int xcd = L & 7, i = L >> 3, q = T >> 3, r = T & 7;
    const int w = xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
    const int per_b = S * units, b = w / per_b, wb = w - b * per_b;
    const int PL = (units + P - 1) / P;            // units per part (the last part may be shorter)
    const int part = wb / (S * PL), rr = wb - part * S * PL;
    const int len = min(PL, units - part * PL);
    const int s = rr / len;
    return WorkItem{part * PL + (rr - s * len), b, s};
}

template <int I>
using Slot = std::integral_constant<int, I>;

// bound_ctrl: the lane without a source reads 0 (no `old` operand to materialise)
__device__ __forceinline__ float from_prev(float v) {  // lane l <- lane l-1 (lane 0 <- 0)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_next(float v) {  // lane l <- lane l+1 (lane 63 <- 0)
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ float hsum3(float v) { return from_prev(v) + v + from_next(v); }

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f); }

template <typename T>
__device__ __forceinline__ T pick4(const T (&a)[4], int i) {
    return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

// bilinear sample (3 channels) and its derivatives w.r.t. the sampling position (grid_sample,
// bilinear, zeros, align_corners=True; same taps / weights as bilinear3, branch-free gathers)
__device__ __forceinline__ void bilinear3_vd(const float* __restrict__ img, int H, int W, float ix, float iy,
                                             float v[3], float dix[3], float diy[3]) {
    const TapAddr t = tap_addr(ix, iy, H, W);
    const uint32_t pb = (uint32_t)(H * W) * 4u;
    float q[3][4];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        q[c][0] = ldg(img, c * pb + t.nw);
        q[c][1] = ldg(img, c * pb + t.ne);
        q[c][2] = ldg(img, c * pb + t.sw);
        q[c][3] = ldg(img, c * pb + t.se);
    }
    const float wnw = t.ax * t.ay, wne = t.bx * t.ay, wsw = t.ax * t.by, wse = t.bx * t.by;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float nw = t.vnw ? q[c][0] : 0.0f, ne = t.vne ? q[c][1] : 0.0f;
        const float sw = t.vsw ? q[c][2] : 0.0f, se = t.vse ? q[c][3] : 0.0f;
        float acc = 0.0f;
        acc += nw * wnw;
        acc += ne * wne;
        acc += sw * wsw;
        acc += se * wse;
        v[c] = acc;
        dix[c] = (ne - nw) * t.ay + (se - sw) * t.by;
        diy[c] = (sw - nw) * t.ax + (se - ne) * t.bx;
    }
}

// Per-channel SSIM terms of one lane from VERTICAL window sums of x, x^2, xy (cross-lane
// horizontal sums taken here -> must be called with all lanes active).  Returns
// mean_c clamp((1-SSIM_c)/2, 0, 1); with GRAD also dSSIM/d(mean x, mean x^2, mean xy) x clamp pass.
template <bool GRAD>
__device__ __forceinline__ float ssim_terms(const float vx[3], const float vxx[3], const float vxy[3],
                                            const float my[3], const float syy[3], float C1, float C2,
                                            float dmx[3], float dsxx[3], float dsxy[3]) {
    // window means as sum * (1/9) and the SSIM quotient via the hardware reciprocal: <= 1-2 ulp
    // from ATen's sum/9 and IEEE division
    constexpr float k9 = 1.0f / 9.0f;
    float ls = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float mx = hsum3(vx[c]) * k9;
        const float sxx = hsum3(vxx[c]) * k9;
        const float sxy = hsum3(vxy[c]) * k9;
        const float mxy = mx * my[c], mx2 = mx * mx, my2 = my[c] * my[c];
        const float A1 = 2.0f * mxy + C1, A2 = 2.0f * (sxy - mxy) + C2;
        const float B1 = mx2 + my2 + C1, B2 = (sxx - mx2) + (syy[c] - my2) + C2;
        const float Nn = A1 * A2, D = B1 * B2;
        const float iD = __builtin_amdgcn_rcpf(D);
        const float l = (1.0f - Nn * iD) * 0.5f;
        ls += fminf(fmaxf(l, 0.0f), 1.0f);
        if (GRAD) {
            const float pass = (l >= 0.0f && l <= 1.0f) ? 1.0f : 0.0f;
            dmx[c] = pass * (2.0f * my[c] * (A2 - A1) * iD - Nn * 2.0f * mx * (B2 - B1) * iD * iD);
            dsxx[c] = pass * (-Nn * B1 * iD * iD);
            dsxy[c] = pass * (2.0f * A1 * iD);
        }
    }
    return ls * (1.0f / 3.0f);
}

__device__ __forceinline__ void target_window(const float (&ya)[3], const float (&yb)[3], const float (&yc)[3],
                                              float my[3], float syy[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        my[c] = hsum3(ya[c] + yb[c] + yc[c]) * (1.0f / 9.0f);
        syy[c] = hsum3(ya[c] * ya[c] + yb[c] * yb[c] + yc[c] * yc[c]) * (1.0f / 9.0f);
    }
}

struct SweepArgs {
    psfm_params p;
    psfm_inputs in;
    psfm_workspace ws;
    const float* grad_out;
    float* grad_sig[PSFM_MAX_SCALES];
};

__device__ __forceinline__ DepthChain depth_chain(const psfm_params& p) {
    return DepthChain{1.0f / fmaxf(p.max_depth, 1e-6f),
                      (float)(1.0 / fmax((double)p.min_depth, 1e-6) - 1.0 / fmax((double)p.max_depth, 1e-6))};
}

// ---------------------------------------------------------------------------------------------
// Packed candidate arithmetic (v3): the contexts of a target are evaluated in PAIRS, one
// context per half of a 64-bit register pair, so every SSIM / L1 / blend operation is one
// v_pk_{add,mul,fma}_f32 for two candidates.  Odd NC: the last pair's high half duplicates
// the last context (computed, never read).
// ---------------------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

// lane l: v[l-1] + v[l] + v[l+1] (lane 0/63 read 0 outside the wave) as two v_add_f32_dpp —
// same association as from_prev(v) + v + from_next(v).  The s_nop covers the VALU-write ->
// DPP-read hazard (the hazard recognizer does not look inside inline asm).  All lanes active.
__device__ __forceinline__ float hsum3a(float v) {
    float t, r;
    asm("s_nop 1\n\t"
        "v_add_f32_dpp %0, %2, %2 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %2, %0 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=&v"(t), "=v"(r)
        : "v"(v));
    return r;
}
__device__ __forceinline__ f2 hsum3p(f2 v) { return f2{hsum3a(v.x), hsum3a(v.y)}; }

// three packed pairs at once: one hazard s_nop for 12 DPP adds
__device__ __forceinline__ void hsum3x3(f2& a, f2& b, f2& c) {
    float t0, t1, t2, t3, t4, t5;
    asm("s_nop 1\n\t"
        "v_add_f32_dpp %0, %6, %6 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %7, %7 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %8, %8 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %3, %9, %9 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %4, %10, %10 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %5, %11, %11 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %0, %6, %0 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %7, %1 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %8, %2 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %3, %9, %3 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %4, %10, %4 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %5, %11, %5 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "=&v"(t5)
        : "v"(a.x), "v"(a.y), "v"(b.x), "v"(b.y), "v"(c.x), "v"(c.y));
    a = f2{t0, t1};
    b = f2{t2, t3};
    c = f2{t4, t5};
}

// 3x3 statistics of the target (shared by every candidate): mean, mean^2, var part.
struct TWin {
    float my[3], my2[3], ty[3];  // ty = E[y^2] - my^2
};
__device__ __forceinline__ TWin target_win(const float (&ya)[3], const float (&yb)[3], const float (&yc)[3]) {
    TWin t;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        t.my[c] = hsum3a(ya[c] + yb[c] + yc[c]) * (1.0f / 9.0f);
        const float syy = hsum3a(ya[c] * ya[c] + yb[c] * yb[c] + yc[c] * yc[c]) * (1.0f / 9.0f);
        t.my2[c] = t.my[c] * t.my[c];
        t.ty[c] = syy - t.my2[c];
    }
    return t;
}

// Photometric candidate of a context pair at the middle row: ssim_w * mean_c clamp((1-SSIM)/2)
// + (1-ssim_w) * mean_c |x-y| (calc_photometric_loss :218-247, SSIM :15-54).  Cross-lane.
__device__ __forceinline__ f2 photo_pair(const f2 (&xa)[3], const f2 (&xb)[3], const f2 (&xc)[3],
                                         const float (&ya)[3], const float (&yb)[3], const float (&yc)[3],
                                         const TWin& tw, float C1, float C2, float ssim_w, float l1w) {
    constexpr float k9 = 1.0f / 9.0f;
    f2 ls = f2{0.0f, 0.0f}, l1 = f2{0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const f2 vx = xa[c] + xb[c] + xc[c];
        const f2 vxx = xa[c] * xa[c] + xb[c] * xb[c] + xc[c] * xc[c];
        const f2 vxy = xa[c] * ya[c] + xb[c] * yb[c] + xc[c] * yc[c];
        f2 hx = vx, hxx = vxx, hxy = vxy;
        hsum3x3(hx, hxx, hxy);
        const f2 mx = hx * k9;
        const f2 sxx = hxx * k9;
        const f2 sxy = hxy * k9;
        const f2 mxy = mx * tw.my[c], mx2 = mx * mx;
        const f2 A1 = 2.0f * mxy + C1, A2 = 2.0f * (sxy - mxy) + C2;
        const f2 B1 = mx2 + tw.my2[c] + C1, B2 = (sxx - mx2) + tw.ty[c] + C2;
        const f2 Nn = A1 * A2, D = B1 * B2;
        const f2 iD = f2{__builtin_amdgcn_rcpf(D.x), __builtin_amdgcn_rcpf(D.y)};
        const f2 l = (1.0f - Nn * iD) * 0.5f;
        ls += f2{__builtin_amdgcn_fmed3f(l.x, 0.0f, 1.0f), __builtin_amdgcn_fmed3f(l.y, 0.0f, 1.0f)};
        const f2 dd = xb[c] - yb[c];
        l1 += f2{fabsf(dd.x), fabsf(dd.y)};
    }
    return ssim_w * (ls * (1.0f / 3.0f)) + l1w * (l1 * (1.0f / 3.0f));
}

// Loss configuration: FAST = the reference default (automask, 'min', smoothness on, no clip,
// no mask) as compile-time constants; otherwise read from psfm_params.
template <bool FAST>
struct Cfg {
    const psfm_params& p;
    __device__ __forceinline__ bool automask() const { return FAST ? true : (bool)p.automask; }
    __device__ __forceinline__ bool is_min() const { return FAST ? true : p.reduce_op == PSFM_REDUCE_MIN; }
    __device__ __forceinline__ bool smooth() const { return FAST ? true : p.smooth_w > 0.0f; }
    __device__ __forceinline__ bool clip() const { return FAST ? false : p.clip_loss > 0.0f; }
};

// ---------------------------------------------------------------------------------------------
// K0: automask candidates — photometric loss of every UN-warped context against the target
// (multiview_photometric_loss.py:394-399).  Scale independent at full resolution, so computed
// once per call instead of once per scale.  One wave per (62-col stripe, K0RB-row band,
// batch): all K0RB+2 rows are loaded up front (independent loads, no sweep latency chain).
// ---------------------------------------------------------------------------------------------
constexpr int K0RB = 4;
__host__ __device__ inline int k0_units(int H, int W) { return k1_stripes(W) * ((H + K0RB - 1) / K0RB); }

template <int NC>
__global__ __launch_bounds__(64) void k0_unwarped(SweepArgs a) {
    constexpr int NP = (NC + 1) / 2;
    const psfm_params& p = a.p;
    const int H = p.H, W = p.W, B = p.B;
    const uint32_t plane = (uint32_t)(H * W);
    const WorkItem wi = work_item();
    const int nst = k1_stripes(W), b = wi.b;
    const int y0 = (wi.unit / nst) * K0RB;
    const int col = (wi.unit % nst) * K1W - 1 + (int)threadIdx.x;
    const int colr = reflect1(col, W);
    const bool pcol = threadIdx.x >= 1 && threadIdx.x <= K1W && col < W;
    const float l1w = 1.0f - p.ssim_w;
    const float* tgt = a.in.tgt + (size_t)b * 3 * plane;
    float Y[K0RB + 2][3];
    f2 X[K0RB + 2][NP][3];
#pragma unroll
    for (int k = 0; k < K0RB + 2; ++k) {
        const uint32_t pix = (uint32_t)(reflect1(y0 - 1 + k, H) * W + colr);
#pragma unroll
        for (int c = 0; c < 3; ++c) Y[k][c] = tgt[c * plane + pix];
#pragma unroll
        for (int j = 0; j < 2 * NP; ++j) {
            const int jj = j < NC ? j : NC - 1;
#pragma unroll
            for (int c = 0; c < 3; ++c) X[k][j >> 1][c][j & 1] = pick4(a.in.ctx, jj)[(size_t)b * 3 * plane + c * plane + pix];
        }
    }
#pragma unroll
    for (int k = 1; k <= K0RB; ++k) {
        const int pv = y0 - 1 + k;
        if (pv >= H) break;  // wave-uniform
        const TWin tw = target_win(Y[k - 1], Y[k], Y[k + 1]);
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const f2 v = photo_pair(X[k - 1][q], X[k][q], X[k + 1][q], Y[k - 1], Y[k], Y[k + 1], tw, p.C1, p.C2,
                                    p.ssim_w, l1w);
            if (pcol) {
                float* o = a.ws.unwarp + ((size_t)(2 * q) * B + b) * plane + (uint32_t)(pv * W + col);
                o[0] = v.x;
                if (2 * q + 1 < NC) o[(size_t)B * plane] = v.y;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K1: forward (+ fused smoothness forward).  NC = number of contexts (exact register arrays).
// STATS: clip-statistics pass (sum / sumsq of every raw candidate map, :249-253).
//
// Software pipeline over four row slots: step k issues row v = y0-1+k (target loads, the
// bilinear gathers of every context — using the sigmoid prefetched one step earlier — and the
// sigmoid of row v+1), then evaluates output row v-2 from rows v-3..v-1 that landed during the
// previous step.  The gathers of row v stay in flight under a full row of SSIM arithmetic.
// ---------------------------------------------------------------------------------------------
template <int NC>
struct K1State {
    static constexpr int NP = (NC + 1) / 2;
    float Y[4][3], SG[4];
    f2 X[4][NP][3];
    float sg_next;
    float acc_photo, acc_ax, acc_ay, acc_m;
    float st[2 * NC][2];
};

template <int NC, bool STATS, bool FAST, int MODEL>
struct K1 {
    static constexpr int NP = (NC + 1) / 2;
    const SweepArgs& a;
    const psfm_params& p;
    Cfg<FAST> cfg;
    int H, W, b, s, unit, y0, col, colr, B;
    int sh, Ws, colc;  // sigmoid storage: (H >> sh, W >> sh) (psfm_params.sig_shift)
    uint32_t plane;
    bool pcol;
    DepthChain dc;
    float l1w;
    const float* tgt;
    const float* sig;
    const float* ctx[NC];
    const float* thr;
    Cams<NC, MODEL> cams;

    __device__ __forceinline__ K1(const SweepArgs& a_) : a(a_), p(a_.p), cfg{a_.p} {
        H = p.H;
        W = p.W;
        B = p.B;
        plane = (uint32_t)(H * W);
        const int nst = k1_stripes(W);
        const WorkItem wi = work_item();
        b = wi.b;
        s = wi.s;
        unit = wi.unit;
        y0 = (unit / nst) * K1RB;
        col = (unit % nst) * K1W - 1 + (int)threadIdx.x;
        colr = reflect1(col, W);
        pcol = threadIdx.x >= 1 && threadIdx.x <= K1W && col < W;
        dc = depth_chain(p);
        l1w = 1.0f - p.ssim_w;
        tgt = a.in.tgt + (size_t)b * 3 * plane;
        sh = pick4(p.sig_shift, s);
        Ws = W >> sh;
        colc = colr >> sh;
        sig = pick4(a.in.sig, s) + (size_t)b * (plane >> (2 * sh));
#pragma unroll
        for (int j = 0; j < NC; ++j) ctx[j] = pick4(a.in.ctx, j) + (size_t)b * 3 * plane;
        cams.load(as_const(a.in.cam + ((size_t)s * NC * B + b) * PSFM_CAMREC), B, H, W);
        thr = (cfg.clip() && !STATS) ? a.ws.clip_thr + (size_t)s * (cfg.automask() ? 2 * NC : NC) : nullptr;
    }

    __device__ __forceinline__ float load_sig(int v) const {  // nearest 2^sh upsampling (K12 load_sig)
        return sig[(uint32_t)((reflect1(v, H) >> sh) * Ws + colc)];
    }

    // issue row v: target, warped contexts (from the prefetched sigmoid sg)
    __device__ __forceinline__ void issue_row(int v, float sg, float (&y)[3], f2 (&x)[NP][3]) const {
        const int r = reflect1(v, H);
        const uint32_t pix = (uint32_t)(r * W + colr);
#pragma unroll
        for (int c = 0; c < 3; ++c) y[c] = tgt[c * plane + pix];
        float d1, inv;
        const float d = dc.warp_depth(sg, d1, inv);
        const Lift l = cams.lift((float)colr, (float)r, d);
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            typename Cams<NC, MODEL>::P pr;
            cams.project(j, l, pr);
            float w[3];
            bilinear3(ctx[j], H, W, pr.ix, pr.iy, w);
#pragma unroll
            for (int c = 0; c < 3; ++c) x[j >> 1][c][j & 1] = w[c];
        }
        if (NC & 1) {
#pragma unroll
            for (int c = 0; c < 3; ++c) x[NP - 1][c].y = x[NP - 1][c].x;
        }
    }

    // step k with slot I: issue row v = y0-1+k into slot I (LOAD), evaluate output row v-2
    // from slots I+1 (row v-3), I+2 (v-2), I+3 (v-1) mod 4 (EVAL)
    template <int I, bool LOAD, bool EVAL>
    __device__ __forceinline__ void step(K1State<NC>& S, int k) const {
        constexpr int IA = (I + 1) & 3, IB = (I + 2) & 3, IC = (I + 3) & 3;
        const int v = y0 - 1 + k;
        if (LOAD) {
            const float sg = S.sg_next;
            S.sg_next = load_sig(v + 1);
            S.SG[I] = sg;
            issue_row(v, sg, S.Y[I], S.X[I]);
        }
        if (EVAL) eval<IA, IB, IC>(S, v - 2);
    }

    // output row pv from slots IA (pv-1), IB (pv), IC (pv+1)
    template <int IA, int IB, int IC>
    __device__ __forceinline__ void eval(K1State<NC>& S, int pv) const {
        if (pv >= H) return;  // wave-uniform (partial last band)
        // ---- cross-lane phase (every lane active) ----
        const TWin tw = target_win(S.Y[IA], S.Y[IB], S.Y[IC]);
        float cand[2 * NC];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const f2 v = photo_pair(S.X[IA][q], S.X[IB][q], S.X[IC][q], S.Y[IA], S.Y[IB], S.Y[IC], tw, p.C1, p.C2,
                                    p.ssim_w, l1w);
            cand[4 * q] = v.x;
            if (2 * q + 1 < NC) cand[4 * q + 2] = v.y;
        }
        float sgn_next = 0.0f, ynext[3] = {0.0f, 0.0f, 0.0f};
        if (!STATS && cfg.smooth()) {
            sgn_next = from_next(S.SG[IB]);
#pragma unroll
            for (int c = 0; c < 3; ++c) ynext[c] = from_next(S.Y[IB][c]);
        }
        // ---- lane-local phase ----
        if (!pcol) return;
        const uint32_t ppix = (uint32_t)(pv * W + col);
        if (cfg.automask()) {  // un-warped candidates (K0, scale independent)
#pragma unroll
            for (int j = 0; j < NC; ++j) cand[2 * j + 1] = a.ws.unwarp[((size_t)j * B + b) * plane + ppix];
        }
        if (STATS) {
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const int sw = cfg.automask() ? 2 * j : j;
                S.st[sw][0] += cand[2 * j];
                S.st[sw][1] += cand[2 * j] * cand[2 * j];
                if (cfg.automask()) {
                    S.st[sw + 1][0] += cand[2 * j + 1];
                    S.st[sw + 1][1] += cand[2 * j + 1] * cand[2 * j + 1];
                }
            }
            return;
        }
        const float mval = (!FAST && a.in.mask) ? a.in.mask[(size_t)b * plane + ppix] : 1.0f;
        float best = INFINITY, sum = 0.0f;
        int arg = 0, kk = 0;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (u == 1 && !cfg.automask()) break;
                float val = cand[2 * j + u];
                if (!FAST) {
                    if (thr) val = fminf(val, thr[u ? 2 * j + 1 : (cfg.automask() ? 2 * j : j)]);
                    val *= mval;
                }
                sum += val;
                if (val < best) {
                    best = val;
                    arg = kk;
                }
                ++kk;
            }
        }
        if (cfg.is_min()) {
            S.acc_photo += best;
            a.ws.argmin[((size_t)s * B + b) * plane + ppix] = (uint8_t)arg;
        } else {
            S.acc_photo += sum;
        }
        if (cfg.smooth()) {  // edge-aware smoothness of the sigmoid map (utils/depth.py:165-198)
            const float sc = S.SG[IB];
            S.acc_m += sc;
            if (col < W - 1) {
                const float m = (fabsf(S.Y[IB][0] - ynext[0]) + fabsf(S.Y[IB][1] - ynext[1]) +
                                 fabsf(S.Y[IB][2] - ynext[2])) * (1.0f / 3.0f);
                S.acc_ax += fabsf(sc - sgn_next) * expf(-m);
            }
            if (pv < H - 1) {
                const float m = (fabsf(S.Y[IB][0] - S.Y[IC][0]) + fabsf(S.Y[IB][1] - S.Y[IC][1]) +
                                 fabsf(S.Y[IB][2] - S.Y[IC][2])) * (1.0f / 3.0f);
                S.acc_ay += fabsf(sc - S.SG[IC]) * expf(-m);
            }
        }
    }
};

template <int NC, bool STATS, bool FAST, int MODEL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void k1_forward(SweepArgs a) {
    static_assert((K1RB - 1) % 4 == 0, "K1 band height must be 4m+1 (4-slot pipeline)");
    K1<NC, STATS, FAST, MODEL> K(a);
    K1State<NC> S;
    S.acc_photo = S.acc_ax = S.acc_ay = S.acc_m = 0.0f;
#pragma unroll
    for (int k = 0; k < 2 * NC; ++k) S.st[k][0] = S.st[k][1] = 0.0f;
    // rows y0-1 .. y0+K1RB are issued at steps k = 0 .. K1RB+1; output rows at k = 3 .. K1RB+2
    S.sg_next = K.load_sig(K.y0 - 1);
    K.template step<0, true, false>(S, 0);
    K.template step<1, true, false>(S, 1);
    K.template step<2, true, false>(S, 2);
    for (int k = 3; k < K1RB + 2; k += 4) {
        K.template step<3, true, true>(S, k);
        K.template step<0, true, true>(S, k + 1);
        K.template step<1, true, true>(S, k + 2);
        K.template step<2, true, true>(S, k + 3);
    }
    K.template step<3, false, true>(S, K1RB + 2);
    const psfm_params& p = a.p;
    const int units = k1_units(p.H, p.W);
    const int blk = K.b * units + K.unit;
    if (STATS) {
        const int nsrc = K.cfg.automask() ? 2 * NC : NC;
        for (int k = 0; k < nsrc; ++k) {
            const float s1 = wave_sum64(S.st[k][0]), s2 = wave_sum64(S.st[k][1]);
            if (threadIdx.x == 0) {
                float* o = a.ws.clip_part + (((size_t)K.s * nsrc + k) * (p.B * units) + blk) * 2;
                o[0] = s1;
                o[1] = s2;
            }
        }
        return;
    }
    const float ph = wave_sum64(S.acc_photo);
    const float ax = wave_sum64(S.acc_ax), ay = wave_sum64(S.acc_ay), m = wave_sum64(S.acc_m);
    if (threadIdx.x == 0) {
        a.ws.photo_part[(size_t)K.s * (p.B * units) + blk] = ph;
        if (K.cfg.smooth()) {
            float* o = a.ws.smooth_part + (((size_t)K.s * p.B + K.b) * units + K.unit) * 4;
            o[0] = ax;
            o[1] = ay;
            o[2] = m;
            o[3] = 0.0f;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K2: backward of the photometric term.  Workgroup = N waves (wave j = context j).
// ---------------------------------------------------------------------------------------------
struct K2State {
    float X[3][3], Y[3][3], SG[3];
    float gT[12];
};

// Wave-private LDS rows (each lane reads back only its own column, so no barrier is needed):
//   co[slot][m] : p-row coefficients cA[3] cB[3] cC[3] (SSIM adjoint x 1/9 x dL/dSSIM) + L1 factor
//   di[slot][m] : d(warp_c)/d(ix), d(warp_c)/d(iy) of the row, used two rows later at q
struct K2Lds {
    float co[3][10][64];
    float di[3][6][64];
};

struct K2 {
    const SweepArgs& a;
    const psfm_params& p;
    int H, W, B, N, b, s, unit, j, y0, col, colr, lane, src;
    size_t plane;
    bool pcol, qcol;
    DepthChain dc;
    float l1w, gscale, wxl, wxr;
    const float* tgt;
    const float* sig;
    const float* ctx;
    const uint8_t* am;
    const float* mask;
    const float* thr;
    CamRec cam;

    __device__ __forceinline__ K2(const SweepArgs& a_) : a(a_), p(a_.p) {
        H = p.H;
        W = p.W;
        B = p.B;
        N = p.N;
        plane = (size_t)H * W;
        const int nst = k2_stripes(W);
        const WorkItem wi = work_item();
        b = wi.b;
        s = wi.s;
        unit = wi.unit;
        lane = threadIdx.x & 63;
        j = threadIdx.x >> 6;
        y0 = (unit / nst) * K2RB;
        col = (unit % nst) * K2W - 2 + lane;
        colr = reflect1(col, W);
        pcol = lane >= 1 && lane <= K2W + 2 && col >= 0 && col < W;
        qcol = lane >= 2 && lane <= K2W + 1 && col < W;
        dc = depth_chain(p);
        l1w = 1.0f - p.ssim_w;
        src = p.automask ? 2 * j : j;
        const int nsrc = p.automask ? 2 * N : N;
        const double cnt = (double)B * H * W;
        const float gout = *a.grad_out;
        gscale = (p.reduce_op == PSFM_REDUCE_MIN) ? (float)(gout / ((double)p.n_scales * cnt))
                                                  : (float)(gout / ((double)p.n_scales * nsrc * cnt));
        wxl = (col == 1) ? 2.0f : 1.0f;      // p = col 0 reflected onto q = col 1 (SSIM reflect pad)
        wxr = (col == W - 2) ? 2.0f : 1.0f;  // p = col W-1 reflected onto q = col W-2
        tgt = a.in.tgt + (size_t)b * 3 * plane;
        sig = pick4(a.in.sig, s) + (size_t)b * plane;
        ctx = pick4(a.in.ctx, j) + (size_t)b * 3 * plane;
        am = a.ws.argmin + ((size_t)s * B + b) * plane;
        mask = a.in.mask ? a.in.mask + (size_t)b * plane : nullptr;
        thr = (p.clip_loss > 0.0f) ? a.ws.clip_thr + (size_t)s * nsrc : nullptr;
        load_cam_uniform(a.in.cam + ((size_t)(__builtin_amdgcn_readfirstlane(s * N + j)) * B + b) * PSFM_CAMREC,
                         cam);
    }

    __device__ __forceinline__ void load_row(int v, float (&x)[3], float (&y)[3], float (&di)[6][64], float& sg) const {
        const int r = reflect1(v, H);
        const size_t pix = (size_t)r * W + colr;
#pragma unroll
        for (int c = 0; c < 3; ++c) y[c] = tgt[c * plane + pix];
        sg = sig[pix];
        float d1, inv;
        const float d = dc.warp_depth(sg, d1, inv);
        Proj pr;
        project(cam, (float)colr, (float)r, d, H, W, pr);
        float dix[3], diy[3];
        bilinear3_vd(ctx, H, W, pr.ix, pr.iy, x, dix, diy);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            di[c][lane] = dix[c];
            di[3 + c][lane] = diy[c];
        }
    }

    // slots: IA = row v-2 (q), IB = row v-1 (p), IC = row v (newest)
    template <int IA, int IB, int IC>
    __device__ __forceinline__ float step(K2State& S, K2Lds& L, int k) const {
        const int v = y0 - 2 + k;
        load_row(v, S.X[IC], S.Y[IC], L.di[IC], S.SG[IC]);
        if (k < 2) return 0.0f;
        // ---- SSIM adjoint coefficients of p-row pv = v-1 (cross-lane: every lane active) ----
        const int pv = v - 1;
        {
            float my[3], syy[3], vx[3], vxx[3], vxy[3], l1 = 0.0f;
            target_window(S.Y[IA], S.Y[IB], S.Y[IC], my, syy);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float xa = S.X[IA][c], xb = S.X[IB][c], xc = S.X[IC][c];
                vx[c] = xa + xb + xc;
                vxx[c] = xa * xa + xb * xb + xc * xc;
                vxy[c] = xa * S.Y[IA][c] + xb * S.Y[IB][c] + xc * S.Y[IC][c];
                l1 += fabsf(xb - S.Y[IB][c]);
            }
            float dmx[3], dsxx[3], dsxy[3];
            const float sm = ssim_terms<true>(vx, vxx, vxy, my, syy, p.C1, p.C2, dmx, dsxx, dsxy);
            float G = 0.0f;
            if (pcol && pv >= 0 && pv < H) {
                const size_t pp = (size_t)pv * W + col;
                G = gscale * (mask ? mask[pp] : 1.0f);
                if (p.reduce_op == PSFM_REDUCE_MIN && am[pp] != src) G = 0.0f;
                if (thr && !(p.ssim_w * sm + l1w * (l1 * (1.0f / 3.0f)) <= thr[src])) G = 0.0f;
            }
            const float kS = G * (-0.5f / 27.0f) * p.ssim_w;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                L.co[IC][c][lane] = kS * dmx[c];
                L.co[IC][3 + c][lane] = kS * dsxx[c];
                L.co[IC][6 + c][lane] = kS * dsxy[c];
            }
            L.co[IC][9][lane] = G * l1w * (1.0f / 3.0f);
        }
        if (k < 4) return 0.0f;
        // ---- adjoint of q-row qv = v-2: weighted 3x3 gather of the coefficients ----
        const int qv = v - 2;
        if (qv >= H || qv >= y0 + K2RB) return 0.0f;  // wave-uniform
        const float wyu = (qv == 1) ? 2.0f : 1.0f, wyd = (qv == H - 2) ? 2.0f : 1.0f;
        float Sm[9];
#pragma unroll
        for (int m = 0; m < 9; ++m) {
            const float vsum = wyu * L.co[IA][m][lane] + L.co[IB][m][lane] + wyd * L.co[IC][m][lane];
            Sm[m] = wxl * from_prev(vsum) + vsum + wxr * from_next(vsum);
        }
        if (!qcol) return 0.0f;
        float gix = 0.0f, giy = 0.0f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float xq = S.X[IA][c], yq = S.Y[IA][c];
            const float dx = Sm[c] + 2.0f * xq * Sm[3 + c] + yq * Sm[6 + c] + L.co[IB][9][lane] * sgnf(xq - yq);
            gix += dx * L.di[IA][c][lane];
            giy += dx * L.di[IA][3 + c][lane];
        }
        float d1, inv;
        const float d = dc.warp_depth(S.SG[IA], d1, inv);
        Proj pr;
        project(cam, (float)col, (float)qv, d, H, W, pr);
        const float gd = project_grad(cam, pr, d, gix, giy, H, W, S.gT);
        return gd * dc.dwarp_ds(d, d1, inv);
    }
};

// dynamic LDS: N x K2Lds (wave-private rows) followed by the [2][N][64] context-sum ring
__host__ __device__ inline size_t k2_lds_bytes(int N) { return (size_t)N * sizeof(K2Lds) + 2 * N * 64 * sizeof(float); }

__global__ __launch_bounds__(256) void k2_backward(SweepArgs a) {
    extern __shared__ __attribute__((aligned(16))) char k2_smem[];
    const K2 K(a);
    K2Lds& L = reinterpret_cast<K2Lds*>(k2_smem)[K.j];
    float* ring = reinterpret_cast<float*>(k2_smem + (size_t)K.N * sizeof(K2Lds));  // [2][N][64]
    K2State S;
#pragma unroll
    for (int m = 0; m < 12; ++m) S.gT[m] = 0.0f;
    const int nk = K2RB + 4;  // rows y0-2 .. y0+K2RB+1
    float* gsig = pick4(a.grad_sig, K.s) + (size_t)K.b * K.plane;
    const int N = K.N;
    auto emit = [&](int k, float gs) {
        if (k < 4) return;
        const int qv = K.y0 - 4 + k;
        if (qv >= K.H || qv >= K.y0 + K2RB) return;
        if (N == 1) {
            if (K.qcol) gsig[(size_t)qv * K.W + K.col] = gs;
            return;
        }
        ring[((k & 1) * N + K.j) * 64 + K.lane] = gs;
        __syncthreads();
        if (K.j == 0 && K.qcol) {
            float t = 0.0f;
            for (int jj = 0; jj < N; ++jj) t += ring[((k & 1) * N + jj) * 64 + K.lane];
            gsig[(size_t)qv * K.W + K.col] = t;
        }
    };
    for (int k = 0; k < nk; k += 3) {
        emit(k, K.step<1, 2, 0>(S, L, k));
        if (k + 1 < nk) emit(k + 1, K.step<2, 0, 1>(S, L, k + 1));
        if (k + 2 < nk) emit(k + 2, K.step<0, 1, 2>(S, L, k + 2));
    }
    const int units = k2_units(a.p.H, a.p.W);
    float* o = a.ws.pose_part + ((((size_t)K.s * N + K.j) * a.p.B + K.b) * units + K.unit) * 12;
#pragma unroll
    for (int m = 0; m < 12; ++m) {
        const float t = wave_sum64(S.gT[m]);
        if (K.lane == 0) o[m] = t;
    }
}

}  // namespace sweep
}  // namespace psfm
