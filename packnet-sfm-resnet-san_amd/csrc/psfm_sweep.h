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

#include "psfm_common.h"

namespace psfm {
namespace sweep {

#ifndef PSFM_K1_RB
#define PSFM_K1_RB 12
#endif
#ifndef PSFM_K2_RB
#define PSFM_K2_RB 24
#endif
#ifndef PSFM_XCD_REMAP
#define PSFM_XCD_REMAP 1
#endif
constexpr int K1RB = PSFM_K1_RB;  // output rows per K0/K1 band
constexpr int K2RB = PSFM_K2_RB;  // output rows per K2 band
constexpr int K1W = 62;           // output columns per K1 stripe (halo 1)
constexpr int K2W = 60;           // output columns per K2 stripe (halo 2)

__host__ __device__ inline int k1_stripes(int W) { return (W + K1W - 1) / K1W; }
__host__ __device__ inline int k2_stripes(int W) { return (W + K2W - 1) / K2W; }
__host__ __device__ inline int k1_units(int H, int W) { return k1_stripes(W) * ((H + K1RB - 1) / K1RB); }
__host__ __device__ inline int k2_units(int H, int W) { return k2_stripes(W) * ((H + K2RB - 1) / K2RB); }

// Which (unit, batch, scale) this workgroup sweeps.  Grid = (units, B, S).  With PSFM_XCD_REMAP
// the linear block id is re-dealt so that the blocks one XCD receives (round-robin dealing:
// blocks i and i+8 share an XCD) form one contiguous run of (b, s, unit) -> one image's context
// frames stay in that XCD's L2 (speed only: any placement is correct).
struct WorkItem {
    int unit, b, s;
};
__device__ __forceinline__ WorkItem work_item() {
#if PSFM_XCD_REMAP
    const int units = gridDim.x, B = gridDim.y, S = gridDim.z;
    const int T = units * B * S;
    const int L = blockIdx.x + units * (blockIdx.y + B * blockIdx.z);
    const int xcd = L & 7, i = L >> 3, q = T >> 3, r = T & 7;
    const int w = xcd < r ? xcd * (q + 1) + i : r * (q + 1) + (xcd - r) * q + i;
    const int bs = w / units;
    return WorkItem{w - bs * units, bs / S, bs % S};
#else
    return WorkItem{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
#endif
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
    const size_t plane = (size_t)H * W;
    float q[3][4];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float* im = img + c * plane;
        q[c][0] = im[t.nw];
        q[c][1] = im[t.ne];
        q[c][2] = im[t.sw];
        q[c][3] = im[t.se];
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
// K0: automask candidates — photometric loss of every UN-warped context against the target
// (multiview_photometric_loss.py:394-399).  Scale independent at full resolution, so computed
// once per call instead of once per scale; one wave per (stripe, band, batch), K1 geometry.
// ---------------------------------------------------------------------------------------------
template <int NC>
__global__ __launch_bounds__(64) void k0_unwarped(SweepArgs a) {
    const psfm_params& p = a.p;
    const int H = p.H, W = p.W, B = p.B;
    const size_t plane = (size_t)H * W;
    const WorkItem wi = work_item();
    const int nst = k1_stripes(W), b = wi.b;
    const int y0 = (wi.unit / nst) * K1RB;
    const int col = (wi.unit % nst) * K1W - 1 + (int)threadIdx.x;
    const int colr = reflect1(col, W);
    const bool pcol = threadIdx.x >= 1 && threadIdx.x <= K1W && col < W;
    const float l1w = 1.0f - p.ssim_w;
    const float* tgt = a.in.tgt + (size_t)b * 3 * plane;
    float Y[3][3], X[3][NC][3];
    auto load = [&](int v, float (&y)[3], float (&x)[NC][3]) {
        const size_t pix = (size_t)reflect1(v, H) * W + colr;
#pragma unroll
        for (int c = 0; c < 3; ++c) y[c] = tgt[c * plane + pix];
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int c = 0; c < 3; ++c) x[j][c] = pick4(a.in.ctx, j)[((size_t)b * 3 + c) * plane + pix];
    };
    auto emit = [&](int k, float (&ya)[3], float (&yb)[3], float (&yc)[3], float (&xa)[NC][3],
                    float (&xb)[NC][3], float (&xc)[NC][3]) {
        const int pv = y0 - 2 + k;
        if (k < 2 || pv >= H || pv >= y0 + K1RB) return;  // wave-uniform
        float my[3], syy[3];
        target_window(ya, yb, yc, my, syy);
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            float vx[3], vxx[3], vxy[3], l1 = 0.0f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                vx[c] = xa[j][c] + xb[j][c] + xc[j][c];
                vxx[c] = xa[j][c] * xa[j][c] + xb[j][c] * xb[j][c] + xc[j][c] * xc[j][c];
                vxy[c] = xa[j][c] * ya[c] + xb[j][c] * yb[c] + xc[j][c] * yc[c];
                l1 += fabsf(xb[j][c] - yb[c]);
            }
            float d0[3], d1[3], d2[3];
            const float sm = ssim_terms<false>(vx, vxx, vxy, my, syy, p.C1, p.C2, d0, d1, d2);
            const float val = p.ssim_w * sm + l1w * (l1 * (1.0f / 3.0f));
            if (pcol) a.ws.unwarp[((size_t)j * B + b) * plane + (size_t)pv * W + col] = val;
        }
    };
    const int nk = K1RB + 2;
    for (int k = 0; k < nk; k += 3) {
        load(y0 - 1 + k, Y[0], X[0]);
        emit(k, Y[1], Y[2], Y[0], X[1], X[2], X[0]);
        if (k + 1 < nk) {
            load(y0 + k, Y[1], X[1]);
            emit(k + 1, Y[2], Y[0], Y[1], X[2], X[0], X[1]);
        }
        if (k + 2 < nk) {
            load(y0 + 1 + k, Y[2], X[2]);
            emit(k + 2, Y[0], Y[1], Y[2], X[0], X[1], X[2]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K1: forward (+ fused smoothness forward).  NC = number of contexts (exact register arrays).
// STATS: clip-statistics pass (sum / sumsq of every raw candidate map, :249-253).
// ---------------------------------------------------------------------------------------------
template <int NC, bool STATS>
struct K1State {
    float Y[3][3], XW[3][NC][3], SG[3];
    float acc_photo, acc_ax, acc_ay, acc_m;
    float st[2 * NC][2];
};

template <int NC, bool STATS>
struct K1 {
    const SweepArgs& a;
    const psfm_params& p;
    int H, W, b, s, unit, y0, col, colr, B;
    size_t plane;
    bool pcol;
    DepthChain dc;
    float l1w;
    const float* tgt;
    const float* sig;
    const float* ctx[NC];
    const float* thr;
    CamRec cam[NC];

    __device__ __forceinline__ K1(const SweepArgs& a_) : a(a_), p(a_.p) {
        H = p.H;
        W = p.W;
        B = p.B;
        plane = (size_t)H * W;
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
        sig = pick4(a.in.sig, s) + (size_t)b * plane;
#pragma unroll
        for (int j = 0; j < NC; ++j) ctx[j] = pick4(a.in.ctx, j) + (size_t)b * 3 * plane;
#pragma unroll
        for (int j = 0; j < NC; ++j)
            load_cam_uniform(a.in.cam + ((size_t)(s * NC + j) * B + b) * PSFM_CAMREC, cam[j]);
        thr = (p.clip_loss > 0.0f && !STATS) ? a.ws.clip_thr + (size_t)s * (p.automask ? 2 * NC : NC) : nullptr;
    }

    __device__ __forceinline__ void load_row(int v, float (&y)[3], float (&xw)[NC][3], float& sg) const {
        const int r = reflect1(v, H);
        const size_t pix = (size_t)r * W + colr;
#pragma unroll
        for (int c = 0; c < 3; ++c) y[c] = tgt[c * plane + pix];
        sg = sig[pix];
        float d1, inv;
        const float d = dc.warp_depth(sg, d1, inv);
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            Proj pr;
            project(cam[j], (float)colr, (float)r, d, H, W, pr);
            bilinear3(ctx[j], H, W, pr.ix, pr.iy, xw[j]);
        }
    }

    // slots: IA = row v-2, IB = row v-1 (output), IC = row v (newest)
    template <int IA, int IB, int IC>
    __device__ __forceinline__ void step(K1State<NC, STATS>& S, int k) const {
        const int v = y0 - 1 + k;
        load_row(v, S.Y[IC], S.XW[IC], S.SG[IC]);
        if (k < 2) return;
        const int pv = v - 1;
        if (pv >= H || pv >= y0 + K1RB) return;  // wave-uniform
        // ---- cross-lane phase (every lane active) ----
        float my[3], syy[3];
        target_window(S.Y[IA], S.Y[IB], S.Y[IC], my, syy);
        float cand[2 * NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            float vx[3], vxx[3], vxy[3], l1 = 0.0f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float xa = S.XW[IA][j][c], xb = S.XW[IB][j][c], xc = S.XW[IC][j][c];
                vx[c] = xa + xb + xc;
                vxx[c] = xa * xa + xb * xb + xc * xc;
                vxy[c] = xa * S.Y[IA][c] + xb * S.Y[IB][c] + xc * S.Y[IC][c];
                l1 += fabsf(xb - S.Y[IB][c]);
            }
            float d0[3], d1[3], d2[3];
            const float sm = ssim_terms<false>(vx, vxx, vxy, my, syy, p.C1, p.C2, d0, d1, d2);
            cand[2 * j] = p.ssim_w * sm + l1w * (l1 * (1.0f / 3.0f));
        }
        float sgn_next = 0.0f, ynext[3] = {0.0f, 0.0f, 0.0f};
        if (!STATS && p.smooth_w > 0.0f) {
            sgn_next = from_next(S.SG[IB]);
#pragma unroll
            for (int c = 0; c < 3; ++c) ynext[c] = from_next(S.Y[IB][c]);
        }
        // ---- lane-local phase ----
        if (!pcol) return;
        const size_t ppix = (size_t)pv * W + col;
        if (p.automask) {  // un-warped candidates (K0, scale independent)
#pragma unroll
            for (int j = 0; j < NC; ++j) cand[2 * j + 1] = a.ws.unwarp[((size_t)j * B + b) * plane + ppix];
        }
        if (STATS) {
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const int sw = p.automask ? 2 * j : j;
                S.st[sw][0] += cand[2 * j];
                S.st[sw][1] += cand[2 * j] * cand[2 * j];
                if (p.automask) {
                    S.st[sw + 1][0] += cand[2 * j + 1];
                    S.st[sw + 1][1] += cand[2 * j + 1] * cand[2 * j + 1];
                }
            }
            return;
        }
        const float mval = a.in.mask ? a.in.mask[(size_t)b * plane + ppix] : 1.0f;
        float best = INFINITY, sum = 0.0f;
        int arg = 0, kk = 0;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (u == 1 && !p.automask) break;
                float val = cand[2 * j + u];
                if (thr) val = fminf(val, thr[u ? 2 * j + 1 : (p.automask ? 2 * j : j)]);
                val *= mval;
                sum += val;
                if (val < best) {
                    best = val;
                    arg = kk;
                }
                ++kk;
            }
        }
        if (p.reduce_op == PSFM_REDUCE_MIN) {
            S.acc_photo += best;
            a.ws.argmin[((size_t)s * B + b) * plane + ppix] = (uint8_t)arg;
        } else {
            S.acc_photo += sum;
        }
        if (p.smooth_w > 0.0f) {  // edge-aware smoothness of the sigmoid map (utils/depth.py:165-198)
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

template <int NC, bool STATS>
__global__ __launch_bounds__(64) void k1_forward(SweepArgs a) {
    K1<NC, STATS> K(a);
    K1State<NC, STATS> S;
    S.acc_photo = S.acc_ax = S.acc_ay = S.acc_m = 0.0f;
#pragma unroll
    for (int k = 0; k < 2 * NC; ++k) S.st[k][0] = S.st[k][1] = 0.0f;
    const int nk = K1RB + 2;  // rows y0-1 .. y0+K1RB
    for (int k = 0; k < nk; k += 3) {
        K.template step<1, 2, 0>(S, k);
        if (k + 1 < nk) K.template step<2, 0, 1>(S, k + 1);
        if (k + 2 < nk) K.template step<0, 1, 2>(S, k + 2);
    }
    const psfm_params& p = a.p;
    const int units = k1_units(p.H, p.W);
    const int blk = K.b * units + K.unit;
    if (STATS) {
        const int nsrc = p.automask ? 2 * NC : NC;
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
        if (p.smooth_w > 0.0f) {
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
