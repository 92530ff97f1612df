// psfm_fused.h — K12: forward AND eager backward of the photometric + smoothness terms in ONE
// row sweep (gfx950).
//
// The backward of the photometric loss needs, per pixel, everything its forward computes — the
// warped samples of every context, the 3x3 SSIM statistics and the min-reprojection choice — so
// a separate backward kernel (K2) re-does the whole forward.  K12 does it once: the gradient of
// the loss w.r.t. the sigmoid maps is linear in dL/dloss, so it is produced during the forward
// for dL/dloss = 1 and scaled later by psfm_photometric_grad_finish (which also adds the one
// per-image term that needs whole-image sums: d/ds of the 1/mean(s) smoothness normaliser).
//
// One wave per (60-column stripe, RB-row band, image, scale), both contexts of a target packed
// in the two halves of 64-bit register pairs (v_pk_* arithmetic).  Lanes = columns c0-2..c0+61;
// the 60 inner lanes are outputs (a 3x3 SSIM window of a 3x3 neighbourhood: halo 2).  Step k
// of the sweep:
//   issue   row v = y0-2+k: target, sigmoid (prefetched one step earlier), lift/project per
//           context and the 12 bilinear gathers per context (results consumed at the END of
//           the step, so their latency hides under the two evaluations below);
//   p-eval  row v-2: SSIM + L1 of every warped context (forward value AND the SSIM adjoint
//           coefficients d/d(mean x, E[x^2], E[xy])), automask candidates (K0 maps), min /
//           argmin (or mean), clip / mask, forward partial sums, smoothness forward terms; the
//           coefficients of the SELECTED candidate (G = 0 for the others) are accumulated
//           vertically into the three q-rows they touch (reflect weights at the image edge);
//   q-eval  row v-3 (its three p-rows are now complete): horizontal 3-sum of the accumulated
//           coefficients (DPP), adjoint through the bilinear sample (d warp / d(ix,iy) stashed
//           in wave-private LDS at issue time) and the projection, dL/d[R|t] per context, plus
//           the per-pixel smoothness gradient -> dL/dsig written once (contexts summed in
//           order in registers: deterministic, no LDS ring, no barrier);
//   resolve the bilinear samples of row v (x and d x/d(ix,iy)).
// Reference: losses/multiview_photometric_loss.py:15-54, :199-297, :301-327,
// utils/depth.py:146-198, geometry/camera.py:111-190, geometry/camera_utils.py:27-59.
#pragma once
#include "psfm_camera.h"
#include "psfm_sweep.h"

namespace psfm {
namespace fused {

using sweep::Cfg;
using sweep::depth_chain;
using sweep::f2;
using sweep::from_next;
using sweep::from_prev;
using sweep::hsum3a;
using sweep::hsum3x3;
using sweep::pick4;
using sweep::sgnf;
using sweep::target_win;
using sweep::TWin;
using sweep::wave_sum64;
using sweep::work_item;

#ifndef PSFM_K12_WAVES
#define PSFM_K12_WAVES 2
#endif
#ifndef PSFM_K12_CAM_RELOAD
#define PSFM_K12_CAM_RELOAD 1
#endif
#ifndef PSFM_K12_DI_B128
#define PSFM_K12_DI_B128 0
#endif
#ifndef PSFM_K12_GT_REG
#define PSFM_K12_GT_REG 0
#endif
#ifndef PSFM_K12_RB
#define PSFM_K12_RB 20
#endif
// Phase boundaries of a sweep step (issue | p-eval | q-eval | resolve): the scheduler may not
// interleave the phases, so the register peak is the largest phase's, not their sum (the
// gathers issued in the first phase still fly under the next two: loads are asynchronous).
#ifndef PSFM_K12_NO_PHASES
#define PSFM_PHASE() __builtin_amdgcn_sched_barrier(0)
#else
#define PSFM_PHASE() ((void)0)
#endif
// channel boundaries inside the SSIM phases: three unrolled channels interleaved by the
// scheduler triple the live temporaries (~40 VGPRs each)
#ifndef PSFM_K12_NO_CHAN
#define PSFM_CHAN() __builtin_amdgcn_sched_barrier(0)
#else
#define PSFM_CHAN() ((void)0)
#endif
constexpr int RB = PSFM_K12_RB;  // q (output) rows per band
constexpr int OW = 60;           // output columns per stripe
constexpr int SIGCH = 16;        // chunks of the per-(scale, image) sigmoid sum pre-pass
static_assert(RB % 4 == 0, "K12 band height must be a multiple of 4 (4-slot pipeline)");

__host__ __device__ inline int stripes(int W) { return (W + OW - 1) / OW; }
__host__ __device__ inline int units(int H, int W) { return stripes(W) * ((H + RB - 1) / RB); }
// wave-private LDS (each lane touches only its own column: no barriers):
//   [3 row slots][6 NC] d warp / d(ix, iy) | [12 NC] per-lane dL/d[R|t] accumulators
// per-lane dL/dT row stride: 12 NC floats padded to 16 NC + ... (28 dwords at NC = 2: the 16
// lanes of a b128 access start on distinct 4-bank groups -> no bank conflicts)
__host__ __device__ constexpr int gt_stride(int NC) { return NC == 1 ? 12 : 28; }
__host__ __device__ inline size_t lds_bytes(int NC) {
    return ((size_t)3 * 6 * NC * 64 + (size_t)gt_stride(NC) * 64) * sizeof(float);
}

struct Args {
    psfm_params p;
    psfm_inputs in;
    psfm_workspace ws;
    float* grad_sig[PSFM_MAX_SCALES];
};

// Bilinear gathers in flight for one context (issued at the top of a step, resolved at its end).
struct Pend {
    float q[3][4];
    float ax, bx, ay, by;
    bool vnw, vne, vsw, vse;
};

__device__ __forceinline__ void gather(const float* __restrict__ img, uint32_t pb, float ix, float iy, int H,
                                       int W, Pend& g) {
    const TapAddr t = tap_addr(ix, iy, H, W);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        g.q[c][0] = ldg(img, c * pb + t.nw);
        g.q[c][1] = ldg(img, c * pb + t.ne);
        g.q[c][2] = ldg(img, c * pb + t.sw);
        g.q[c][3] = ldg(img, c * pb + t.se);
    }
    g.ax = t.ax;
    g.bx = t.bx;
    g.ay = t.ay;
    g.by = t.by;
    g.vnw = t.vnw;
    g.vne = t.vne;
    g.vsw = t.vsw;
    g.vse = t.vse;
}

// grid_sample value and d/d(ix), d/d(iy) (same arithmetic as sweep::bilinear3_vd)
__device__ __forceinline__ void resolve(const Pend& g, float v[3], float dix[3], float diy[3]) {
    const float wnw = g.ax * g.ay, wne = g.bx * g.ay, wsw = g.ax * g.by, wse = g.bx * g.by;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float nw = g.vnw ? g.q[c][0] : 0.0f, ne = g.vne ? g.q[c][1] : 0.0f;
        const float sw = g.vsw ? g.q[c][2] : 0.0f, se = g.vse ? g.q[c][3] : 0.0f;
        float acc = 0.0f;
        acc += nw * wnw;
        acc += ne * wne;
        acc += sw * wsw;
        acc += se * wse;
        v[c] = acc;
        dix[c] = (ne - nw) * g.ay + (se - sw) * g.by;
        diy[c] = (sw - nw) * g.ax + (se - ne) * g.bx;
    }
}

// Adjoint of project_lifted for one context: (gix, giy) -> dL/d(warp depth), dL/dT += ...
// (same arithmetic as psfm::project_grad)
// dL/dT += gc (X, 1)^T into 12 accumulators (registers, or a lane-private LDS row)
template <typename P>
__device__ __forceinline__ void acc_gT(float* g, const float (&gc)[3], const P& r) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        g[4 * i + 0] += gc[i] * r.X0;
        g[4 * i + 1] += gc[i] * r.X1;
        g[4 * i + 2] += gc[i] * r.X2;
        g[4 * i + 3] += gc[i];
    }
}

__device__ __forceinline__ f2 pk_rcp(f2 v) { return f2{__builtin_amdgcn_rcpf(v.x), __builtin_amdgcn_rcpf(v.y)}; }
__device__ __forceinline__ f2 pk_sel01(f2 l) {  // 1 where 0 <= l <= 1 (clamp pass-through), else 0
    return f2{(l.x >= 0.0f && l.x <= 1.0f) ? 1.0f : 0.0f, (l.y >= 0.0f && l.y <= 1.0f) ? 1.0f : 0.0f};
}

// Photometric candidate of a context pair at the middle row AND the SSIM adjoint coefficients
// cf[c] = dSSIM_c/d(mean x), cf[3+c] = dSSIM_c/dE[x^2], cf[6+c] = dSSIM_c/dE[xy] (x clamp
// pass-through).  Forward value as sweep::photo_pair; coefficients as sweep::ssim_terms<true>.
// Cross-lane: all lanes active.
__device__ __forceinline__ f2 photo_grad_pair(const f2 (&xa)[3], const f2 (&xb)[3], const f2 (&xc)[3],
                                              const float (&ya)[3], const float (&yb)[3], const float (&yc)[3],
                                              const TWin& tw, float C1, float C2, float ssim_w, float l1w,
                                              f2 (&cf)[9]) {
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
        const float my = tw.my[c];
        const f2 mxy = mx * my, mx2 = mx * mx;
        const f2 A1 = 2.0f * mxy + C1, A2 = 2.0f * (sxy - mxy) + C2;
        const f2 B1 = mx2 + tw.my2[c] + C1, B2 = (sxx - mx2) + tw.ty[c] + C2;
        const f2 Nn = A1 * A2, D = B1 * B2;
        const f2 iD = pk_rcp(D);
        const f2 l = (1.0f - Nn * iD) * 0.5f;
        ls += f2{__builtin_amdgcn_fmed3f(l.x, 0.0f, 1.0f), __builtin_amdgcn_fmed3f(l.y, 0.0f, 1.0f)};
        const f2 pass = pk_sel01(l);
        const f2 iD2 = iD * iD;
        cf[c] = pass * (2.0f * my * (A2 - A1) * iD - Nn * 2.0f * mx * (B2 - B1) * iD2);
        cf[3 + c] = pass * (-Nn * B1 * iD2);
        cf[6 + c] = pass * (2.0f * A1 * iD);
        const f2 dd = xb[c] - yb[c];
        l1 += f2{fabsf(dd.x), fabsf(dd.y)};
        PSFM_CHAN();
    }
    return ssim_w * (ls * (1.0f / 3.0f)) + l1w * (l1 * (1.0f / 3.0f));
}

template <int NC>
struct State {
    static constexpr int NP = (NC + 1) / 2;
    // four row slots as separate members (compile-time slot selection; no indexed aggregate
    // that could be demoted to scratch)
    float Y0[3], Y1[3], Y2[3], Y3[3];
    float SG0, SG1, SG2, SG3;
    f2 X0[NP][3], X1[NP][3], X2[NP][3], X3[NP][3];
    float sg_next;
    float un[NC], mv;  // K0 candidates and mask of this step's p-row (loaded before the gathers)
    template <int I> __device__ __forceinline__ float (&Y())[3] {
        if constexpr (I == 0) return Y0; else if constexpr (I == 1) return Y1; else if constexpr (I == 2) return Y2; else return Y3;
    }
    template <int I> __device__ __forceinline__ float& SG() {
        if constexpr (I == 0) return SG0; else if constexpr (I == 1) return SG1; else if constexpr (I == 2) return SG2; else return SG3;
    }
    template <int I> __device__ __forceinline__ f2 (&X())[NP][3] {
        if constexpr (I == 0) return X0; else if constexpr (I == 1) return X1; else if constexpr (I == 2) return X2; else return X3;
    }
    // dL/d(warped sample) per channel (context pairs packed) of the q-rows a p-row touches:
    // D0 = row p-1 (completed by this p-row), D1 = row p, D2 = row p+1
    f2 D0[NP][3], D1[NP][3], D2[NP][3];
    float h_p, h_n;           // smoothness x-term sgn(s - s_right) w of p-row q / this p-row
    float t_pp, t_p, t_n;     // y-term sgn(s - s_below) w of p-rows q-1, q, this p-row
    float acc_photo, acc_ax, acc_ay, acc_m;
#if PSFM_K12_GT_REG
    float gT[NC][12];
#endif
};

template <int NC, bool FAST, int MODEL>
struct K12 {
    using CM = Cams<NC, MODEL>;
    static constexpr int NP = (NC + 1) / 2;
    const Args& a;
    const psfm_params& p;
    Cfg<FAST> cfg;
    int H, W, B, b, s, unit, y0, col, colr, lane;
    int sh, Ws, colc;  // sigmoid storage: (H >> sh, W >> sh), this lane's stored column
    uint32_t plane, pb;
    bool pcol, qcol, border;
    DepthChain dc;
    float l1w, gscale, cx, cy, mc, wxl, wxr;
    const float* tgt;
    const float* sig;
    const float* ctx[NC];
    const float* thr;
    const float* mask;
    float* gsig;
    float* di;  // wave-private LDS [3][NC*6][64]
    float* gt;  // (PSFM_K12_GT_REG=0) this lane's dL/dT accumulators: gt[j*12 + m], 16-B aligned
    const float* camrec;  // record of (s, context 0, b); context j is j*B records further

    // The 51 camera scalars are re-loaded at each use (s_load through the constant address
    // space: scalar cache, no VGPRs) instead of being held in SGPRs for the whole sweep; the
    // laundered pointer stops the compiler from keeping them live across the SSIM phase.
    __device__ __forceinline__ CM load_cams() const {
        uint64_t rp = reinterpret_cast<uint64_t>(camrec);
#if PSFM_K12_CAM_RELOAD
        asm volatile("" : "+s"(rp));
#endif
        CM c;
        c.load(reinterpret_cast<cfloat*>(rp), B, H, W);
        return c;
    }

    __device__ __forceinline__ K12(const Args& a_, float* lds) : a(a_), p(a_.p), cfg{a_.p} {
        H = p.H;
        W = p.W;
        B = p.B;
        plane = (uint32_t)(H * W);
        pb = plane * 4u;
        const int nst = stripes(W);
        const sweep::WorkItem wi = work_item();
        b = wi.b;
        s = wi.s;
        unit = wi.unit;
        lane = threadIdx.x;
        y0 = (unit / nst) * RB;
        const int c0 = (unit % nst) * OW;
        col = c0 - 2 + lane;
        colr = reflect1(col, W);
        pcol = lane >= 1 && lane <= OW + 2 && col >= 0 && col < W;
        qcol = lane >= 2 && lane <= OW + 1 && col < W;
        border = c0 <= 1 || c0 + OW >= W - 2;  // this stripe holds column 1 or W-2
        wxl = (col == 1) ? 2.0f : 1.0f;        // p = col 0 reflected onto q = col 1 (SSIM reflect pad)
        wxr = (col == W - 2) ? 2.0f : 1.0f;    // p = col W-1 reflected onto q = col W-2
        dc = depth_chain(p);
        l1w = 1.0f - p.ssim_w;
        const double cnt = (double)B * H * W;
        const int nsrc = p.automask ? 2 * p.N : p.N;
        gscale = cfg.is_min() ? (float)(1.0 / ((double)p.n_scales * cnt))
                              : (float)(1.0 / ((double)p.n_scales * nsrc * cnt));
        const int gsi = p.scale0 + s;
        const double base = (double)p.smooth_w / ((double)p.n_scales * (double)(1 << gsi));
        cx = (float)(base / ((double)B * H * (W - 1)));
        cy = (float)(base / ((double)B * (H - 1) * W));
        tgt = a.in.tgt + (size_t)b * 3 * plane;
        sh = pick4(p.sig_shift, s);
        Ws = W >> sh;
        colc = colr >> sh;
        sig = pick4(a.in.sig, s) + (size_t)b * (plane >> (2 * sh));
#pragma unroll
        for (int j = 0; j < NC; ++j) ctx[j] = pick4(a.in.ctx, j) + (size_t)b * 3 * plane;
        thr = (cfg.clip()) ? a.ws.clip_thr + (size_t)s * (cfg.automask() ? 2 * NC : NC) : nullptr;
        mask = (!FAST && a.in.mask) ? a.in.mask + (size_t)b * plane : nullptr;
        gsig = pick4(a.grad_sig, s) + (size_t)b * plane;
        di = lds;
        gt = lds + 3 * 6 * NC * 64 + lane * gt_stride(NC);
        camrec = a.in.cam + ((size_t)s * NC * B + b) * PSFM_CAMREC;
        // per-image mean of the sigmoid map (smoothness normaliser, utils/depth.py:183-185),
        // from the SIGCH chunk sums of the pre-pass, summed in chunk order in fp64 (wave-uniform
        // scalar loads: written by the previous launch, read-only here)
        mc = 1.0f;
        if (cfg.smooth()) {
            typedef __attribute__((address_space(4))) const float cfloat;
            cfloat* sp = reinterpret_cast<cfloat*>(reinterpret_cast<uint64_t>(a.ws.sig_part) +
                                                   (((size_t)s * B + b) * SIGCH) * sizeof(float));
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < SIGCH; ++i) v += (double)sp[i];
            mc = fmaxf((float)(v / ((double)H * W)), 1e-6f);
        }
    }

    // d warp / d(ix, iy) of a row slot: [slot][m][64] (b32, conflict-free) or, with
    // PSFM_K12_DI_B128, [slot][lane][6 NC] (b128: a quarter of the LDS instructions)
    __device__ __forceinline__ void di_store(int slot, const float (&dv)[NC * 6]) const {
#if PSFM_K12_DI_B128
        float4* d4 = reinterpret_cast<float4*>(di + (slot * 64 + lane) * (NC * 6));
#pragma unroll
        for (int i = 0; i < NC * 6 / 4; ++i) d4[i] = make_float4(dv[4 * i], dv[4 * i + 1], dv[4 * i + 2], dv[4 * i + 3]);
        if ((NC * 6) % 4) {
            float2* d2 = reinterpret_cast<float2*>(di + (slot * 64 + lane) * (NC * 6) + (NC * 6 / 4) * 4);
            d2[0] = make_float2(dv[NC * 6 - 2], dv[NC * 6 - 1]);
        }
#else
        float* ds = di + slot * (NC * 6 * 64);
#pragma unroll
        for (int m = 0; m < NC * 6; ++m) ds[m * 64 + lane] = dv[m];
#endif
    }
    __device__ __forceinline__ void di_load(int slot, float (&dv)[NC * 6]) const {
#if PSFM_K12_DI_B128
        const float4* d4 = reinterpret_cast<const float4*>(di + (slot * 64 + lane) * (NC * 6));
#pragma unroll
        for (int i = 0; i < NC * 6 / 4; ++i) {
            const float4 t = d4[i];
            dv[4 * i] = t.x; dv[4 * i + 1] = t.y; dv[4 * i + 2] = t.z; dv[4 * i + 3] = t.w;
        }
        if ((NC * 6) % 4) {
            const float2 t = reinterpret_cast<const float2*>(di + (slot * 64 + lane) * (NC * 6) + (NC * 6 / 4) * 4)[0];
            dv[NC * 6 - 2] = t.x;
            dv[NC * 6 - 1] = t.y;
        }
#else
        const float* ds = di + slot * (NC * 6 * 64);
#pragma unroll
        for (int m = 0; m < NC * 6; ++m) dv[m] = ds[m * 64 + lane];
#endif
    }

    // the sigmoid at full-resolution row v, this lane's column: nearest upsampling of the stored
    // (H >> sh, W >> sh) map by 2^sh (upsample_output, model_utils.py:152-196)
    __device__ __forceinline__ float load_sig(int v) const {
        return sig[(uint32_t)((reflect1(v, H) >> sh) * Ws + colc)];
    }

    template <int I, bool LOAD, bool PEVAL, bool QEVAL>
    __device__ __forceinline__ void step(State<NC>& S, int k) const {
        constexpr int IA = (I + 1) & 3, IB = (I + 2) & 3, IC = (I + 3) & 3;
        const int v = y0 - 2 + k;
        Pend pd[NC];
        if (PEVAL) {
            // the p-row's K0 candidates / mask FIRST: vmcnt retires in issue order, so loads issued
            // after the gathers would make the p-eval wait for the gathers too
            const int pv = v - 2;
            const bool pin = pcol && pv >= 0 && pv < H;
            const uint32_t ppix = (uint32_t)(pv * W + col);
#pragma unroll
            for (int j = 0; j < NC; ++j)
                S.un[j] = (cfg.automask() && pin) ? a.ws.unwarp[((size_t)j * B + b) * plane + ppix] : 0.0f;
            S.mv = (mask && pin) ? mask[ppix] : 1.0f;
        }
        if (LOAD) {
            const float sg = S.sg_next;
            S.sg_next = load_sig(v + 1);
            S.template SG<I>() = sg;
            const int r = reflect1(v, H);
            const uint32_t pix = (uint32_t)(r * W + colr);
#pragma unroll
            for (int c = 0; c < 3; ++c) S.template Y<I>()[c] = tgt[c * plane + pix];
            const CM cams = load_cams();
            float d1, inv;
            const float d = dc.warp_depth(sg, d1, inv);
            const Lift l = cams.lift((float)colr, (float)r, d);
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                typename CM::P pr;
                cams.project(j, l, pr);
                gather(ctx[j], pb, pr.ix, pr.iy, H, W, pd[j]);
            }
        }
#ifdef PSFM_K12_NOPIPE
        if (LOAD) resolve_row<I>(S, k, pd);
#endif
        PSFM_PHASE();
        if (PEVAL) peval<IA, IB, IC>(S, v - 2);
        PSFM_PHASE();
        if (QEVAL) qeval<IA>(S, v - 3, k);
        PSFM_PHASE();
        if (PEVAL) {  // rotate the carried per-row terms
            S.t_pp = S.t_p;
            S.t_p = S.t_n;
            S.h_p = S.h_n;
#pragma unroll
            for (int q = 0; q < NP; ++q)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    S.D0[q][c] = S.D1[q][c];
                    S.D1[q][c] = S.D2[q][c];
                }
        }
#ifndef PSFM_K12_NOPIPE
        if (LOAD) resolve_row<I>(S, k, pd);
#endif
    }

    template <int I>
    __device__ __forceinline__ void resolve_row(State<NC>& S, int k, const Pend (&pd)[NC]) const {
        {
            float dv[NC * 6];
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                float x[3], dix[3], diy[3];
                resolve(pd[j], x, dix, diy);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    S.template X<I>()[j >> 1][c][j & 1] = x[c];
                    dv[j * 6 + c] = dix[c];
                    dv[j * 6 + 3 + c] = diy[c];
                }
            }
            di_store(k % 3, dv);
            if (NC & 1) {
#pragma unroll
                for (int c = 0; c < 3; ++c) S.template X<I>()[NP - 1][c].y = S.template X<I>()[NP - 1][c].x;
            }
        }
    }

    // p-row pv from slots IA (pv-1), IB (pv), IC (pv+1)
    template <int IA, int IB, int IC>
    __device__ __forceinline__ void peval(State<NC>& S, int pv) const {
        // ---- cross-lane phase (every lane active) ----
        const TWin tw = target_win(S.template Y<IA>(), S.template Y<IB>(), S.template Y<IC>());
        f2 cf[NP][9], cand[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q)
            cand[q] = photo_grad_pair(S.template X<IA>()[q], S.template X<IB>()[q], S.template X<IC>()[q], S.template Y<IA>(), S.template Y<IB>(), S.template Y<IC>(), tw, p.C1,
                                      p.C2, p.ssim_w, l1w, cf[q]);
        const float sg_r = from_next(S.template SG<IB>());
        float y_r[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) y_r[c] = from_next(S.template Y<IB>()[c]);
        // ---- lane-local phase ----
        const bool pin = pcol && pv >= 0 && pv < H;  // a real pixel
        const bool pout = pin && qcol && pv >= y0 && pv < y0 + RB;  // an output pixel of this wave
        float G[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) G[j] = 0.0f;
        if (pin) {
            float raw[2 * NC];
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                raw[2 * j] = (j & 1) ? cand[j >> 1].y : cand[j >> 1].x;
                raw[2 * j + 1] = S.un[j];
            }
            const float mval = S.mv;
            float best = INFINITY, sum = 0.0f;
            int arg = 0, kk = 0;
            bool keep[NC];
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                keep[j] = true;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    if (u == 1 && !cfg.automask()) break;
                    float val = raw[2 * j + u];
                    if (!FAST) {
                        if (thr) {
                            const float th = thr[u ? 2 * j + 1 : (cfg.automask() ? 2 * j : j)];
                            if (u == 0) keep[j] = raw[2 * j] <= th;  // clamp(max) passes where x <= max
                            val = fminf(val, th);
                        }
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
            if (pout) S.acc_photo += cfg.is_min() ? best : sum;
            const float g = gscale * mval;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const bool sel = cfg.is_min() ? (arg == (cfg.automask() ? 2 * j : j)) : true;
                G[j] = (sel && keep[j]) ? g : 0.0f;
            }
        }
        // smoothness terms of this p-row: forward sums (output pixels) and the carried
        // x / y gradient pieces (every real pixel; utils/depth.py:165-198)
        float h = 0.0f, t = 0.0f;
        if (cfg.smooth()) {
            const float c = S.template SG<IB>();
            if (pin && col < W - 1) {
                const float m = (fabsf(S.template Y<IB>()[0] - y_r[0]) + fabsf(S.template Y<IB>()[1] - y_r[1]) +
                                 fabsf(S.template Y<IB>()[2] - y_r[2])) * (1.0f / 3.0f);
                const float w = expf(-m);
                h = sgnf(c - sg_r) * w;
                if (pout) S.acc_ax += fabsf(c - sg_r) * w;
            }
            if (pin && pv < H - 1) {
                const float m = (fabsf(S.template Y<IB>()[0] - S.template Y<IC>()[0]) + fabsf(S.template Y<IB>()[1] - S.template Y<IC>()[1]) +
                                 fabsf(S.template Y<IB>()[2] - S.template Y<IC>()[2])) * (1.0f / 3.0f);
                const float w = expf(-m);
                t = sgnf(c - S.template SG<IC>()) * w;
                if (pout) S.acc_ay += fabsf(c - S.template SG<IC>()) * w;
            }
            if (pout) S.acc_m += c;
        }
        S.h_n = h;
        S.t_n = t;
        // coefficients of the selected candidates (G = 0 elsewhere), horizontally summed over the
        // 3 q-columns they touch (cross-lane: every lane active again here), then pushed into
        // dL/dx of the 3 q-rows: dx_c(q) += Ha_c + 2 x_c(q) Hb_c + y_c(q) He_c
        const float wyd = (pv == H - 1) ? 2.0f : 1.0f;  // p = row H-1 reflected onto q = row H-2
        const float wyu = (pv == 0) ? 2.0f : 1.0f;      // p = row 0 reflected onto q = row 1
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            const f2 Gq = f2{G[2 * q], (2 * q + 1 < NC) ? G[2 * q + 1] : 0.0f};
            const f2 kS = Gq * ((-0.5f / 27.0f) * p.ssim_w);
            const f2 kL = Gq * (l1w * (1.0f / 3.0f));
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                f2 ha = kS * cf[q][c], hb = kS * cf[q][3 + c], he = kS * cf[q][6 + c];
                hsum_w(ha, hb, he);
                const f2 xa = S.template X<IA>()[q][c], xb = S.template X<IB>()[q][c], xc = S.template X<IC>()[q][c];
                const f2 xa2 = xa + xa, xb2 = xb + xb, xc2 = xc + xc;
                S.D0[q][c] += wyd * (ha + xa2 * hb + S.template Y<IA>()[c] * he);
                const f2 db = xb - S.template Y<IB>()[c];
                S.D1[q][c] += (ha + xb2 * hb + S.template Y<IB>()[c] * he) + kL * f2{sgnf(db.x), sgnf(db.y)};
                S.D2[q][c] = wyu * (ha + xc2 * hb + S.template Y<IC>()[c] * he);
            }
        }
    }

    // weighted horizontal 3-sum: wxl * v[l-1] + v[l] + wxr * v[l+1] (cross-lane)
    __device__ __forceinline__ void hsum_w(f2& a0, f2& a1, f2& a2) const {
        f2 b0 = a0, b1 = a1, b2 = a2;
        hsum3x3(b0, b1, b2);
        if (border) {  // wave-uniform: only the stripes holding column 1 or W-2
            const float el = wxl - 1.0f, er = wxr - 1.0f;
            b0 += f2{el * from_prev(a0.x) + er * from_next(a0.x), el * from_prev(a0.y) + er * from_next(a0.y)};
            b1 += f2{el * from_prev(a1.x) + er * from_next(a1.x), el * from_prev(a1.y) + er * from_next(a1.y)};
            b2 += f2{el * from_prev(a2.x) + er * from_next(a2.x), el * from_prev(a2.y) + er * from_next(a2.y)};
        }
        a0 = b0;
        a1 = b1;
        a2 = b2;
    }

    // q-row qv from slot IQ (its dL/dx complete in S.D0); d warp / d(ix, iy) from LDS slot k % 3
    template <int IQ>
    __device__ __forceinline__ void qeval(State<NC>& S, int qv, int k) const {
        const float h_left = cfg.smooth() ? from_prev(S.h_p) : 0.0f;  // cross-lane
        if (qv >= H || qv >= y0 + RB || !qcol) return;
        float dv[NC * 6];
        di_load(k % 3, dv);
        const CM cams = load_cams();
        float d1, inv;
        const float d = dc.warp_depth(S.template SG<IQ>(), d1, inv);
        const float dw = dc.dwarp_ds(d, d1, inv);
        const Lift l = cams.lift((float)col, (float)qv, d);
        float gs = 0.0f;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const int q = j >> 1;
            float gix = 0.0f, giy = 0.0f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float dx = (j & 1) ? S.D0[q][c].y : S.D0[q][c].x;
                gix += dx * dv[j * 6 + c];
                giy += dx * dv[j * 6 + 3 + c];
            }
            typename CM::P pr;
            cams.project(j, l, pr);
            float gc[3];
            gs += cams.grad(j, pr, gix, giy, gc) * dw;
#if PSFM_K12_GT_REG
            acc_gT(S.gT[j], gc, pr);
#else
            {  // lane-private LDS row: 3 x b128 read-modify-write
                float4* g4 = reinterpret_cast<float4*>(gt + j * 12);
                float g[12];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const float4 t = g4[i];
                    g[4 * i] = t.x; g[4 * i + 1] = t.y; g[4 * i + 2] = t.z; g[4 * i + 3] = t.w;
                }
                acc_gT(g, gc, pr);
#pragma unroll
                for (int i = 0; i < 3; ++i) g4[i] = make_float4(g[4 * i], g[4 * i + 1], g[4 * i + 2], g[4 * i + 3]);
            }
#endif
        }
        if (cfg.smooth()) gs += (cx * (S.h_p - h_left) + cy * (S.t_p - S.t_pp)) / mc;
        gsig[(uint32_t)(qv * W + col)] = gs;
    }
};

template <int NC, bool FAST, int MODEL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PSFM_K12_WAVES))) void k12_fwd_grad(Args a) {
    extern __shared__ __attribute__((aligned(16))) float k12_lds[];
    const K12<NC, FAST, MODEL> K(a, k12_lds);
    constexpr int NP = (NC + 1) / 2;
    State<NC> S;
    S.acc_photo = S.acc_ax = S.acc_ay = S.acc_m = 0.0f;
    S.h_p = S.h_n = S.t_pp = S.t_p = S.t_n = 0.0f;
#pragma unroll
    for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int c = 0; c < 3; ++c) S.D0[q][c] = S.D1[q][c] = S.D2[q][c] = f2{0.0f, 0.0f};
#if PSFM_K12_GT_REG
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int m = 0; m < 12; ++m) S.gT[j][m] = 0.0f;
#else
#pragma unroll
    for (int m = 0; m < 12 * NC; ++m) K.gt[m] = 0.0f;
#endif
    // rows y0-2 .. y0+RB+1 issued at k = 0 .. RB+3; p-rows y0-1 .. y0+RB at k = 3 .. RB+4;
    // q-rows y0 .. y0+RB-1 at k = 5 .. RB+4 (the last step's issue is a harmless extra row)
    S.sg_next = K.load_sig(K.y0 - 2);
    K.template step<0, true, false, false>(S, 0);
    K.template step<1, true, false, false>(S, 1);
    K.template step<2, true, false, false>(S, 2);
    K.template step<3, true, true, false>(S, 3);
    K.template step<0, true, true, false>(S, 4);
#pragma unroll 1
    for (int k = 5; k < RB + 5; k += 4) {
        K.template step<1, true, true, true>(S, k);
        K.template step<2, true, true, true>(S, k + 1);
        K.template step<3, true, true, true>(S, k + 2);
        K.template step<0, true, true, true>(S, k + 3);
    }
    // per-wave partial sums (fixed-order wave butterflies)
    const psfm_params& p = a.p;
    const int nu = units(p.H, p.W);
    const float ph = wave_sum64(S.acc_photo);
    const float ax = wave_sum64(S.acc_ax), ay = wave_sum64(S.acc_ay), m = wave_sum64(S.acc_m);
    if (threadIdx.x == 0) {
        a.ws.photo_part[(size_t)K.s * (p.B * nu) + K.b * nu + K.unit] = ph;
        if (K.cfg.smooth()) {
            float* o = a.ws.smooth_part + (((size_t)K.s * p.B + K.b) * nu + K.unit) * 4;
            o[0] = ax;
            o[1] = ay;
            o[2] = m;
            o[3] = 0.0f;
        }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        float* o = a.ws.pose_part + ((((size_t)K.s * NC + j) * p.B + K.b) * nu + K.unit) * 12;
#pragma unroll
        for (int mm = 0; mm < 12; ++mm) {
#if PSFM_K12_GT_REG
            const float t = wave_sum64(S.gT[j][mm]);
#else
            const float t = wave_sum64(K.gt[j * 12 + mm]);
#endif
            if (threadIdx.x == 0) o[mm] = t;
        }
    }
}

}  // namespace fused
}  // namespace psfm
