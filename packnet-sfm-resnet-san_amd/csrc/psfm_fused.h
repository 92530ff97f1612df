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
// One wave per (60-column stripe, RB-row band, image, scale).  The (at most two) contexts of a
// target live in the two halves of 64-bit register pairs end to end: projection (pinhole: the
// camera records of both contexts interleaved by the prepass, ws.cam_pairs, so every camera
// entry is one SGPR pair operand of a v_pk_fma_f32), bilinear resolve, SSIM / L1, the SSIM
// adjoint, the bilinear and projection adjoints and the dL/d[R|t] accumulation are v_pk_*
// instructions for both contexts at once.  Lanes = columns c0-2..c0+61; the 60 inner lanes are
// outputs (a 3x3 SSIM window of a 3x3 neighbourhood: halo 2).  Step k of the sweep:
//   issue   row v = y0-2+k: target, sigmoid (prefetched one step earlier), lift/project and the
//           12 bilinear gathers per context (results consumed at the END of the step, so their
//           latency hides under the two evaluations below);
//   p-eval  row v-2: SSIM + L1 of both warped contexts (forward value AND the SSIM adjoint
//           coefficients d/d(mean x, E[x^2], E[xy])), automask candidates (K0 maps), min /
//           argmin (or mean), clip / mask, forward partial sums, smoothness forward terms; the
//           coefficients of the SELECTED candidate (G = 0 for the others) are accumulated
//           vertically into the three q-rows they touch (reflect weights at the image edge);
//   q-eval  row v-3 (its three p-rows are now complete): horizontal 3-sum of the accumulated
//           coefficients (DPP), adjoint through the bilinear sample (d warp / d(ix,iy) stashed
//           in wave-private LDS at issue time) and the projection — pinhole: from the issue's
//           stashed 1/z, warp depth and d warp / d sigmoid, p = d A [u, v, 1]^T + m (A = K_ref R K^-1,
//           PairProj) and dL/dd = dL/dp . dp/dd, no second depth chain or projection — dL/dp (X, 1)^T of both
//           contexts (taken through K_ref^T once per wave), plus the per-pixel smoothness
//           gradient -> dL/dsig written once (no LDS ring, no barrier, no atomics: deterministic);
//   resolve the bilinear samples of row v (x and d x/d(ix,iy)); the gathers are range-checked
//           raw buffer loads, so an out-of-bounds tap arrives as 0 (grid_sample's zero padding)
//           and needs neither a clamped address nor a mask.
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

// Phase boundaries of a sweep step (issue | p-eval | q-eval | resolve): the scheduler may not
// interleave the phases, so the register peak is the largest phase's, not their sum (the
// gathers issued in the first phase still fly under the next two: loads are asynchronous).
#define PSFM_PHASE() __builtin_amdgcn_sched_barrier(0)
// channel boundaries inside the SSIM phases: three unrolled channels interleaved by the
// scheduler triple the live temporaries (~40 VGPRs each)
#define PSFM_CHAN() __builtin_amdgcn_sched_barrier(0)
constexpr int WAVES = 2;         // waves per SIMD the register budget is sized for (<= 256 VGPRs)
// q (output) rows per band: chosen per launch among RB_LO / RB_HI by rb_for() (psfm_photometric.hip)
// from the wave count against the device's wave slots — a wave costs RB + 5 sweep steps
constexpr int RB_LO = 18, RB_HI = 28;
constexpr int OW = 60;           // output columns per stripe
constexpr int SIGCH = 16;        // chunks of the per-(scale, image) sigmoid sum pre-pass
constexpr int GTS = 28;          // per-lane dL/dT row: 12 entries x 2 contexts, padded to 28 dwords
                                 // (the 16 lanes of a b128 access start on distinct bank groups)

constexpr int PAIR_REC = 48;     // entries (f2: both contexts) of the context-paired camera record
                                 // ws.cam_pairs: Ki 0-8 | Kr 9-17 | T 18-29 | pad | E = Kr R Ki - I 32-40 |
                                 // m = Kr t 41-43 | pad (psfm_photometric.hip k_sig_sum builds it)

__host__ __device__ inline int stripes(int W) { return (W + OW - 1) / OW; }
__host__ __device__ inline int units(int H, int W, int rb) { return stripes(W) * ((H + rb - 1) / rb); }
// wave-private LDS (each lane touches only its own column: no barriers):
//   [3 row slots][6][64] f2  d warp / d(ix, iy) of both contexts | [64][GTS] dL/dT accumulators |
//   [4 row slots][64] float4  the issue phase's projection terms the q-eval reuses (pinhole: 1/z of
//   both contexts with the z-clamp pass in the sign, the warp depth, d warp / d sigmoid)
// 20 KB: 8 waves per CU (two per SIMD) fill the 160 KB exactly
__host__ __device__ inline size_t lds_bytes(int NC) {
    (void)NC;
    return ((size_t)3 * 6 * 64 * 2 + (size_t)GTS * 64 + (size_t)4 * 64 * 4) * sizeof(float);
}

// Optional per-wave timestamps (psfm_k12_stamps): when set, lane 0 of every wave writes the
// constant 100 MHz real-time clock at its start and its end to p[2 L], p[2 L + 1] (L = linear
// workgroup id < cap) with vector stores.  A device global, not a kernel argument, so a captured
// step graph can be timed in place: bench.py reads K12's in-step span from it.
struct StampBuf {
    unsigned long long* p;
    int cap;
};
__device__ StampBuf g_k12_stamp;

__device__ __forceinline__ void k12_stamp(int slot) {
    const StampBuf sb = g_k12_stamp;
    if (sb.p == nullptr) return;  // wave-uniform
    const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    int tid = threadIdx.x;   // laundered: a lane-0 mask shared with the prologue was kept across the sweep
    asm volatile("" : "+v"(tid));
    if (L < sb.cap && tid == 0) sb.p[2 * L + slot] = t;
}

struct Args {
    psfm_params p;
    psfm_inputs in;
    psfm_workspace ws;
    float* grad_sig[PSFM_MAX_SCALES];
    // Wave-pair balance (psfm_photometric.hip k12_priority): the workgroups of an XCD are dealt
    // round-robin to its SIMDs, so in a one-round launch the in-XCD index i = L >> 3 >= young_from
    // (= the XCD's SIMD count) marks the SECOND wave on its SIMD, which loses every VALU
    // arbitration tie to the older one by age.  prio_mode 2: the younger wave runs one priority
    // level higher in the p-eval; 0: off.
    int young_from, prio_mode;
    int xcd_parts;   // sweep::work_item_parts: parts per image in an XCD's run (k12_dealing)
};

__device__ __forceinline__ f2 bc(float v) { return f2{v, v}; }   // both halves (op_sel broadcast)
__device__ __forceinline__ f2 mask01(bool a, bool b) { return f2{a ? 1.0f : 0.0f, b ? 1.0f : 0.0f}; }

// Bilinear gathers in flight for one context (issued at the top of a step, resolved at its end).
struct Pend {
    float q[3][4];
    float ax, bx, ay, by;
};

// The context image of (b) as a range-checked buffer: V# with the image's 3 planes as num_records,
// stride 0 (raw), gfx9 dword3.  A raw buffer load whose offset lies past num_records returns 0, which
// is grid_sample's zero padding of an out-of-bounds tap (padding_mode='zeros'): the 12 gathers need
// no coordinate clamps and the resolve no per-channel tap masks.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t img_rsrc(const float* img, uint32_t pb) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0, (int)(3u * pb), 0x00020000);
}

// one tap's byte offset when valid, else past the buffer (channel c adds c * pb as the SGPR offset:
// the result stays past 3 * pb either way the hardware counts it)
constexpr uint32_t TAP_OOB = 0x80000000u;

__device__ __forceinline__ void gather(__amdgpu_buffer_rsrc_t rs, uint32_t pb, float ix, float iy, int H, int W,
                                       Pend& g) {
    // some tap may be in bounds iff ix in [-1, W) (and y alike); the wider open interval keeps the
    // float -> int conversion defined (and rejects NaN): outside it every tap is out of bounds
    const bool ok = (ix > -2.0f) && (ix < (float)W + 1.0f) && (iy > -2.0f) && (iy < (float)H + 1.0f);
    const float fx0 = floorf(ix), fy0 = floorf(iy);
    const int x0 = ok ? (int)fx0 : -2, y0 = ok ? (int)fy0 : -2;
    const bool xw = (unsigned)x0 < (unsigned)W, xe = (unsigned)(x0 + 1) < (unsigned)W;
    const bool yn = (unsigned)y0 < (unsigned)H, ys = (unsigned)(y0 + 1) < (unsigned)H;
    const uint32_t o = (uint32_t)(y0 * W + x0) * 4u, row = (uint32_t)W * 4u;
    const uint32_t onw = (yn && xw) ? o : TAP_OOB, one = (yn && xe) ? o + 4u : TAP_OOB;
    const uint32_t osw = (ys && xw) ? o + row : TAP_OOB, ose = (ys && xe) ? o + row + 4u : TAP_OOB;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int so = (int)(c * pb);
        g.q[c][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, onw, so, 0));
        g.q[c][1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, one, so, 0));
        g.q[c][2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, osw, so, 0));
        g.q[c][3] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, ose, so, 0));
    }
    g.ax = (fx0 + 1.0f) - ix;
    g.bx = ix - fx0;
    g.ay = (fy0 + 1.0f) - iy;
    g.by = iy - fy0;
}

// grid_sample value and d/d(ix), d/d(iy) of one context (same arithmetic as sweep::bilinear3_vd;
// out-of-bounds taps arrived as 0)
__device__ __forceinline__ void resolve1(const Pend& g, float v[3], float dix[3], float diy[3]) {
    const float wnw = g.ax * g.ay, wne = g.bx * g.ay, wsw = g.ax * g.by, wse = g.bx * g.by;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float nw = g.q[c][0], ne = g.q[c][1], sw = g.q[c][2], se = g.q[c][3];
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
__device__ __forceinline__ void resolve_pair(const Pend& a, const Pend& b, f2 (&v)[3], f2 (&dix)[3],
                                             f2 (&diy)[3]) {
    float va[3], xa[3], ya[3], vb[3], xb[3], yb[3];
    resolve1(a, va, xa, ya);
    resolve1(b, vb, xb, yb);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        v[c] = f2{va[c], vb[c]};
        dix[c] = f2{xa[c], xb[c]};
        diy[c] = f2{ya[c], yb[c]};
    }
}

// ---------------------------------------------------------------------------------------------
// Pinhole projection of both contexts at once (Camera.reconstruct -> Pose -> Camera.project ->
// grid_sample's normalise / unnormalise round trip, geometry/camera.py:111-190), from the
// context-paired record of (s, b): entry k = (context 0, context 1) floats 2k, 2k+1.
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(4))) const f2 cf2;

// The pinhole pair record at run time.  Lift, transform and intrinsics fold into one 3x3 per
// context, A = K_ref R K^-1:  p = K_ref (R (d K^-1 x) + t) = d A x + m, x = [u, v, 1]^T, m = K_ref t.
// The record holds E = A - I (fp64, rounded once) and p is evaluated as p = d (E x) + (d x + m):
// E x is small (the image motion per unit depth) and d x + m is one rounding at the magnitude of p,
// which halves the sampling positions' fp32 error against the lift + R X + t + K_ref chain
// (max 1.4-1.8e-4 px vs 3.0-5.5e-4, mean 1.0e-5 vs 1.6e-5 over 1M KITTI-shaped points).  A lane's
// column u is fixed for the whole sweep, so E's u- and constant columns are folded once per wave
// (K12::ea) and a row costs e = ea + E[:, 1] v and two fma per entry of p: nine v_pk_fma for both
// contexts, where the chain took 9 + 21.  The adjoint needs no intermediate point either:
// dL/dd = dL/dp . dp/dd = dL/dp . (e + x).  dL/d[R|t] is accumulated as dL/dp (X, 1)^T and taken
// through K_ref^T once per wave (bwd_pose_rows).
struct PairProj {
    f2 p0, p1, p2;  // K_ref (R X + t)
    f2 iz;          // 1 / clamp(p2, 1e-5)
    f2 ix, iy;      // sampling position in pixels
};

__device__ __forceinline__ f2 roundtrip(f2 pz, float sm1, float rsm1) {
    const f2 t = pz + pz;
    f2 q = t * bc(rsm1);
    q = (t - q * bc(sm1)) * bc(rsm1) + q;
    const f2 n = q - f2{1.0f, 1.0f};
    return ((n + f2{1.0f, 1.0f}) * f2{0.5f, 0.5f}) * bc(sm1);
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
        const f2 lc = f2{__builtin_amdgcn_fmed3f(l.x, 0.0f, 1.0f), __builtin_amdgcn_fmed3f(l.y, 0.0f, 1.0f)};
        ls += lc;
        // adjoint coefficients with the clamp pass (l inside [0, 1]: the clamped value is l; NaN fails)
        // folded into the common factor u = pass / D:  dSSIM/dmx = 2 u (my (A2 - A1) - mx (Nn / D) (B2 - B1)),
        // dSSIM/dE[x^2] = -(Nn / D) B1 u, dSSIM/dE[xy] = 2 A1 u
        const f2 u = f2{lc.x == l.x ? iD.x : 0.0f, lc.y == l.y ? iD.y : 0.0f};
        const f2 u2 = u + u, q = Nn * iD;
        cf[c] = u2 * (my * (A2 - A1) - (mx * q) * (B2 - B1));
        cf[3 + c] = -(q * B1) * u;
        cf[6 + c] = A1 * u2;
        const f2 dd = xb[c] - yb[c];
        l1 += f2{fabsf(dd.x), fabsf(dd.y)};
        PSFM_CHAN();
    }
    return ssim_w * (ls * (1.0f / 3.0f)) + l1w * (l1 * (1.0f / 3.0f));
}

template <int NC>
struct State {
    static constexpr int NP = 1;
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
    // dL/d(warped sample) per channel (the contexts packed) of the q-rows a p-row touches:
    // D0 = row p-1 (completed by this p-row), D1 = row p, D2 = row p+1
    f2 D0[NP][3], D1[NP][3], D2[NP][3];
    float h_p, h_n;           // smoothness x-term sgn(s - s_right) w of p-row q / this p-row
    float t_pp, t_p, t_n;     // y-term sgn(s - s_below) w of p-rows q-1, q, this p-row
    float acc_photo, acc_ax, acc_ay, acc_m;
};

template <int NC, bool FAST, int MODEL, int RB>
struct K12 {
    static_assert(NC == 1 || NC == 2, "K12: one context pair (N <= 2, fused_ok)");
    static constexpr bool PAIR_CAM = MODEL == PSFM_CAM_PINHOLE;  // packed pinhole projection
    using CM = Cams<NC, MODEL>;
    static constexpr int NP = 1;
    const Args& a;
    const psfm_params& p;
    Cfg<FAST> cfg;
    int H, W, B, b, s, unit, y0, col, colr, lane;
    int sh, Ws, colc;  // sigmoid storage: (H >> sh, W >> sh), this lane's stored column
    uint32_t plane, pb;
    bool pcol, qcol, border_l, border_r;
    DepthChain dc;
    float l1w, gscale, cx, cy, mc, rmc, wxl, wxr;
    const float* tgt;
    const float* sig;
    const float* ctx[NC];
    const float* thr;
    const float* mask;
    float* gsig;
    f2* di;      // wave-private LDS [3][6][64] f2
    float* gt;   // this lane's dL/dT accumulators: gt[2 m + j] (entry m, context j), 16-B aligned;
                 // pinhole: dL/dp (X, 1)^T (K_ref^T applied per wave at the end), fisheye: dL/d[R|t]
    float4* stash;  // wave-private LDS [4][64]: the issue phase's projection terms for the q-eval
    const float* camrec;   // record of (s, context 0, b); context j is j*B records further
    const float* campair;  // context-paired record of (s, b) (ws.cam_pairs)
    f2 ea[3];              // pinhole: E[:, 0] u + E[:, 2] of this lane's column u (PairProj)
    float xa[3];           // pinhole: K^-1[:, 0] u + K^-1[:, 2] (the point X = d K^-1 [u, v, 1]^T)
    bool young;            // the second wave dispatched to its SIMD (Args::young_from), wave-uniform
    int prio_mode;

    // phase priorities: 2 (issue / q-eval / resolve) and 0 (p-eval), the younger wave of a SIMD
    // pair one level up in its p-eval (Args::prio_mode 2; the round-4 mode 1, younger +1 in every
    // phase, only put a wave-uniform branch around each setprio: profiles/r05/k12/variants_ab.log,
    // 97.7 -> 96.5 us per launch without it)
    __device__ __forceinline__ void prio_hi() const { __builtin_amdgcn_s_setprio(2); }
    __device__ __forceinline__ void prio_lo() const {
        if (young) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    }

    // Camera scalars are re-loaded at each use (s_load through the constant address space:
    // scalar cache, no VGPRs) instead of being held in SGPRs for the whole sweep; the laundered
    // pointer stops the compiler from keeping them live across the SSIM phase.
    __device__ __forceinline__ CM load_cams() const {
        uint64_t rp = reinterpret_cast<uint64_t>(camrec);
        asm volatile("" : "+s"(rp));
        CM c;
        c.load(reinterpret_cast<cfloat*>(rp), B, H, W);
        return c;
    }
    // the context-paired pinhole record, read (s_load through the scalar cache) at each use: held
    // across the phases its entries lived in SGPRs spilled to VGPR lanes, and every use cost a
    // v_readlane per dword (profiles/r06/k12/kab_noslp.log: 90.9 -> 90.2-90.5 us)
    __device__ __forceinline__ cf2* pair_rec() const {
        uint64_t rp = reinterpret_cast<uint64_t>(campair);
        asm volatile("" : "+s"(rp));
        return reinterpret_cast<cf2*>(rp);
    }
    // e = E [u, v, 1]^T of this lane at row v and p = d e + (d [u, v, 1]^T + m) (both contexts)
    __device__ __forceinline__ void pair_p(cf2* rec, float v, float d, f2 (&e)[3], f2 (&p)[3]) const {
        const f2 vv = bc(v), dd = bc(d);
#pragma unroll
        for (int k = 0; k < 3; ++k) e[k] = rec[33 + 3 * k] * vv + ea[k];
        p[0] = e[0] * dd + (dd * bc((float)colr) + rec[41]);
        p[1] = e[1] * dd + (dd * vv + rec[42]);
        p[2] = e[2] * dd + (dd + rec[43]);
    }

    __device__ __forceinline__ K12(const Args& a_, float* lds) : a(a_), p(a_.p), cfg{a_.p} {
        H = p.H;
        W = p.W;
        B = p.B;
        plane = (uint32_t)(H * W);
        pb = plane * 4u;
        const int nst = stripes(W);
        const sweep::WorkItem wi = sweep::work_item_parts(a_.xcd_parts);
        b = wi.b;
        s = wi.s;
        unit = wi.unit;
        lane = threadIdx.x;
        prio_mode = a_.prio_mode;
        {
            const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
            young = prio_mode != 0 && (L >> 3) >= a_.young_from;
        }
        y0 = (unit / nst) * RB;
        const int c0 = (unit % nst) * OW;
        col = c0 - 2 + lane;
        colr = reflect1(col, W);
        pcol = lane >= 1 && lane <= OW + 2 && col >= 0 && col < W;
        qcol = lane >= 2 && lane <= OW + 1 && col < W;
        border_l = c0 <= 1;                    // this stripe holds column 1
        border_r = c0 + OW >= W - 2;           // ... or column W-2
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
        di = reinterpret_cast<f2*>(lds);
        gt = lds + 3 * 6 * 64 * 2 + lane * GTS;
        stash = reinterpret_cast<float4*>(lds + 3 * 6 * 64 * 2 + GTS * 64);
        camrec = a.in.cam + ((size_t)s * NC * B + b) * PSFM_CAMREC;
        campair = a.ws.cam_pairs + ((size_t)s * B + b) * 2 * PAIR_REC;
        // per-image mean of the sigmoid map (smoothness normaliser, utils/depth.py:183-185),
        // from the SIGCH chunk sums of the pre-pass, summed in chunk order in fp64 (wave-uniform
        // scalar loads: written by the previous launch, read-only here)
        mc = 1.0f;
        if (cfg.smooth()) {
            cfloat* sp = reinterpret_cast<cfloat*>(reinterpret_cast<uint64_t>(a.ws.sig_part) +
                                                   (((size_t)s * B + b) * SIGCH) * sizeof(float));
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < SIGCH; ++i) v += (double)sp[i];
            mc = fmaxf((float)(v / ((double)H * W)), 1e-6f);
        }
        rmc = 1.0f / mc;   // once per wave: the q-eval multiplies (within 1 ulp of dividing)
        if constexpr (PAIR_CAM) {
            cf2* rec = reinterpret_cast<cf2*>(reinterpret_cast<uint64_t>(campair));
            const float u = (float)colr;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                ea[k] = rec[32 + 3 * k] * bc(u) + rec[34 + 3 * k];
                xa[k] = rec[3 * k].x * u + rec[3 * k + 2].x;
            }
        }
    }

    // d warp / d(ix, iy) of a row slot, both contexts: [slot][m][64] f2 (b64, conflict-free)
    __device__ __forceinline__ void di_store(int slot, const f2 (&dv)[6]) const {
        f2* ds = di + slot * (6 * 64);
#pragma unroll
        for (int m = 0; m < 6; ++m) ds[m * 64 + lane] = dv[m];
    }
    __device__ __forceinline__ void di_load(int slot, f2 (&dv)[6]) const {
        const f2* ds = di + slot * (6 * 64);
#pragma unroll
        for (int m = 0; m < 6; ++m) dv[m] = ds[m * 64 + lane];
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
            // unconditional loads from a clamped address, the selection after: a load under a
            // lane-divergent branch makes the wait-count pass merge its paths pessimistically, and
            // the p-eval then waited for every gather of the step (s_waitcnt vmcnt(0))
            const int pv = v - 2;
            const bool pin = pcol && pv >= 0 && pv < H;
            const uint32_t ppix = (uint32_t)(min(max(pv, 0), H - 1) * W + min(max(col, 0), W - 1));
            if (cfg.automask()) {
#pragma unroll
                for (int j = 0; j < NC; ++j) {
                    const float u = a.ws.unwarp[((size_t)j * B + b) * plane + ppix];
                    S.un[j] = pin ? u : 0.0f;
                }
            } else {
#pragma unroll
                for (int j = 0; j < NC; ++j) S.un[j] = 0.0f;
            }
            if (mask) {
                const float mv = mask[ppix];
                S.mv = pin ? mv : 1.0f;
            } else {
                S.mv = 1.0f;
            }
        }
        // wave priority (two waves share a SIMD): everything but the long p-eval — the q-eval (an
        // LDS read-modify-write chain), the resolve and the next issue (its gathers go out first) —
        // runs at priority 2, the p-eval at 0, so the other wave's p-eval fills the latency
        // (kbench B=4 104.7-105.8 -> 98.4 us, B=6 146-147 -> 138 us; profiles/r03/k12ab)
        prio_hi();
        if (LOAD) {
            const float sg = S.sg_next;
            S.sg_next = load_sig(v + 1);
            S.template SG<I>() = sg;
            const int r = reflect1(v, H);
            const uint32_t pix = (uint32_t)(r * W + colr);
#pragma unroll
            for (int c = 0; c < 3; ++c) S.template Y<I>()[c] = tgt[c * plane + pix];
            float d1, inv;
            const float d = dc.warp_depth(sg, d1, inv);
            if constexpr (PAIR_CAM) {
                // p = d A [u, v, 1]^T + m, z = clamp(p2, 1e-5), 1/z (rcp + one Newton step), u = p0 / z
                // (rcp-refined quotient), then grid_sample's ((2u/(W-1) - 1) + 1)/2 (W-1) round trip
                f2 e[3], pp[3];
                pair_p(pair_rec(), (float)r, d, e, pp);
                PairProj pr;
                pr.p0 = pp[0];
                pr.p1 = pp[1];
                pr.p2 = pp[2];
                const f2 z = f2{fmaxf(pr.p2.x, 1e-5f), fmaxf(pr.p2.y, 1e-5f)};
                const f2 r0 = f2{__builtin_amdgcn_rcpf(z.x), __builtin_amdgcn_rcpf(z.y)};
                pr.iz = (f2{1.0f, 1.0f} - z * r0) * r0 + r0;
                f2 pu = pr.p0 * pr.iz, pv = pr.p1 * pr.iz;
                pu = (pr.p0 - pu * z) * pr.iz + pu;
                pv = (pr.p1 - pv * z) * pr.iz + pv;
                const float wm1 = (float)(W - 1), hm1 = (float)(H - 1);
                pr.ix = roundtrip(pu, wm1, rcp_nr(wm1));
                pr.iy = roundtrip(pv, hm1, rcp_nr(hm1));
                gather(img_rsrc(ctx[0], pb), pb, pr.ix.x, pr.iy.x, H, W, pd[0]);
                if (NC == 2) gather(img_rsrc(ctx[NC - 1], pb), pb, pr.ix.y, pr.iy.y, H, W, pd[NC - 1]);
                // what the q-eval of this row (step k + 3, slot I) takes from here instead of
                // re-running the depth chain and the projection: 1/z of both contexts (negated where
                // z = p2 was clamped: no gradient through it), the warp depth, d warp / d sigmoid
                stash[I * 64 + lane] = make_float4(pr.p2.x >= 1e-5f ? pr.iz.x : -pr.iz.x,
                                                   pr.p2.y >= 1e-5f ? pr.iz.y : -pr.iz.y, d, dc.dwarp_ds(d, d1, inv));
            } else {
                const CM cams = load_cams();
                const Lift l = cams.lift((float)colr, (float)r, d);
#pragma unroll
                for (int j = 0; j < NC; ++j) {
                    typename CM::P pr;
                    cams.project(j, l, pr);
                    gather(img_rsrc(ctx[j], pb), pb, pr.ix, pr.iy, H, W, pd[j]);
                }
            }
        }
        prio_lo();
        PSFM_PHASE();
        if (PEVAL) peval<IA, IB, IC>(S, v - 2);
        PSFM_PHASE();
        prio_hi();
        if (QEVAL) qeval<IA>(S, v - 3, k);
        PSFM_PHASE();
        if (PEVAL) {  // rotate the carried per-row terms
            S.t_pp = S.t_p;
            S.t_p = S.t_n;
            S.h_p = S.h_n;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                S.D0[0][c] = S.D1[0][c];
                S.D1[0][c] = S.D2[0][c];
            }
        }
        if (LOAD) resolve_row<I>(S, k, pd);
    }

    // the bilinear samples of the issued row (the duplicate context of NC = 1 is computed in the
    // high half and never read)
    template <int I>
    __device__ __forceinline__ void resolve_row(State<NC>& S, int k, const Pend (&pd)[NC]) const {
        f2 x[3], dix[3], diy[3];
        resolve_pair(pd[0], pd[NC - 1], x, dix, diy);
        f2 dv[6];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            S.template X<I>()[0][c] = x[c];
            dv[c] = dix[c];
            dv[3 + c] = diy[c];
        }
        di_store(k % 3, dv);
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
                const float w = __expf(-m);   // v_exp_f32(-m log2 e): m in [0, 1], within 2 ulp of expf
                h = sgnf(c - sg_r) * w;
                if (pout) S.acc_ax += fabsf(c - sg_r) * w;
            }
            if (pin && pv < H - 1) {
                const float m = (fabsf(S.template Y<IB>()[0] - S.template Y<IC>()[0]) + fabsf(S.template Y<IB>()[1] - S.template Y<IC>()[1]) +
                                 fabsf(S.template Y<IB>()[2] - S.template Y<IC>()[2])) * (1.0f / 3.0f);
                const float w = __expf(-m);   // v_exp_f32(-m log2 e): m in [0, 1], within 2 ulp of expf
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
            const f2 kS2 = kS + kS;   // the E[x^2] term's factor 2 (d x^2 / dx = 2 x) on the coefficient:
                                      // (x + x) hb == x (2 hb) exactly
            const f2 kL = Gq * (l1w * (1.0f / 3.0f));
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                f2 ha = kS * cf[q][c], hb = kS2 * cf[q][3 + c], he = kS * cf[q][6 + c];
                hsum_w(ha, hb, he);
                const f2 xa = S.template X<IA>()[q][c], xb = S.template X<IB>()[q][c], xc = S.template X<IC>()[q][c];
                S.D0[q][c] += wyd * (ha + xa * hb + S.template Y<IA>()[c] * he);
                const f2 db = xb - S.template Y<IB>()[c];
                S.D1[q][c] += (ha + xb * hb + S.template Y<IB>()[c] * he) + kL * f2{sgnf(db.x), sgnf(db.y)};
                S.D2[q][c] = wyu * (ha + xc * hb + S.template Y<IC>()[c] * he);
            }
        }
    }

    // weighted horizontal 3-sum: wxl * v[l-1] + v[l] + wxr * v[l+1] (cross-lane)
    __device__ __forceinline__ void hsum_w(f2& a0, f2& a1, f2& a2) const {
        f2 b0 = a0, b1 = a1, b2 = a2;
        hsum3x3(b0, b1, b2);
        // wave-uniform: only the stripes holding column 1 / W-2, and only that side's term (a border
        // wave doing both sides' DPP terms ran 4-5 % longer than an interior one and set the span:
        // profiles/r04/prio/stamps_mode2.txt)
        if (border_l) {
            const float el = wxl - 1.0f;
            b0 += f2{el * from_prev(a0.x), el * from_prev(a0.y)};
            b1 += f2{el * from_prev(a1.x), el * from_prev(a1.y)};
            b2 += f2{el * from_prev(a2.x), el * from_prev(a2.y)};
        }
        if (border_r) {
            const float er = wxr - 1.0f;
            b0 += f2{er * from_next(a0.x), er * from_next(a0.y)};
            b1 += f2{er * from_next(a1.x), er * from_next(a1.y)};
            b2 += f2{er * from_next(a2.x), er * from_next(a2.y)};
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
        f2 dv[6];
        di_load(k % 3, dv);
        // dL/d(ix, iy) of both contexts: the channels' dL/dx through d warp / d(ix, iy)
        f2 gix = S.D0[0][0] * dv[0], giy = S.D0[0][0] * dv[3];
#pragma unroll
        for (int c = 1; c < 3; ++c) {
            gix += S.D0[0][c] * dv[c];
            giy += S.D0[0][c] * dv[3 + c];
        }
        float gs;
        if constexpr (PAIR_CAM) {
            // the row's 1/z, warp depth and d warp / d sigmoid from its issue (stash slot IQ); the
            // projection's first two rows again as p = d w + m (PairProj), and the adjoint
            // (camera.py:111-190): dL/dp -> dL/d(depth) = dL/dp . w; dL/dp (X, 1)^T accumulated for dL/d[R|t]
            const float4 st = stash[IQ * 64 + lane];
            const float d = st.z, dw = st.w;
            cf2* rec = pair_rec();
            const float qf = (float)qv;
            f2 e[3], pp[3];
            pair_p(rec, qf, d, e, pp);
            const f2 p0 = pp[0], p1 = pp[1];
            const f2 iz = f2{fabsf(st.x), fabsf(st.y)};
            const f2 t = -(gix * p0 + giy * p1) * (iz * iz);
            f2 gp[3];
            gp[0] = gix * iz;
            gp[1] = giy * iz;
            gp[2] = f2{st.x > 0.0f ? t.x : 0.0f, st.y > 0.0f ? t.y : 0.0f};
            // dp/dd = E x + x
            const f2 gd = gp[0] * (e[0] + bc((float)colr)) + gp[1] * (e[1] + bc(qf)) + gp[2] * (e[2] + f2{1.0f, 1.0f});
            gs = (NC == 2 ? gd.x + gd.y : gd.x) * dw;
            // X = d K^-1 [u, v, 1]^T
            const f2 X0 = bc((rec[1].x * qf + xa[0]) * d), X1 = bc((rec[4].x * qf + xa[1]) * d),
                     X2 = bc((rec[7].x * qf + xa[2]) * d);
            // G += dL/dp (X, 1)^T for both contexts: lane-private LDS row, b128 read-modify-write
            float4* g4 = reinterpret_cast<float4*>(gt);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const float4 ta = g4[2 * i], tb = g4[2 * i + 1];
                f2 e0 = f2{ta.x, ta.y}, e1 = f2{ta.z, ta.w}, e2 = f2{tb.x, tb.y}, e3 = f2{tb.z, tb.w};
                e0 += gp[i] * X0;
                e1 += gp[i] * X1;
                e2 += gp[i] * X2;
                e3 += gp[i];
                g4[2 * i] = make_float4(e0.x, e0.y, e1.x, e1.y);
                g4[2 * i + 1] = make_float4(e2.x, e2.y, e3.x, e3.y);
            }
        } else {
            float d1, inv;
            const float d = dc.warp_depth(S.template SG<IQ>(), d1, inv);
            const float dw = dc.dwarp_ds(d, d1, inv);
            const CM cams = load_cams();
            const Lift l = cams.lift((float)col, (float)qv, d);
            gs = 0.0f;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                typename CM::P pr;
                cams.project(j, l, pr);
                float gc[3];
                gs += cams.grad(j, pr, j ? gix.y : gix.x, j ? giy.y : giy.x, gc) * dw;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    gt[2 * (4 * i + 0) + j] += gc[i] * pr.X0;
                    gt[2 * (4 * i + 1) + j] += gc[i] * pr.X1;
                    gt[2 * (4 * i + 2) + j] += gc[i] * pr.X2;
                    gt[2 * (4 * i + 3) + j] += gc[i];
                }
            }
        }
        if (cfg.smooth()) gs += (cx * (S.h_p - h_left) + cy * (S.t_p - S.t_pp)) * rmc;
        gsig[(uint32_t)(qv * W + col)] = gs;
    }
};

template <int NC, bool FAST, int MODEL, int RB>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WAVES))) void k12_fwd_grad(Args a) {
    static_assert(RB >= 4, "K12 band height");
    k12_stamp(0);
    extern __shared__ __attribute__((aligned(16))) float k12_lds[];
    const K12<NC, FAST, MODEL, RB> K(a, k12_lds);
    State<NC> S;
    S.acc_photo = S.acc_ax = S.acc_ay = S.acc_m = 0.0f;
    S.h_p = S.h_n = S.t_pp = S.t_p = S.t_n = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) S.D0[0][c] = S.D1[0][c] = S.D2[0][c] = f2{0.0f, 0.0f};
#pragma unroll
    for (int m = 0; m < 24; ++m) K.gt[m] = 0.0f;
    // the work item (scale, image, unit), which only the partial-sum stores after the sweep need, parked
    // in lane 0's dL/dT row padding (dwords 24-26 of the GTS = 28) instead of SGPRs across the sweep
    if (threadIdx.x == 0) {
        int* pad = reinterpret_cast<int*>(K.gt) + 24;
        pad[0] = K.s;
        pad[1] = K.b;
        pad[2] = K.unit;
    }
    // rows y0-2 .. y0+RB+1 issued at k = 0 .. RB+3; p-rows y0-1 .. y0+RB at k = 3 .. RB+4;
    // q-rows y0 .. y0+RB-1 at k = 5 .. RB+4.  Step k uses row slot k & 3; the loop leaves after
    // step RB+4 (wave-uniform branches, any RB).  That step's issue is a harmless extra row (reflect-
    // clamped reads): skipping it behind a branch made the wait-count pass merge a path without the
    // gathers, and every p-eval then waited for all of its step's gathers (s_waitcnt vmcnt(0))
    constexpr int KE = RB + 4;
    S.sg_next = K.load_sig(K.y0 - 2);
    K.template step<0, true, false, false>(S, 0);
    K.template step<1, true, false, false>(S, 1);
    K.template step<2, true, false, false>(S, 2);
    K.template step<3, true, true, false>(S, 3);
    K.template step<0, true, true, false>(S, 4);
#pragma unroll 1
    for (int k0 = 5;; k0 += 4) {
        // opaque step index: no loop-carried strength-reduced addresses (each one an SGPR that the
        // sweep's register peak spills to VGPR lanes and re-loads every step)
        int k = k0;
        asm volatile("" : "+s"(k));
        K.template step<1, true, true, true>(S, k);
        if (k == KE) break;
        K.template step<2, true, true, true>(S, k + 1);
        if (k + 1 == KE) break;
        K.template step<3, true, true, true>(S, k + 2);
        if (k + 2 == KE) break;
        K.template step<0, true, true, true>(S, k + 3);
        if (k + 3 == KE) break;
    }
    // per-wave partial sums (fixed-order wave butterflies).  The output pointers are read here, after the
    // sweep, through a laundered kernarg pointer: read as plain arguments they were loaded in the
    // prologue and held across the sweep in SGPRs spilled to VGPR lanes
    const psfm_params& p = a.p;
    const int nu = units(p.H, p.W, RB);
    uint64_t kp = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());   // `a`: offset 0
    asm volatile("" : "+s"(kp));
    const __attribute__((address_space(4))) Args* ka = reinterpret_cast<const __attribute__((address_space(4))) Args*>(kp);
    const int* pad = reinterpret_cast<const int*>(k12_lds + 3 * 6 * 64 * 2) + 24;   // lane 0's row
    const int ws_ = __builtin_amdgcn_readfirstlane(pad[0]), wb = __builtin_amdgcn_readfirstlane(pad[1]),
              wu = __builtin_amdgcn_readfirstlane(pad[2]);
    int tid = threadIdx.x;   // re-derived: the prologue's lane-0 mask was kept across the sweep too
    asm volatile("" : "+v"(tid));
    const float ph = wave_sum64(S.acc_photo);
    const float ax = wave_sum64(S.acc_ax), ay = wave_sum64(S.acc_ay), m = wave_sum64(S.acc_m);
    if (tid == 0) {
        ka->ws.photo_part[(size_t)ws_ * (p.B * nu) + wb * nu + wu] = ph;
        if (K.cfg.smooth()) {
            float* o = ka->ws.smooth_part + (((size_t)ws_ * p.B + wb) * nu + wu) * 4;
            o[0] = ax;
            o[1] = ay;
            o[2] = m;
            o[3] = 0.0f;
        }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        float* o = ka->ws.pose_part + ((((size_t)ws_ * NC + j) * p.B + wb) * nu + wu) * 12;
        float t[12];
#pragma unroll
        for (int mm = 0; mm < 12; ++mm) t[mm] = wave_sum64(K.gt[2 * mm + j]);
        if constexpr (K12<NC, FAST, MODEL, RB>::PAIR_CAM) {
            // dL/d[R|t] row r' = sum_r K_ref[r][r'] G[r] (G = sum dL/dp (X, 1)^T, rows r of p)
            cf2* rec = reinterpret_cast<cf2*>(reinterpret_cast<uint64_t>(K.campair));
            float Kr[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) Kr[i] = j ? rec[9 + i].y : rec[9 + i].x;
            float u[12];
#pragma unroll
            for (int r2 = 0; r2 < 3; ++r2)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    u[4 * r2 + c] = Kr[r2] * t[c] + Kr[3 + r2] * t[4 + c] + Kr[6 + r2] * t[8 + c];
#pragma unroll
            for (int mm = 0; mm < 12; ++mm) t[mm] = u[mm];
        }
        if (tid == 0) {
#pragma unroll
            for (int mm = 0; mm < 12; ++mm) o[mm] = t[mm];
        }
    }
    k12_stamp(1);
}

}  // namespace fused
}  // namespace psfm
