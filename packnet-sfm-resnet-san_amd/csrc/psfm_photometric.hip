// psfm_photometric.hip — fused view-synthesis + SSIM/L1 + min-reprojection + smoothness
// kernels for MI355X (gfx950), behind the C-ABI of include/psfm.h.
//
// Reference op chain replaced (paths relative to the reference's packnet_sfm/):
//   losses/multiview_photometric_loss.py:331-410 (forward), :131-195 (warp_ref_image),
//   :15-54 + :199-267 (SSIM, calc_photometric_loss), :269-297 (reduce_photometric_loss),
//   :301-327 + utils/depth.py:146-198 (smoothness), geometry/camera.py:111-190,
//   geometry/camera_utils.py:27-59 (view_synthesis), and the autograd backward of all of it.
//
// Design: one 256-thread workgroup owns a 64x4 tile of output pixels of
// one image.  K1 (forward) stages the target and each warped/unwarped candidate image of the
// tile + 1-pixel reflect halo in LDS, evaluates the 3x3 SSIM windows from LDS, keeps the
// candidates of a scale in registers and reduces min/argmin in-register; per-tile partial
// sums go to a workspace and a single finalize kernel reduces them in a fixed order
// (bitwise deterministic, no float atomics).  K2 (backward) recomputes the warp on a
// 2-pixel halo, forms the SSIM adjoint coefficients on a 1-pixel halo in LDS and gathers
// them (reflect-aware weights) per pixel, then back-propagates through bilinear sampling and
// the projection; dL/d[R|t] is reduced per tile (wave butterfly + fixed-order wave sum).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "psfm_common.h"
#include "psfm_sweep.h"
#include "psfm_fused.h"

// fused::Args::prio_mode = the K12_PRIO knob (psfm_knobs.hip, default 2 = the younger wave of a SIMD
// pair one level up in its p-eval; A/B on one box, profiles/r04/prio: kbench B=4 101.0 -> 98.0 us,
// B=6 141.3 -> 135.4 us; in the step 95.6-97.3 -> 93.8-94.1 us); 0 = off
#include "psfm_knobs.h"

using namespace psfm;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define PSFM_LAUNCH_CHECK()                                                          \
    do {                                                                             \
        hipError_t e_ = hipGetLastError();                                           \
        if (e_ != hipSuccess) return fail((int)e_, std::string("launch: ") +        \
                                                       hipGetErrorString(e_));       \
    } while (0)

struct KArgs {
    psfm_params p;
    psfm_inputs in;
    psfm_workspace ws;
    const float* grad_out;
    float* grad_sig[MAXS];
    const float* smooth_stats;
};

template <typename T>
__device__ __forceinline__ T pick4(const T (&a)[4], int i) {
    return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

__device__ __forceinline__ float sgnf(float v) { return v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f); }

// number of candidate SOURCES per scale (warped per context, + unwarped per context with automask)
__host__ __device__ __forceinline__ int n_src(const psfm_params& p) { return p.automask ? 2 * p.N : p.N; }
__host__ __device__ __forceinline__ int src_warp(const psfm_params& p, int j) { return p.automask ? 2 * j : j; }
__host__ __device__ __forceinline__ int src_unwarp(int j) { return 2 * j + 1; }

struct TileGeom {
    int b, tile, x0, y0, lx, ly, gx, gy;
    bool inside;
};

__device__ __forceinline__ TileGeom tile_geom(int H, int W) {
    TileGeom g;
    g.tile = blockIdx.x;
    g.b = blockIdx.y;
    const int tx = tiles_x(W);
    g.x0 = (g.tile % tx) * TX;
    g.y0 = (g.tile / tx) * TY;
    g.lx = threadIdx.x % TX;
    g.ly = threadIdx.x / TX;
    g.gx = g.x0 + g.lx;
    g.gy = g.y0 + g.ly;
    g.inside = g.gx < W && g.gy < H;
    return g;
}

// ---------------------------------------------------------------------------------------------
// SSIM (3x3, reflect) of one output pixel from LDS windows (halo stride HX); x = estimate, y =
// target.  Returns mean_c clamp((1-SSIM_c)/2, 0, 1) and mean_c |x-y| (SSIM :15-54, :199-247).
// ---------------------------------------------------------------------------------------------
template <int HX, int HY>
__device__ __forceinline__ void photo_terms(const float (&sX)[3][HY][HX], const float (&sY)[3][HY][HX],
                                            int cy, int cx, const float my[3], const float syy[3],
                                            float C1, float C2, float& ssim_mean, float& l1_mean,
                                            float l1c[3]) {
    float ls = 0.0f, as = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float mx = 0.0f, sxx = 0.0f, sxy = 0.0f;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const float xv = sX[c][cy + dy][cx + dx];
                const float yv = sY[c][cy + dy][cx + dx];
                mx += xv;
                sxx += xv * xv;
                sxy += xv * yv;
            }
        mx /= 9.0f;
        sxx /= 9.0f;
        sxy /= 9.0f;
        const float mxy = mx * my[c], mx2 = mx * mx, my2 = my[c] * my[c];
        const float v1 = 2.0f * (sxy - mxy) + C2;
        const float v2 = (sxx - mx2) + (syy[c] - my2) + C2;
        const float ssim = ((2.0f * mxy + C1) * v1) / ((mx2 + my2 + C1) * v2);
        ls += fminf(fmaxf((1.0f - ssim) / 2.0f, 0.0f), 1.0f);
        const float a = fabsf(sX[c][cy][cx] - sY[c][cy][cx]);
        l1c[c] = a;
        as += a;
    }
    ssim_mean = ls / 3.0f;
    l1_mean = as / 3.0f;
}

template <int HX, int HY>
__device__ __forceinline__ void target_stats(const float (&sY)[3][HY][HX], int cy, int cx,
                                             float my[3], float syy[3]) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float m = 0.0f, s2 = 0.0f;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                const float v = sY[c][cy + dy][cx + dx];
                m += v;
                s2 += v * v;
            }
        my[c] = m / 9.0f;
        syy[c] = s2 / 9.0f;
    }
}

// Fill an LDS halo image (origin y0-OFF, x0-OFF; reflect-padded) from a planar [3,H,W] image.
template <int HX, int HY, int OFF>
__device__ __forceinline__ void fill_plain(float (&dst)[3][HY][HX], const float* __restrict__ img,
                                           int H, int W, int y0, int x0) {
    const size_t plane = (size_t)H * W;
    for (int i = threadIdx.x; i < HX * HY; i += NT) {
        const int hy = i / HX, hx = i % HX;
        const size_t o = (size_t)reflect1(y0 - OFF + hy, H) * W + reflect1(x0 - OFF + hx, W);
#pragma unroll
        for (int c = 0; c < 3; ++c) dst[c][hy][hx] = img[c * plane + o];
    }
}

// Fill an LDS halo with the view-synthesised context image (camera_utils.py:27-59).
template <int HX, int HY, int OFF>
__device__ __forceinline__ void fill_warped(float (&dst)[3][HY][HX], const float* __restrict__ ctx,
                                            const float* __restrict__ sig, const CamRec& cam,
                                            const DepthChain& dc, int H, int W, int y0, int x0) {
    for (int i = threadIdx.x; i < HX * HY; i += NT) {
        const int hy = i / HX, hx = i % HX;
        const int yy = reflect1(y0 - OFF + hy, H), xx = reflect1(x0 - OFF + hx, W);
        float d1, inv;
        const float d = dc.warp_depth(sig[(size_t)yy * W + xx], d1, inv);
        Proj r;
        project(cam, (float)xx, (float)yy, d, H, W, r);
        float w[3];
        bilinear3(ctx, H, W, r.ix, r.iy, w);
        dst[0][hy][hx] = w[0];
        dst[1][hy][hx] = w[1];
        dst[2][hy][hx] = w[2];
    }
}

// ---------------------------------------------------------------------------------------------
// K1: forward.  STATS=true is the clip-statistics pass (sum/sumsq per candidate map).
// ---------------------------------------------------------------------------------------------
template <bool L1ONLY, bool STATS>
__global__ __launch_bounds__(NT) void k_photo_fwd(KArgs a) {
    const psfm_params& p = a.p;
    const int H = p.H, W = p.W, N = p.N, B = p.B;
    const TileGeom g = tile_geom(H, W);
    constexpr int HX = TX + 2, HY = TY + 2;
    __shared__ float sX[3][HY][HX];
    __shared__ float sY[3][HY][HX];
    __shared__ float red[NWAVE * 16];

    const size_t plane = (size_t)H * W;
    const int tiles = tiles_img(H, W);
    const int blk = g.b * tiles + g.tile;
    const size_t pix = (size_t)g.gy * W + g.gx;
    const int cy = g.ly + 1, cx = g.lx + 1;
    const DepthChain dc{1.0f / fmaxf(p.max_depth, 1e-6f),
                        (float)(1.0 / fmax((double)p.min_depth, 1e-6) - 1.0 / fmax((double)p.max_depth, 1e-6))};
    const float l1w = 1.0f - p.ssim_w;
    const int nsrc = n_src(p);

    fill_plain<HX, HY, 1>(sY, a.in.tgt + (size_t)g.b * 3 * plane, H, W, g.y0, g.x0);
    __syncthreads();
    float my[3] = {0, 0, 0}, syy[3] = {0, 0, 0};
    if (!L1ONLY) target_stats<HX, HY>(sY, cy, cx, my, syy);
    const float mval = (a.in.mask == nullptr) ? 1.0f : (g.inside ? a.in.mask[(size_t)g.b * plane + pix] : 0.0f);

    // candidate photometric values (raw: before clip and mask)
    float cu[MAXN][3], cw[MAXN][3];
    auto eval = [&](float (&out)[3]) {
        float sm, lm, l1c[3];
        photo_terms<HX, HY>(sX, sY, cy, cx, my, syy, p.C1, p.C2, sm, lm, l1c);
        if (L1ONLY) {
            out[0] = l1c[0]; out[1] = l1c[1]; out[2] = l1c[2];
        } else {
            out[0] = p.ssim_w * sm + l1w * lm;
        }
    };

    // automask: un-warped context losses (identical for every full-res scale: computed once)
    if (p.automask) {
#pragma unroll
        for (int j = 0; j < MAXN; ++j) {
            if (j >= N) break;
            fill_plain<HX, HY, 1>(sX, pick4(a.in.ctx, j) + (size_t)g.b * 3 * plane, H, W, g.y0, g.x0);
            __syncthreads();
            eval(cu[j]);
            __syncthreads();
        }
    }

    const int C = L1ONLY ? 3 : 1;
    for (int s = 0; s < p.S; ++s) {
        const float* sig = pick4(a.in.sig, s) + (size_t)g.b * plane;
#pragma unroll
        for (int j = 0; j < MAXN; ++j) {
            if (j >= N) break;
            CamRec cam;
            load_cam(a.in.cam + ((size_t)(s * N + j) * B + g.b) * PSFM_CAMREC, cam);
            fill_warped<HX, HY, 1>(sX, pick4(a.in.ctx, j) + (size_t)g.b * 3 * plane, sig, cam, dc,
                                   H, W, g.y0, g.x0);
            __syncthreads();
            eval(cw[j]);
            __syncthreads();
        }

        if (STATS) {
            // per candidate map: sum and sum of squares of the raw photometric values (:251)
            float st[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) st[k] = 0.0f;
            if (g.inside) {
#pragma unroll
                for (int j = 0; j < MAXN; ++j) {
                    if (j >= N) break;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        if (c >= C) break;
                        const int sw = p.automask ? 2 * j : j;
                        st[2 * sw] += cw[j][c];
                        st[2 * sw + 1] += cw[j][c] * cw[j][c];
                        if (p.automask) {
                            st[2 * (sw + 1)] += cu[j][c];
                            st[2 * (sw + 1) + 1] += cu[j][c] * cu[j][c];
                        }
                    }
                }
            }
            block_sum<16>(st, red);
            if (threadIdx.x == 0) {
                for (int k = 0; k < nsrc; ++k) {
                    float* o = a.ws.clip_part + (((size_t)s * nsrc + k) * (B * tiles) + blk) * 2;
                    o[0] = st[2 * k];
                    o[1] = st[2 * k + 1];
                }
            }
            continue;
        }

        // clip (:249-253) -> mask (:256-264) -> min / mean over candidates (:284-288)
        const float* thr = (p.clip_loss > 0.0f) ? a.ws.clip_thr + (size_t)s * nsrc : nullptr;
        float best = INFINITY, sum = 0.0f;
        int arg = 0, k = 0;
#pragma unroll
        for (int j = 0; j < MAXN; ++j) {
            if (j >= N) break;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (u == 1 && !p.automask) break;
                const int src = u ? src_unwarp(j) : src_warp(p, j);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    if (c >= C) break;
                    float v = u ? cu[j][c] : cw[j][c];
                    if (thr) v = fminf(v, thr[src]);
                    v = v * mval;
                    sum += v;
                    if (v < best) {
                        best = v;
                        arg = k;
                    }
                    ++k;
                }
            }
        }
        float val[1] = {0.0f};
        if (g.inside) {
            if (p.reduce_op == PSFM_REDUCE_MIN) {
                val[0] = best;
                a.ws.argmin[((size_t)s * B + g.b) * plane + pix] = (uint8_t)arg;
            } else {
                val[0] = sum;
            }
        }
        block_sum<1>(val, red);
        if (threadIdx.x == 0) a.ws.photo_part[(size_t)s * (B * tiles) + blk] = val[0];
    }
}

// ---------------------------------------------------------------------------------------------
// K2: backward of the photometric term.
// ---------------------------------------------------------------------------------------------
template <bool L1ONLY>
__global__ __launch_bounds__(NT) void k_photo_bwd(KArgs a) {
    const psfm_params& p = a.p;
    const int H = p.H, W = p.W, N = p.N, B = p.B;
    const TileGeom g = tile_geom(H, W);
    constexpr int HX2 = TX + 4, HY2 = TY + 4;  // warped / target: tile + 2
    constexpr int HX1 = TX + 2, HY1 = TY + 2;  // SSIM adjoint coefficients: tile + 1
    __shared__ float sX[3][HY2][HX2];
    __shared__ float sY[3][HY2][HX2];
    __shared__ float sC[10][HY1][HX1];
    __shared__ float red[NWAVE * 12];

    const size_t plane = (size_t)H * W;
    const int tiles = tiles_img(H, W);
    const int blk = g.b * tiles + g.tile;
    const size_t pix = (size_t)g.gy * W + g.gx;
    const DepthChain dc{1.0f / fmaxf(p.max_depth, 1e-6f),
                        (float)(1.0 / fmax((double)p.min_depth, 1e-6) - 1.0 / fmax((double)p.max_depth, 1e-6))};
    const float l1w = 1.0f - p.ssim_w;
    const int nsrc = n_src(p);
    const int ncand = nsrc * (L1ONLY ? 3 : 1);
    const float gout = *a.grad_out;
    const double cnt = (double)B * H * W;
    const float gscale = (p.reduce_op == PSFM_REDUCE_MIN)
                             ? (float)(gout / ((double)p.n_scales * cnt))
                             : (float)(gout / ((double)p.n_scales * (double)nsrc * cnt * (L1ONLY ? 3.0 : 1.0)));
    const float* mask = a.in.mask ? a.in.mask + (size_t)g.b * plane : nullptr;
    (void)ncand;

    fill_plain<HX2, HY2, 2>(sY, a.in.tgt + (size_t)g.b * 3 * plane, H, W, g.y0, g.x0);
    __syncthreads();

    for (int s = 0; s < p.S; ++s) {
        const float* sig = pick4(a.in.sig, s) + (size_t)g.b * plane;
        const uint8_t* am = a.ws.argmin + ((size_t)s * B + g.b) * plane;
        const float* thr = (p.clip_loss > 0.0f) ? a.ws.clip_thr + (size_t)s * nsrc : nullptr;
        float gs = 0.0f;
        float qd = 1.0f, qd1 = 1.0f, qinv = 1.0f;
        if (g.inside) qd = dc.warp_depth(sig[pix], qd1, qinv);

        for (int j = 0; j < N; ++j) {
            const int src = src_warp(p, j);
            CamRec cam;
            load_cam(a.in.cam + ((size_t)(s * N + j) * B + g.b) * PSFM_CAMREC, cam);
            const float* ctx = pick4(a.in.ctx, j) + (size_t)g.b * 3 * plane;
            float gT[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) gT[k] = 0.0f;

            // does any pixel whose SSIM window touches this tile select this candidate?
            bool any = (p.reduce_op != PSFM_REDUCE_MIN);
            if (!any) {
                for (int i = threadIdx.x; i < HX1 * HY1; i += NT) {
                    const int py = g.y0 - 1 + i / HX1, px = g.x0 - 1 + i % HX1;
                    if (py < 0 || py >= H || px < 0 || px >= W) continue;
                    const int ai = am[(size_t)py * W + px];
                    any |= L1ONLY ? (ai / 3 == src) : (ai == src);
                }
            }
            any = __syncthreads_or(any);

            if (any && L1ONLY) {
                // 3-channel L1 candidates (:246): no SSIM window, per-pixel adjoint
                if (g.inside) {
                    Proj r;
                    project(cam, (float)g.gx, (float)g.gy, qd, H, W, r);
                    float w[3];
                    bilinear3(ctx, H, W, r.ix, r.iy, w);
                    float gw[3];
                    const float mv = mask ? mask[pix] : 1.0f;
                    bool nz = false;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const float y = a.in.tgt[((size_t)g.b * 3 + c) * plane + pix];
                        const float raw = fabsf(w[c] - y);
                        float G = gscale * mv;
                        if (p.reduce_op == PSFM_REDUCE_MIN && am[pix] != src * 3 + c) G = 0.0f;
                        if (thr && !(raw <= thr[src])) G = 0.0f;
                        gw[c] = G * sgnf(w[c] - y);
                        nz |= gw[c] != 0.0f;
                    }
                    if (nz) {
                        float gix, giy;
                        bilinear3_grad_pos(ctx, H, W, r.ix, r.iy, gw, gix, giy);
                        const float gd = project_grad(cam, r, qd, gix, giy, H, W, gT);
                        gs += gd * dc.dwarp_ds(qd, qd1, qinv);
                    }
                }
            } else if (any) {
                fill_warped<HX2, HY2, 2>(sX, ctx, sig, cam, dc, H, W, g.y0, g.x0);
                __syncthreads();
                // SSIM adjoint coefficients on the tile + 1 halo
                for (int i = threadIdx.x; i < HX1 * HY1; i += NT) {
                    const int hy = i / HX1, hx = i % HX1;
                    const int py = g.y0 - 1 + hy, px = g.x0 - 1 + hx;
                    float co[10];
#pragma unroll
                    for (int k = 0; k < 10; ++k) co[k] = 0.0f;
                    if (py >= 0 && py < H && px >= 0 && px < W) {
                        const size_t pp = (size_t)py * W + px;
                        float G = gscale * (mask ? mask[pp] : 1.0f);
                        if (p.reduce_op == PSFM_REDUCE_MIN && am[pp] != src) G = 0.0f;
                        if (G != 0.0f) {
                            const int cy = hy + 1, cx = hx + 1;  // in the tile + 2 frame
                            float dS_dmx[3], dS_dsxx[3], dS_dsxy[3], pass[3];
                            float ls = 0.0f, as = 0.0f;
#pragma unroll
                            for (int c = 0; c < 3; ++c) {
                                float mx = 0.0f, sxx = 0.0f, sxy = 0.0f, my = 0.0f, syy = 0.0f;
#pragma unroll
                                for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                                    for (int dx = -1; dx <= 1; ++dx) {
                                        const float xv = sX[c][cy + dy][cx + dx];
                                        const float yv = sY[c][cy + dy][cx + dx];
                                        mx += xv;
                                        sxx += xv * xv;
                                        sxy += xv * yv;
                                        my += yv;
                                        syy += yv * yv;
                                    }
                                mx /= 9.0f; sxx /= 9.0f; sxy /= 9.0f; my /= 9.0f; syy /= 9.0f;
                                const float mxy = mx * my, mx2 = mx * mx, my2 = my * my;
                                const float A1 = 2.0f * mxy + p.C1, A2 = 2.0f * (sxy - mxy) + p.C2;
                                const float B1 = mx2 + my2 + p.C1, B2 = (sxx - mx2) + (syy - my2) + p.C2;
                                const float Nn = A1 * A2, D = B1 * B2;
                                const float ssim = Nn / D;
                                const float l = (1.0f - ssim) / 2.0f;
                                pass[c] = (l >= 0.0f && l <= 1.0f) ? 1.0f : 0.0f;
                                ls += fminf(fmaxf(l, 0.0f), 1.0f);
                                as += fabsf(sX[c][cy][cx] - sY[c][cy][cx]);
                                const float iD = 1.0f / D;
                                dS_dmx[c] = 2.0f * my * (A2 - A1) * iD - Nn * 2.0f * mx * (B2 - B1) * iD * iD;
                                dS_dsxx[c] = -Nn * B1 * iD * iD;
                                dS_dsxy[c] = 2.0f * A1 * iD;
                            }
                            if (thr) {
                                const float raw = p.ssim_w * (ls / 3.0f) + l1w * (as / 3.0f);
                                if (!(raw <= thr[src])) G = 0.0f;
                            }
                            const float kS = G * (-0.5f) * (p.ssim_w / 3.0f) / 9.0f;
#pragma unroll
                            for (int c = 0; c < 3; ++c) {
                                co[c] = kS * pass[c] * dS_dmx[c];
                                co[3 + c] = kS * pass[c] * dS_dsxx[c];
                                co[6 + c] = kS * pass[c] * dS_dsxy[c];
                            }
                            co[9] = G * l1w / 3.0f;
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 10; ++k) sC[k][hy][hx] = co[k];
                }
                __syncthreads();
                if (g.inside) {
                    const int qy2 = g.ly + 2, qx2 = g.lx + 2;
                    float gw[3] = {0.0f, 0.0f, 0.0f};
                    bool nz = false;
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const float xq = sX[c][qy2][qx2], yq = sY[c][qy2][qx2];
                        float acc = 0.0f;
#pragma unroll
                        for (int dy = -1; dy <= 1; ++dy) {
                            const int py = g.gy + dy;
                            if (py < 0 || py >= H) continue;
                            const float wy = 1.0f + ((py == 0 && g.gy == 1) ? 1.0f : 0.0f) +
                                             ((py == H - 1 && g.gy == H - 2) ? 1.0f : 0.0f);
#pragma unroll
                            for (int dx = -1; dx <= 1; ++dx) {
                                const int px = g.gx + dx;
                                if (px < 0 || px >= W) continue;
                                const float wx = 1.0f + ((px == 0 && g.gx == 1) ? 1.0f : 0.0f) +
                                                 ((px == W - 1 && g.gx == W - 2) ? 1.0f : 0.0f);
                                const int hy = g.ly + 1 + dy, hx = g.lx + 1 + dx;
                                acc += (wy * wx) * (sC[c][hy][hx] + 2.0f * xq * sC[3 + c][hy][hx] +
                                                    yq * sC[6 + c][hy][hx]);
                            }
                        }
                        acc += sC[9][g.ly + 1][g.lx + 1] * sgnf(xq - yq);
                        gw[c] = acc;
                        nz |= acc != 0.0f;
                    }
                    if (nz) {
                        Proj r;
                        project(cam, (float)g.gx, (float)g.gy, qd, H, W, r);
                        float gix, giy;
                        bilinear3_grad_pos(ctx, H, W, r.ix, r.iy, gw, gix, giy);
                        const float gd = project_grad(cam, r, qd, gix, giy, H, W, gT);
                        gs += gd * dc.dwarp_ds(qd, qd1, qinv);
                    }
                }
            }
            block_sum<12>(gT, red);  // (its barriers also retire sX / sC before the next fill)
            if (threadIdx.x == 0) {
                float* o = a.ws.pose_part + (((size_t)(s * N + j) * B + g.b) * tiles + g.tile) * 12;
#pragma unroll
                for (int k = 0; k < 12; ++k) o[k] = gT[k];
            }
        }
        if (g.inside) pick4(a.grad_sig, s)[(size_t)g.b * plane + pix] = gs;
    }
    (void)blk;
}

// ---------------------------------------------------------------------------------------------
// K3: smoothness (utils/depth.py:146-198, multiview_photometric_loss.py:301-327)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float edge_weight(const float* __restrict__ img, size_t plane, size_t p,
                                             size_t q) {
    const float m = (fabsf(img[p] - img[q]) + fabsf(img[plane + p] - img[plane + q]) +
                     fabsf(img[2 * plane + p] - img[2 * plane + q])) / 3.0f;
    return expf(-m);
}

__global__ __launch_bounds__(NT) void k_smooth_fwd(KArgs a) {
    const psfm_params& p = a.p;
    const int H = p.H, W = p.W, B = p.B;
    const TileGeom g = tile_geom(H, W);
    __shared__ float red[NWAVE * 4];
    const size_t plane = (size_t)H * W;
    const int tiles = tiles_img(H, W);
    const size_t pix = (size_t)g.gy * W + g.gx;
    const float* img = a.in.tgt + (size_t)g.b * 3 * plane;
    const bool hx = g.inside && g.gx < W - 1, hy = g.inside && g.gy < H - 1;
    const float wx = hx ? edge_weight(img, plane, pix, pix + 1) : 0.0f;
    const float wy = hy ? edge_weight(img, plane, pix, pix + W) : 0.0f;
    for (int s = 0; s < p.S; ++s) {
        const float* sg = pick4(a.in.sig, s) + (size_t)g.b * plane;
        float v[3] = {0.0f, 0.0f, 0.0f};
        if (g.inside) {
            const float c = sg[pix];
            v[0] = hx ? fabsf(c - sg[pix + 1]) * wx : 0.0f;
            v[1] = hy ? fabsf(c - sg[pix + W]) * wy : 0.0f;
            v[2] = c;
        }
        block_sum<3>(v, red);
        if (threadIdx.x == 0) {
            float* o = a.ws.smooth_part + (((size_t)s * B + g.b) * tiles + g.tile) * 4;
            o[0] = v[0];
            o[1] = v[1];
            o[2] = v[2];
            o[3] = 0.0f;
        }
    }
}

__global__ __launch_bounds__(NT) void k_smooth_bwd(KArgs a) {
    const psfm_params& p = a.p;
    const int H = p.H, W = p.W, B = p.B;
    const TileGeom g = tile_geom(H, W);
    if (!g.inside) return;
    const size_t plane = (size_t)H * W;
    const size_t pix = (size_t)g.gy * W + g.gx;
    const float* img = a.in.tgt + (size_t)g.b * 3 * plane;
    const float gout = *a.grad_out;
    const bool r = g.gx < W - 1, l = g.gx > 0, d = g.gy < H - 1, u = g.gy > 0;
    const float wr = r ? edge_weight(img, plane, pix, pix + 1) : 0.0f;
    const float wl = l ? edge_weight(img, plane, pix - 1, pix) : 0.0f;
    const float wd = d ? edge_weight(img, plane, pix, pix + W) : 0.0f;
    const float wu = u ? edge_weight(img, plane, pix - W, pix) : 0.0f;
    for (int s = 0; s < p.S; ++s) {
        const int gsi = p.scale0 + s;
        const float* st = a.smooth_stats + ((size_t)gsi * B + g.b) * 4;  // Ax, Ay, m, m_clamped
        const double base = (double)gout * p.smooth_w / ((double)p.n_scales * (double)(1 << gsi));
        const float cx = (float)(base / ((double)B * H * (W - 1)));
        const float cy = (float)(base / ((double)B * (H - 1) * W));
        const float mc = st[3];
        const float* sg = pick4(a.in.sig, s) + (size_t)g.b * plane;
        const float c = sg[pix];
        float gx = 0.0f, gy = 0.0f;
        if (r) gx += sgnf(c - sg[pix + 1]) * wr;
        if (l) gx -= sgnf(sg[pix - 1] - c) * wl;
        if (d) gy += sgnf(c - sg[pix + W]) * wd;
        if (u) gy -= sgnf(sg[pix - W] - c) * wu;
        float gsm = (cx * gx + cy * gy) / mc;
        if (st[2] >= 1e-6f) gsm -= (cx * st[0] + cy * st[1]) / (mc * mc) / (float)(H * W);
        pick4(a.grad_sig, s)[(size_t)g.b * plane + pix] += gsm;
    }
}

// ---------------------------------------------------------------------------------------------
// Finalize: fixed-order reductions of the per-tile partials (one 1024-thread block, one wave per
// item, fp64 accumulation).  out = {loss, metrics.photometric_loss, metrics.smoothness_loss}.
// ---------------------------------------------------------------------------------------------
struct FinCall {
    const float* photo_part;
    const float* smooth_part;
    int S, scale0, B, H, W, tiles;
    double photo_scale;
};
struct FinArgs {
    FinCall c[MAXS];
    int ncalls, n_scales, has_smooth;
    float smooth_w;
    float* smooth_stats;
    float* out;
};

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(1024) void k_finalize(FinArgs f) {
    // items: photo (call, s) and smooth (call, s, b); smooth item stores 3 sums
    __shared__ double photo_item[MAXS * MAXS];
    __shared__ double smooth_item[MAXS * MAXS * 64][3];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    int item = 0;
    for (int ci = 0; ci < f.ncalls; ++ci) {
        const FinCall& c = f.c[ci];
        const int nparts = c.B * c.tiles;
        for (int s = 0; s < c.S; ++s, ++item) {
            if (item % nw != wave) continue;
            double acc = 0.0;
            // unrolled: the loads of 8 trips go out together (one latency instead of 8; the adds keep
            // their order)
#pragma unroll 8
            for (int k = lane; k < nparts; k += 64) acc += (double)c.photo_part[(size_t)s * nparts + k];
            acc = wave_sum_d(acc);
            if (lane == 0) photo_item[ci * MAXS + s] = acc * c.photo_scale;
        }
    }
    if (f.has_smooth) {
        item = 0;
        for (int ci = 0; ci < f.ncalls; ++ci) {
            const FinCall& c = f.c[ci];
            for (int s = 0; s < c.S; ++s)
                for (int b = 0; b < c.B; ++b, ++item) {
                    if (item % nw != wave) continue;
                    const float* sp = c.smooth_part + ((size_t)s * c.B + b) * c.tiles * 4;
                    double ax = 0.0, ay = 0.0, m = 0.0;
#pragma unroll 4
                    for (int k = lane; k < c.tiles; k += 64) {
                        ax += (double)sp[k * 4];
                        ay += (double)sp[k * 4 + 1];
                        m += (double)sp[k * 4 + 2];
                    }
                    ax = wave_sum_d(ax);
                    ay = wave_sum_d(ay);
                    m = wave_sum_d(m);
                    if (lane == 0 && item < MAXS * MAXS * 64) {
                        // the item's smoothness statistics and its term of the loss, here, in parallel
                        // over the waves (thread 0's serial tail of fp64 divisions took most of the launch)
                        const float mf = (float)(m / ((double)c.H * c.W));
                        const float mc = fmaxf(mf, 1e-6f);
                        smooth_item[item][0] = ax / ((double)c.B * c.H * (c.W - 1)) / mc +
                                               ay / ((double)c.B * (c.H - 1) * c.W) / mc;
                        float* st = f.smooth_stats + ((size_t)(c.scale0 + s) * c.B + b) * 4;
                        st[0] = (float)ax;
                        st[1] = (float)ay;
                        st[2] = mf;
                        st[3] = mc;
                    }
                }
        }
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double photo = 0.0;
    for (int ci = 0; ci < f.ncalls; ++ci)
        for (int s = 0; s < f.c[ci].S; ++s) photo += photo_item[ci * MAXS + s];
    double smooth = 0.0;
    if (f.has_smooth) {
        item = 0;
        for (int ci = 0; ci < f.ncalls; ++ci) {
            const FinCall& c = f.c[ci];
            for (int s = 0; s < c.S; ++s) {
                const int gsi = c.scale0 + s;
                double term = 0.0;
                for (int b = 0; b < c.B; ++b, ++item) term += smooth_item[item][0];
                smooth += term / (double)(1 << gsi);
            }
        }
        smooth = (double)f.smooth_w * (smooth / (double)f.n_scales);
    }
    const float photo_f = (float)photo;
    const float smooth_f = (float)smooth;
    const float loss = f.has_smooth ? photo_f + smooth_f : photo_f;
    f.out[0] = loss;
    f.out[1] = loss;  // metrics['photometric_loss'] aliases the loss storage
    f.out[2] = smooth_f;
}

// clip thresholds: thr[s][src] = mean + clip * std (unbiased) of each candidate map (:251-253)
struct ThrArgs {
    const float* part;
    float* thr;
    int S, nsrc, nparts;
    double count;
    float clip;
};

__global__ __launch_bounds__(1024) void k_clip_thr(ThrArgs t) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int item = wave; item < t.S * t.nsrc; item += nw) {
        const float* pp = t.part + (size_t)item * t.nparts * 2;
        double s1 = 0.0, s2 = 0.0;
        for (int k = lane; k < t.nparts; k += 64) {
            s1 += (double)pp[2 * k];
            s2 += (double)pp[2 * k + 1];
        }
        s1 = wave_sum_d(s1);
        s2 = wave_sum_d(s2);
        if (lane == 0) {
            const double mean = s1 / t.count;
            const double var = fmax((s2 - s1 * mean) / (t.count - 1.0), 0.0);
            t.thr[item] = (float)(mean + (double)t.clip * sqrt(var));
        }
    }
}

// dL/dT: sum over calls, scales and tiles (fixed order) -> grad_T [N][B][stride] (stride 16: the
// [4][4] pose matrix, bottom row zero)
struct PoseRedCall {
    const float* part;
    int S, N, B, tiles;
};
struct PoseRedArgs {
    PoseRedCall c[MAXS];
    int ncalls, N, B, stride;
    float* grad_T;
    const float* grad_out;  // K12 path: partials are for dL/dloss = 1 (NULL: already scaled)
};

__global__ __launch_bounds__(256) void k_pose_reduce(PoseRedArgs r) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int item = blockIdx.x * nw + wave; item < r.N * r.B * 12; item += gridDim.x * nw) {
        const int k = item % 12, jb = item / 12, b = jb % r.B, j = jb / r.B;
        double acc = 0.0;
        for (int ci = 0; ci < r.ncalls; ++ci) {
            const PoseRedCall& c = r.c[ci];
            for (int s = 0; s < c.S; ++s) {
                const float* pp = c.part + (((size_t)(s * c.N + j) * c.B + b) * c.tiles) * 12;
                double part = 0.0;
#pragma unroll 4
                for (int t = lane; t < c.tiles; t += 64) part += (double)pp[(size_t)t * 12 + k];
                acc += wave_sum_d(part);
            }
        }
        if (lane == 0) {
            r.grad_T[(size_t)jb * r.stride + k] = (float)(r.grad_out ? acc * (double)*r.grad_out : acc);
            if (r.stride == 16 && k < 4) r.grad_T[(size_t)jb * 16 + 12 + k] = 0.0f;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K12 companions: sigmoid-sum pre-pass (smoothness normaliser) and the gradient finish.
// ---------------------------------------------------------------------------------------------
struct SigSumArgs {
    const float* sig[MAXS];
    int shift[MAXS];
    float* part;  // [S][B][SIGCH]
    const float* cam;  // [S][N][B][CAMREC]
    float* cam_pairs;  // [S][B][fused::PAIR_REC][2]
    int B, W, N, smooth;
    uint32_t plane;
};

// fixed-order sums over the FULL-resolution plane (the upsampled map's mean, utils/depth.py:183),
// a stored coarse map read through the nearest 2^shift mapping: the same values in the same
// order as summing the materialised upsample
__global__ __launch_bounds__(NT) void k_sig_sum(SigSumArgs a) {
    __shared__ float red[NWAVE];
    const int ch = blockIdx.x, b = blockIdx.y, s = blockIdx.z;
    if (ch == 0 && threadIdx.x < 2 * fused::PAIR_REC) {  // K12's context-paired camera record of (s, b)
        const int k = threadIdx.x >> 1, j = min((int)(threadIdx.x & 1), a.N - 1);
        const float* c = a.cam + (((size_t)s * a.N + j) * a.B + b) * PSFM_CAMREC;
        float v = 0.0f;
        if (k < PSFM_CAMREC) {
            v = c[k];   // Ki | Kr | T | pad
        } else if (k < 41) {  // E = K_ref R K^-1 - I, row-major (fp64, rounded once: fused.h PairProj)
            const int r = (k - 32) / 3, q = (k - 32) % 3;
            double acc = r == q ? -1.0 : 0.0;
            for (int i = 0; i < 3; ++i) {
                double mri = 0.0;   // (K_ref R)[r][i]
                for (int jj = 0; jj < 3; ++jj) mri += (double)c[9 + 3 * r + jj] * (double)c[18 + 4 * jj + i];
                acc += mri * (double)c[3 * i + q];
            }
            v = (float)acc;
        } else if (k < 44) {  // m = K_ref t (fp64, rounded once)
            const int r = k - 41;
            v = (float)((double)c[9 + 3 * r] * c[18 + 3] + (double)c[9 + 3 * r + 1] * c[18 + 7] +
                        (double)c[9 + 3 * r + 2] * c[18 + 11]);
        }
        a.cam_pairs[((size_t)s * a.B + b) * 2 * fused::PAIR_REC + threadIdx.x] = v;
    }
    if (!a.smooth) return;
    const int sh = pick4(a.shift, s);
    const uint32_t per = (a.plane + fused::SIGCH - 1) / fused::SIGCH;
    const uint32_t lo = ch * per, hi = min(a.plane, lo + per);
    const float* x = pick4(a.sig, s) + (size_t)b * (a.plane >> (2 * sh));
    const uint32_t W = (uint32_t)a.W, Ws = W >> sh;
    float v[1] = {0.0f};
    // 16 loads in flight per thread, then the adds in the plain loop's order (i = lo + tid, + NT, ...).
    // The loads are unconditional (index clamped, the value masked after): a load under `i < hi`
    // made the compiler branch around each one and wait for it (vmcnt(0)) before the next
    for (uint32_t i0 = lo + threadIdx.x; i0 < hi; i0 += 16 * NT) {
        float t[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint32_t i = i0 + u * NT, ic = min(i, hi - 1);
            float val;
            if (sh == 0) {
                val = x[ic];
            } else {
                const uint32_t y = ic / W, c = ic - y * W;
                val = x[(y >> sh) * Ws + (c >> sh)];
            }
            t[u] = i < hi ? val : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) v[0] += t[u];
    }
    block_sum<1>(v, red);
    if (threadIdx.x == 0) a.part[((size_t)s * a.B + b) * fused::SIGCH + ch] = v[0];
}

struct GradFinishArgs {
    const float* gin[MAXS];
    float* g[MAXS];
    int shift[MAXS];
    const float* smooth_stats;  // [n][B][4] = Ax, Ay, m, max(m, 1e-6)   (finalize)
    const float* grad_out;
    int B, H, W, scale0, n_scales, has_smooth;
    float smooth_w;
};

// the F x F block of the full-resolution gradient under one stored coarse pixel, summed in
// row-major order: every load issued before the first add (F = 2, 4, 8: 16-byte row loads for
// F >= 4), so a thread waits for memory once, not F*F times
template <int F>
__device__ __forceinline__ float block_sum_rowmajor(const float* __restrict__ r, int W, float go, float c) {
    float v[F][F];
#pragma unroll
    for (int dy = 0; dy < F; ++dy) {
        const float* row = r + (size_t)dy * W;
        if constexpr (F >= 4) {
#pragma unroll
            for (int q = 0; q < F / 4; ++q) {
                const float4 t = reinterpret_cast<const float4*>(row)[q];
                v[dy][4 * q] = t.x, v[dy][4 * q + 1] = t.y, v[dy][4 * q + 2] = t.z, v[dy][4 * q + 3] = t.w;
            }
        } else {
            const float2 t = *reinterpret_cast<const float2*>(row);
            v[dy][0] = t.x, v[dy][1] = t.y;
        }
    }
    float acc = 0.0f;
#pragma unroll
    for (int dy = 0; dy < F; ++dy)
#pragma unroll
        for (int dx = 0; dx < F; ++dx) acc += go * (v[dy][dx] + c);
    return acc;
}

// g = gout * (g + c[s][b]); c = -(cx Ax + cy Ay) / mc^2 / (H W) where the mean is not clamped
// (the d/ds of the 1/mean(s) normaliser; same expression as k_smooth_bwd)
__global__ __launch_bounds__(NT) void k_grad_finish(GradFinishArgs a) {
    const int b = blockIdx.y, s = blockIdx.z;
    const uint32_t plane = (uint32_t)(a.H * a.W);
    float c = 0.0f;
    if (a.has_smooth) {
        const int gsi = a.scale0 + s;
        const float* st = a.smooth_stats + ((size_t)gsi * a.B + b) * 4;
        const double base = (double)a.smooth_w / ((double)a.n_scales * (double)(1 << gsi));
        const float cx = (float)(base / ((double)a.B * a.H * (a.W - 1)));
        const float cy = (float)(base / ((double)a.B * (a.H - 1) * a.W));
        const float mc = st[3];
        if (st[2] >= 1e-6f) c = -((cx * st[0] + cy * st[1]) / (mc * mc) / (float)(a.H * a.W));
    }
    const float go = *a.grad_out;
    const float* gi = pick4(a.gin, s) + (size_t)b * plane;
    const int sh = pick4(a.shift, s);
    const uint32_t cplane = plane >> (2 * sh);
    float* g = pick4(a.g, s) + (size_t)b * cplane;
    const uint32_t i0 = blockIdx.x * (NT * 4) + threadIdx.x;
    if (sh == 0) {
        float v[4];   // the four loads first, unconditional (clamped index), then the guarded stores
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = gi[min(i0 + u * NT, plane - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t i = i0 + u * NT;
            if (i < plane) g[i] = go * (v[u] + c);
        }
        return;
    }
    // stored coarse map: the adjoint of the nearest 2^sh upsampling sums each 2^sh x 2^sh block of
    // the full-resolution gradient (row-major, fixed order: deterministic, no atomics).  One
    // coarse pixel per thread (the grid covers the full plane, >= 4x the coarse one)
    const int f = 1 << sh;
    const uint32_t Ws = (uint32_t)(a.W >> sh);
    const uint32_t i = blockIdx.x * NT + threadIdx.x;
    if (i >= cplane) return;
    const uint32_t Y = i / Ws, X = i - Y * Ws;
    const float* r = gi + ((size_t)Y * f) * a.W + (size_t)X * f;
    float acc;
    if (sh == 1) {
        acc = block_sum_rowmajor<2>(r, a.W, go, c);
    } else if (sh == 2) {
        acc = block_sum_rowmajor<4>(r, a.W, go, c);
    } else if (sh == 3) {
        acc = block_sum_rowmajor<8>(r, a.W, go, c);
    } else {
        acc = 0.0f;
        for (int dy = 0; dy < f; ++dy)
            for (int dx = 0; dx < f; ++dx) acc += go * (r[(size_t)dy * a.W + dx] + c);
    }
    g[i] = acc;
}

// ---------------------------------------------------------------------------------------------
// standalone view_synthesis (camera_utils.py:27-59) forward / backward
// ---------------------------------------------------------------------------------------------
struct VSArgs {
    int B, H, W;
    const float* ref;
    const float* depth;
    const float* cam;
    const float* grad_warped;
    float* warped;
    float* grad_depth;
    float* pose_part;
};

template <int MODEL>
__global__ __launch_bounds__(NT) void k_vs_fwd(VSArgs v) {
    const TileGeom g = tile_geom(v.H, v.W);
    if (!g.inside) return;
    const size_t plane = (size_t)v.H * v.W, pix = (size_t)g.gy * v.W + g.gx;
    Cams<1, MODEL> cam;
    cam.load(as_const(v.cam + (size_t)g.b * PSFM_CAMREC), v.B, v.H, v.W);
    typename Cams<1, MODEL>::P r;
    cam.project(0, cam.lift((float)g.gx, (float)g.gy, v.depth[(size_t)g.b * plane + pix]), r);
    float w[3];
    bilinear3(v.ref + (size_t)g.b * 3 * plane, v.H, v.W, r.ix, r.iy, w);
#pragma unroll
    for (int c = 0; c < 3; ++c) v.warped[((size_t)g.b * 3 + c) * plane + pix] = w[c];
}

template <int MODEL>
__global__ __launch_bounds__(NT) void k_vs_bwd(VSArgs v) {
    const TileGeom g = tile_geom(v.H, v.W);
    __shared__ float red[NWAVE * 12];
    const size_t plane = (size_t)v.H * v.W, pix = (size_t)g.gy * v.W + g.gx;
    Cams<1, MODEL> cam;
    cam.load(as_const(v.cam + (size_t)g.b * PSFM_CAMREC), v.B, v.H, v.W);
    float gT[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) gT[k] = 0.0f;
    if (g.inside) {
        const float d = v.depth[(size_t)g.b * plane + pix];
        typename Cams<1, MODEL>::P r;
        cam.project(0, cam.lift((float)g.gx, (float)g.gy, d), r);
        float gw[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) gw[c] = v.grad_warped[((size_t)g.b * 3 + c) * plane + pix];
        float gix, giy, gc[3];
        bilinear3_grad_pos(v.ref + (size_t)g.b * 3 * plane, v.H, v.W, r.ix, r.iy, gw, gix, giy);
        v.grad_depth[(size_t)g.b * plane + pix] = cam.grad(0, r, gix, giy, gc);
#pragma unroll
        for (int i = 0; i < 3; ++i) {  // dL/dT = gc (X, 1)^T
            gT[4 * i + 0] += gc[i] * r.X0;
            gT[4 * i + 1] += gc[i] * r.X1;
            gT[4 * i + 2] += gc[i] * r.X2;
            gT[4 * i + 3] += gc[i];
        }
    }
    block_sum<12>(gT, red);
    if (threadIdx.x == 0) {
        float* o = v.pose_part + ((size_t)g.b * tiles_img(v.H, v.W) + g.tile) * 12;
#pragma unroll
        for (int k = 0; k < 12; ++k) o[k] = gT[k];
    }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
int validate_shift(const psfm_params* p);
int validate(const psfm_params* p, const psfm_inputs* in) {
    if (!p || !in) return fail(-1, "null params/inputs");
    if (p->B < 1 || p->H < 2 || p->W < 2) return fail(-2, "bad B/H/W (need B>=1, H>=2, W>=2)");
    if (p->N < 1 || p->N > MAXN) return fail(-3, "N (contexts) must be in [1, 4]");
    if (p->S < 1 || p->S > MAXS) return fail(-4, "S (scales per call) must be in [1, 4]");
    if (p->n_scales < 1 || p->n_scales > MAXS || p->scale0 < 0 || p->scale0 + p->S > p->n_scales)
        return fail(-5, "scale0/S/n_scales inconsistent");
    if (p->reduce_op != PSFM_REDUCE_MIN && p->reduce_op != PSFM_REDUCE_MEAN)
        return fail(-6, "unknown reduce_op");
    if (p->automask && p->reduce_op != PSFM_REDUCE_MIN)
        return fail(-7, "For automasking only the min photometric_reduce_op is supported.");
    if (!in->tgt || !in->cam) return fail(-8, "null tgt/cam");
    for (int j = 0; j < p->N; ++j)
        if (!in->ctx[j]) return fail(-9, "null context pointer");
    for (int s = 0; s < p->S; ++s)
        if (!in->sig[s]) return fail(-10, "null sigmoid pointer");
    if ((long long)p->B * p->H * p->W > (1LL << 31)) return fail(-11, "image too large");
    if (p->cam_model != PSFM_CAM_PINHOLE && p->cam_model != PSFM_CAM_FISHEYE) return fail(-16, "unknown cam_model");
    if (p->cam_model == PSFM_CAM_FISHEYE && (p->N > 2 || p->l1_only))
        return fail(-16, "fisheye calls: N <= 2 and SSIM candidates (ssim_loss_weight > 0)");
    if (int e = validate_shift(p)) return e;
    return 0;
}

// stored-resolution shifts of the sigmoid maps (psfm_params.sig_shift)
bool any_shift(const psfm_params* p) {
    for (int s = 0; s < p->S; ++s)
        if (p->sig_shift[s]) return true;
    return false;
}
int validate_shift(const psfm_params* p) {
    for (int s = 0; s < p->S; ++s) {
        const int k = p->sig_shift[s];
        if (k < 0 || k > 8) return fail(-17, "sig_shift must be in [0, 8]");
        if (k && ((p->H & ((1 << k) - 1)) || (p->W & ((1 << k) - 1))))
            return fail(-17, "sig_shift: H and W must be multiples of 2^sig_shift");
    }
    if (any_shift(p) && p->l1_only) return fail(-17, "sig_shift > 0: SSIM candidates only (the K1 / K12 sweeps)");
    return 0;
}

dim3 tile_grid(const psfm_params* p) { return dim3(tiles_img(p->H, p->W), p->B); }

// partial-sum units per image: the v2 sweep kernels handle every config except the 3-channel
// L1-only candidates (ssim_loss_weight == 0), which keep the v1 tile kernels.
bool use_sweep(const psfm_params* p) { return !p->l1_only; }
// partial-sum units of the clip-statistics pass (always K1 / v1 tiles)
int stats_units(const psfm_params* p) { return use_sweep(p) ? sweep::k1_units(p->H, p->W) : tiles_img(p->H, p->W); }
bool fused_ok(const psfm_params* p) { return use_sweep(p) && p->N <= 2; }
// K12 band height for this launch.  K12 is issue-bound with at most WAVES waves resident per SIMD,
// and every wave of a launch costs RB + 5 sweep steps (4 halo rows + the pipeline tail), so the
// launch time follows the busiest SIMD: waves per SIMD n -> about n / 2 two-wave rounds, a lone
// wave running ~0.6 of a shared one.  Pick the candidate with the smallest steps x rounds on this
// device's CU count (B = 4 at 192 x 640: RB 18 -> 1936 waves, one round; B = 6: RB 28 -> 1848
// waves beat RB 18's 2904 = three waves on some SIMDs).
int simd_count();
int rb_for(const psfm_params* p) {
    const int simds = simd_count();
    auto cost = [&](int rb) {
        const double waves = (double)fused::units(p->H, p->W, rb) * p->B * p->S;
        const int n = (int)std::ceil(waves / simds);
        return (double)(rb + 5) * ((n / 2) + ((n & 1) ? 0.6 : 0.0));
    };
    return cost(fused::RB_HI) < cost(fused::RB_LO) ? fused::RB_HI : fused::RB_LO;
}
// K12 wave-pair balance (fused::Args young_from / prio_mode): the XCD's SIMD count, and the mode
// from PSFM_K12_PRIO (0 off, 2 younger +1 in the p-eval); only meaningful when the launch fits one
// wave round
int simd_count() {
    static int simds[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (!simds[dev]) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        simds[dev] = 4 * cus;
    }
    return simds[dev];
}
void k12_priority(fused::Args& fa, long waves) {
    const int simds = simd_count();
    fa.prio_mode = knob(KNOB_K12_PRIO);
    fa.young_from = simds / 8;  // SIMDs per XCD (8 XCDs)
    if (waves > 2L * simds || fa.prio_mode != 2) fa.prio_mode = 0;
    // XCD dealing: with fewer than 8 images each image's bands are split over 8 / B XCDs, every
    // XCD sweeping its part for all scales (sweep::work_item_parts); the K12_PARTS knob overrides (A/B)
    const int B = fa.p.B, parts = knob(KNOB_K12_PARTS);
    fa.xcd_parts = parts > 0 ? parts : (B < 8 ? 8 / B : 1);
}

int fwd_units(const psfm_params* p) {
    if (p->grad_fused && fused_ok(p)) return fused::units(p->H, p->W, rb_for(p));
    return stats_units(p);
}
int bwd_units(const psfm_params* p) {
    if (p->grad_fused && fused_ok(p)) return fused::units(p->H, p->W, rb_for(p));
    return use_sweep(p) ? sweep::k2_units(p->H, p->W) : tiles_img(p->H, p->W);
}

sweep::SweepArgs sweep_args(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws) {
    sweep::SweepArgs a{};
    a.p = *p;
    a.in = *in;
    if (ws) a.ws = *ws;
    return a;
}

void launch_k0(const psfm_params* p, const sweep::SweepArgs& a, hipStream_t st) {
    const dim3 grid(sweep::k0_units(p->H, p->W), p->B);
    switch (p->N) {
        case 1: hipLaunchKernelGGL((sweep::k0_unwarped<1>), grid, dim3(64), 0, st, a); break;
        case 2: hipLaunchKernelGGL((sweep::k0_unwarped<2>), grid, dim3(64), 0, st, a); break;
        case 3: hipLaunchKernelGGL((sweep::k0_unwarped<3>), grid, dim3(64), 0, st, a); break;
        default: hipLaunchKernelGGL((sweep::k0_unwarped<4>), grid, dim3(64), 0, st, a); break;
    }
}

// FAST: the reference default configuration (automask, 'min', smoothness, no clip, no mask)
// with its flags as compile-time constants.
bool fast_cfg(const psfm_params* p, const psfm_inputs* in) {
    return p->automask && p->reduce_op == PSFM_REDUCE_MIN && p->smooth_w > 0.0f && !(p->clip_loss > 0.0f) &&
           !in->mask;
}

template <bool STATS, bool FAST>
void launch_k1_t(const psfm_params* p, const sweep::SweepArgs& a, hipStream_t st) {
    const dim3 grid(sweep::k1_units(p->H, p->W), p->B, p->S);
    constexpr int PIN = PSFM_CAM_PINHOLE, FISH = PSFM_CAM_FISHEYE;
    if (p->cam_model == FISH) {  // N <= 2 (validated)
        if (p->N == 1) hipLaunchKernelGGL((sweep::k1_forward<1, STATS, FAST, FISH>), grid, dim3(64), 0, st, a);
        else hipLaunchKernelGGL((sweep::k1_forward<2, STATS, FAST, FISH>), grid, dim3(64), 0, st, a);
        return;
    }
    switch (p->N) {
        case 1: hipLaunchKernelGGL((sweep::k1_forward<1, STATS, FAST, PIN>), grid, dim3(64), 0, st, a); break;
        case 2: hipLaunchKernelGGL((sweep::k1_forward<2, STATS, FAST, PIN>), grid, dim3(64), 0, st, a); break;
        case 3: hipLaunchKernelGGL((sweep::k1_forward<3, STATS, FAST, PIN>), grid, dim3(64), 0, st, a); break;
        default: hipLaunchKernelGGL((sweep::k1_forward<4, STATS, FAST, PIN>), grid, dim3(64), 0, st, a); break;
    }
}

template <bool STATS>
void launch_k1(const psfm_params* p, const sweep::SweepArgs& a, hipStream_t st) {
    if (!STATS && fast_cfg(p, &a.in))
        launch_k1_t<false, true>(p, a, st);
    else
        launch_k1_t<STATS, false>(p, a, st);
}

template <int RB>
void launch_k12(const psfm_params* p, bool fast, dim3 grid, size_t lds, hipStream_t st, const fused::Args& fa) {
    constexpr int PIN = PSFM_CAM_PINHOLE, FISH = PSFM_CAM_FISHEYE;
    if (p->cam_model == FISH) {
        if (p->N == 1) {
            if (fast) hipLaunchKernelGGL((fused::k12_fwd_grad<1, true, FISH, RB>), grid, dim3(64), lds, st, fa);
            else hipLaunchKernelGGL((fused::k12_fwd_grad<1, false, FISH, RB>), grid, dim3(64), lds, st, fa);
        } else {
            if (fast) hipLaunchKernelGGL((fused::k12_fwd_grad<2, true, FISH, RB>), grid, dim3(64), lds, st, fa);
            else hipLaunchKernelGGL((fused::k12_fwd_grad<2, false, FISH, RB>), grid, dim3(64), lds, st, fa);
        }
    } else if (p->N == 1) {
        if (fast) hipLaunchKernelGGL((fused::k12_fwd_grad<1, true, PIN, RB>), grid, dim3(64), lds, st, fa);
        else hipLaunchKernelGGL((fused::k12_fwd_grad<1, false, PIN, RB>), grid, dim3(64), lds, st, fa);
    } else {
        if (fast) hipLaunchKernelGGL((fused::k12_fwd_grad<2, true, PIN, RB>), grid, dim3(64), lds, st, fa);
        else hipLaunchKernelGGL((fused::k12_fwd_grad<2, false, PIN, RB>), grid, dim3(64), lds, st, fa);
    }
}

}  // namespace

extern "C" {

int psfm_tiles_per_image(int H, int W) { return tiles_img(H, W); }

int psfm_workspace_floats(const psfm_params* p, size_t* photo, size_t* smooth, size_t* clip,
                          size_t* clip_thr, size_t* pose, size_t* argmin_bytes, size_t* unwarp,
                          size_t* sig_part, size_t* cam_pairs) {
    if (!p) return fail(-1, "null params");
    const int u = std::max(std::max(tiles_img(p->H, p->W), fused::units(p->H, p->W, fused::RB_LO)),
                           std::max(sweep::k1_units(p->H, p->W), sweep::k2_units(p->H, p->W)));
    const size_t t = (size_t)u * p->B;
    const size_t ns = (size_t)n_src(*p);
    if (photo) *photo = (size_t)p->S * t;
    if (smooth) *smooth = (size_t)p->S * t * 4;
    if (clip) *clip = (size_t)p->S * ns * t * 2;
    if (clip_thr) *clip_thr = (size_t)p->S * ns;
    if (pose) *pose = (size_t)p->S * p->N * t * 12;
    if (argmin_bytes) *argmin_bytes = (size_t)p->S * p->B * p->H * p->W;
    if (unwarp) *unwarp = (p->automask && !p->l1_only) ? (size_t)p->N * p->B * p->H * p->W : 0;
    if (sig_part) *sig_part = (size_t)p->S * p->B * fused::SIGCH;
    if (cam_pairs) *cam_pairs = (size_t)p->S * p->B * fused::PAIR_REC * 2;
    return 0;
}

int psfm_photometric_clip_stats(const psfm_params* p, const psfm_inputs* in,
                                const psfm_workspace* ws, void* stream) {
    if (int e = validate(p, in)) return e;
    if (!ws || !ws->clip_part || !ws->clip_thr) return fail(-12, "null clip workspace");
    KArgs a{};
    a.p = *p;
    a.in = *in;
    a.ws = *ws;
    hipStream_t st = (hipStream_t)stream;
    if (p->l1_only) {
        hipLaunchKernelGGL((k_photo_fwd<true, true>), tile_grid(p), dim3(NT), 0, st, a);
    } else {
        if (p->automask && !ws->unwarp) return fail(-12, "automask needs ws->unwarp");
        const sweep::SweepArgs sa = sweep_args(p, in, ws);
        if (p->automask) launch_k0(p, sa, st);
        launch_k1<true>(p, sa, st);
    }
    PSFM_LAUNCH_CHECK();
    ThrArgs t{ws->clip_part, ws->clip_thr, p->S, n_src(*p), p->B * stats_units(p),
              (double)p->B * p->H * p->W * (p->l1_only ? 3.0 : 1.0), p->clip_loss};
    hipLaunchKernelGGL(k_clip_thr, dim3(1), dim3(1024), 0, st, t);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_photometric_fwd(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws,
                         void* stream) {
    if (int e = validate(p, in)) return e;
    if (!ws || !ws->photo_part || (p->reduce_op == PSFM_REDUCE_MIN && !ws->argmin))
        return fail(-12, "null workspace");
    if (p->clip_loss > 0.0f && !ws->clip_thr) return fail(-12, "clip needs clip_thr");
    KArgs a{};
    a.p = *p;
    a.in = *in;
    a.ws = *ws;
    hipStream_t st = (hipStream_t)stream;
    if (p->l1_only) {
        hipLaunchKernelGGL((k_photo_fwd<true, false>), tile_grid(p), dim3(NT), 0, st, a);
    } else {
        if (p->smooth_w > 0.0f && !ws->smooth_part) return fail(-12, "null smoothness workspace");
        if (p->automask && !ws->unwarp) return fail(-12, "automask needs ws->unwarp");
        const sweep::SweepArgs sa = sweep_args(p, in, ws);
        if (p->automask && !(p->clip_loss > 0.0f)) launch_k0(p, sa, st);  // clip: done by clip_stats
        launch_k1<false>(p, sa, st);  // also writes the smoothness partials
    }
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_smoothness_fwd(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws,
                        void* stream) {
    if (int e = validate(p, in)) return e;
    if (!ws || !ws->smooth_part) return fail(-12, "null smoothness workspace");
    if (use_sweep(p)) return 0;  // fused into psfm_photometric_fwd (K1 sweep)
    KArgs a{};
    a.p = *p;
    a.in = *in;
    a.ws = *ws;
    hipLaunchKernelGGL(k_smooth_fwd, tile_grid(p), dim3(NT), 0, (hipStream_t)stream, a);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_finalize(int ncalls, const psfm_params* const* calls, const psfm_workspace* const* ws,
                  float* smooth_stats, float* out, void* stream) {
    if (ncalls < 1 || ncalls > MAXS || !calls || !ws || !out) return fail(-1, "bad finalize args");
    FinArgs f{};
    f.ncalls = ncalls;
    f.n_scales = calls[0]->n_scales;
    f.smooth_w = calls[0]->smooth_w;
    f.has_smooth = calls[0]->smooth_w > 0.0f;
    f.smooth_stats = smooth_stats;
    f.out = out;
    int items = 0;
    for (int i = 0; i < ncalls; ++i) {
        const psfm_params& p = *calls[i];
        FinCall& c = f.c[i];
        c.photo_part = ws[i]->photo_part;
        c.smooth_part = ws[i]->smooth_part;
        c.S = p.S;
        c.scale0 = p.scale0;
        c.B = p.B;
        c.H = p.H;
        c.W = p.W;
        c.tiles = fwd_units(&p);
        const double cnt = (double)p.B * p.H * p.W;
        c.photo_scale = (p.reduce_op == PSFM_REDUCE_MIN)
                            ? 1.0 / ((double)p.n_scales * cnt)
                            : 1.0 / ((double)p.n_scales * n_src(p) * cnt * (p.l1_only ? 3.0 : 1.0));
        items += p.S * p.B;
        if (f.has_smooth && (!c.smooth_part || !smooth_stats)) return fail(-12, "null smoothness buffers");
    }
    if (items > MAXS * MAXS * 64) return fail(-13, "too many (scale, batch) items");
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1024), 0, (hipStream_t)stream, f);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_photometric_bwd(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws,
                         const float* grad_out, float* const* grad_sig, void* stream) {
    if (int e = validate(p, in)) return e;
    if (p->cam_model != PSFM_CAM_PINHOLE) return fail(-16, "K2 backward is pinhole-only: use psfm_photometric_fwd_grad");
    if (any_shift(p)) return fail(-17, "sig_shift > 0: use psfm_photometric_fwd_grad (K12) for the gradient");
    if (!ws || !ws->pose_part || (p->reduce_op == PSFM_REDUCE_MIN && !ws->argmin))
        return fail(-12, "null workspace");
    if (!grad_out || !grad_sig) return fail(-14, "null grad buffers");
    KArgs a{};
    a.p = *p;
    a.in = *in;
    a.ws = *ws;
    a.grad_out = grad_out;
    for (int s = 0; s < p->S; ++s) {
        if (!grad_sig[s]) return fail(-14, "null grad_sig");
        a.grad_sig[s] = grad_sig[s];
    }
    hipStream_t st = (hipStream_t)stream;
    if (p->l1_only) {
        hipLaunchKernelGGL((k_photo_bwd<true>), tile_grid(p), dim3(NT), 0, st, a);
    } else {
        sweep::SweepArgs sa = sweep_args(p, in, ws);
        sa.grad_out = grad_out;
        for (int s = 0; s < p->S; ++s) sa.grad_sig[s] = grad_sig[s];
        hipLaunchKernelGGL(sweep::k2_backward, dim3(sweep::k2_units(p->H, p->W), p->B, p->S), dim3(64 * p->N),
                           sweep::k2_lds_bytes(p->N), st, sa);
    }
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_smoothness_bwd(const psfm_params* p, const psfm_inputs* in, const float* smooth_stats,
                        const float* grad_out, float* const* grad_sig, void* stream) {
    if (int e = validate(p, in)) return e;
    if (!smooth_stats || !grad_out || !grad_sig) return fail(-14, "null smoothness grad buffers");
    if (any_shift(p)) return fail(-17, "sig_shift > 0: use psfm_photometric_fwd_grad (K12) for the gradient");
    KArgs a{};
    a.p = *p;
    a.in = *in;
    a.grad_out = grad_out;
    a.smooth_stats = smooth_stats;
    for (int s = 0; s < p->S; ++s) {
        if (!grad_sig[s]) return fail(-14, "null grad_sig");
        a.grad_sig[s] = grad_sig[s];
    }
    hipLaunchKernelGGL(k_smooth_bwd, tile_grid(p), dim3(NT), 0, (hipStream_t)stream, a);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_pose_grad_reduce(int ncalls, const psfm_params* const* calls,
                          const psfm_workspace* const* ws, float* grad_T, int grad_stride, void* stream) {
    if (ncalls < 1 || ncalls > MAXS || !calls || !ws || !grad_T) return fail(-1, "bad pose reduce args");
    if (grad_stride != 12 && grad_stride != 16) return fail(-2, "grad_stride must be 12 or 16");
    PoseRedArgs r{};
    r.stride = grad_stride;
    r.ncalls = ncalls;
    r.N = calls[0]->N;
    r.B = calls[0]->B;
    r.grad_T = grad_T;
    for (int i = 0; i < ncalls; ++i) {
        if (calls[i]->N != r.N || calls[i]->B != r.B) return fail(-1, "calls disagree on N/B");
        r.c[i] = PoseRedCall{ws[i]->pose_part, calls[i]->S, calls[i]->N, calls[i]->B, bwd_units(calls[i])};
    }
    const int items = r.N * r.B * 12;
    hipLaunchKernelGGL(k_pose_reduce, dim3((items + 3) / 4), dim3(256), 0, (hipStream_t)stream, r);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_view_synthesis_fwd(int cam_model, int B, int H, int W, const float* ref, const float* depth,
                            const float* cam, float* warped, void* stream) {
    if (B < 1 || H < 2 || W < 2 || !ref || !depth || !cam || !warped) return fail(-1, "bad view_synthesis args");
    if (cam_model != PSFM_CAM_PINHOLE && cam_model != PSFM_CAM_FISHEYE) return fail(-16, "unknown cam_model");
    VSArgs v{B, H, W, ref, depth, cam, nullptr, warped, nullptr, nullptr};
    if (cam_model == PSFM_CAM_FISHEYE)
        hipLaunchKernelGGL(k_vs_fwd<PSFM_CAM_FISHEYE>, dim3(tiles_img(H, W), B), dim3(NT), 0, (hipStream_t)stream, v);
    else
        hipLaunchKernelGGL(k_vs_fwd<PSFM_CAM_PINHOLE>, dim3(tiles_img(H, W), B), dim3(NT), 0, (hipStream_t)stream, v);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_view_synthesis_bwd(int cam_model, int B, int H, int W, const float* ref, const float* depth,
                            const float* cam, const float* grad_warped, float* grad_depth,
                            float* pose_part, float* grad_T, void* stream) {
    if (B < 1 || H < 2 || W < 2 || !ref || !depth || !cam || !grad_warped || !grad_depth || !pose_part || !grad_T)
        return fail(-1, "bad view_synthesis_bwd args");
    if (cam_model != PSFM_CAM_PINHOLE && cam_model != PSFM_CAM_FISHEYE) return fail(-16, "unknown cam_model");
    VSArgs v{B, H, W, ref, depth, cam, grad_warped, nullptr, grad_depth, pose_part};
    hipStream_t st = (hipStream_t)stream;
    if (cam_model == PSFM_CAM_FISHEYE)
        hipLaunchKernelGGL(k_vs_bwd<PSFM_CAM_FISHEYE>, dim3(tiles_img(H, W), B), dim3(NT), 0, st, v);
    else
        hipLaunchKernelGGL(k_vs_bwd<PSFM_CAM_PINHOLE>, dim3(tiles_img(H, W), B), dim3(NT), 0, st, v);
    PSFM_LAUNCH_CHECK();
    PoseRedArgs r{};
    r.ncalls = 1;
    r.N = 1;
    r.B = B;
    r.stride = 12;
    r.grad_T = grad_T;
    r.c[0] = PoseRedCall{pose_part, 1, 1, B, tiles_img(H, W)};
    hipLaunchKernelGGL(k_pose_reduce, dim3((B * 12 + 3) / 4), dim3(256), 0, st, r);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_photometric_prepass(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws, void* stream) {
    if (int e = validate(p, in)) return e;
    if (!fused_ok(p)) return fail(-15, "prepass/fwd_grad need ssim_loss_weight > 0 and N <= 2 (use fwd + bwd)");
    if (!ws) return fail(-12, "null workspace");
    if (p->smooth_w > 0.0f && !ws->sig_part) return fail(-12, "null sig_part workspace");
    if (!ws->cam_pairs) return fail(-12, "null cam_pairs workspace");
    if (p->automask && !ws->unwarp) return fail(-12, "automask needs ws->unwarp");
    hipStream_t st = (hipStream_t)stream;
    if (p->automask && !(p->clip_loss > 0.0f)) launch_k0(p, sweep_args(p, in, ws), st);  // clip: clip_stats did
    {  // sigmoid chunk sums (smoothness normaliser) + the context-paired camera records
        SigSumArgs sa{};
        for (int s = 0; s < p->S; ++s) {
            sa.sig[s] = in->sig[s];
            sa.shift[s] = p->sig_shift[s];
        }
        sa.part = ws->sig_part;
        sa.cam = in->cam;
        sa.cam_pairs = ws->cam_pairs;
        sa.B = p->B;
        sa.W = p->W;
        sa.N = p->N;
        sa.smooth = p->smooth_w > 0.0f;
        sa.plane = (uint32_t)(p->H * p->W);
        hipLaunchKernelGGL(k_sig_sum, dim3(sa.smooth ? fused::SIGCH : 1, p->B, p->S), dim3(NT), 0, st, sa);
    }
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_photometric_fwd_grad(const psfm_params* p, const psfm_inputs* in, const psfm_workspace* ws,
                              float* const* grad_sig, void* stream) {
    if (int e = validate(p, in)) return e;
    if (!fused_ok(p)) return fail(-15, "fwd_grad needs ssim_loss_weight > 0 and N <= 2 (use fwd + bwd)");
    if (!p->grad_fused) return fail(-15, "fwd_grad needs p->grad_fused = 1 (finalize reads its unit grid)");
    if (!ws || !ws->photo_part || !ws->pose_part) return fail(-12, "null workspace");
    if (p->smooth_w > 0.0f && (!ws->smooth_part || !ws->sig_part)) return fail(-12, "null smoothness workspace");
    if (!ws->cam_pairs) return fail(-12, "null cam_pairs workspace (written by psfm_photometric_prepass)");
    if (p->automask && !ws->unwarp) return fail(-12, "automask needs ws->unwarp");
    if (p->clip_loss > 0.0f && !ws->clip_thr) return fail(-12, "clip needs clip_thr");
    if (!grad_sig) return fail(-14, "null grad_sig");
    fused::Args fa{};
    fa.p = *p;
    fa.in = *in;
    fa.ws = *ws;
    for (int s = 0; s < p->S; ++s) {
        if (!grad_sig[s]) return fail(-14, "null grad_sig");
        fa.grad_sig[s] = grad_sig[s];
    }
    hipStream_t st = (hipStream_t)stream;
    const int rb = rb_for(p);
    const dim3 grid(fused::units(p->H, p->W, rb), p->B, p->S);
    const size_t lds = fused::lds_bytes(p->N);
    const bool fast = fast_cfg(p, in);
    k12_priority(fa, (long)grid.x * grid.y * grid.z);
    if (rb == fused::RB_HI) launch_k12<fused::RB_HI>(p, fast, grid, lds, st, fa);
    else launch_k12<fused::RB_LO>(p, fast, grid, lds, st, fa);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_photometric_grad_finish(const psfm_params* p, const float* smooth_stats, const float* grad_out,
                                 const float* const* grad_k12, float* const* grad_sig, void* stream) {
    if (!p || !grad_out || !grad_sig || !grad_k12) return fail(-14, "null grad_finish args");
    if (p->B < 1 || p->H < 2 || p->W < 2 || p->S < 1 || p->S > MAXS) return fail(-2, "bad B/H/W/S");
    const bool sm = p->smooth_w > 0.0f;
    if (sm && !smooth_stats) return fail(-14, "null smooth_stats");
    GradFinishArgs a{};
    if (int e = validate_shift(p)) return e;
    for (int s = 0; s < p->S; ++s) {
        if (!grad_sig[s] || !grad_k12[s]) return fail(-14, "null grad_sig");
        if (p->sig_shift[s] && grad_sig[s] == grad_k12[s])
            return fail(-14, "grad_finish with sig_shift > 0 cannot run in place");
        a.gin[s] = grad_k12[s];
        a.g[s] = grad_sig[s];
        a.shift[s] = p->sig_shift[s];
    }
    a.smooth_stats = smooth_stats;
    a.grad_out = grad_out;
    a.B = p->B;
    a.H = p->H;
    a.W = p->W;
    a.scale0 = p->scale0;
    a.n_scales = p->n_scales;
    a.has_smooth = sm;
    a.smooth_w = p->smooth_w;
    const int plane = p->H * p->W;
    hipLaunchKernelGGL(k_grad_finish, dim3((plane + NT * 4 - 1) / (NT * 4), p->B, p->S), dim3(NT), 0,
                       (hipStream_t)stream, a);
    PSFM_LAUNCH_CHECK();
    return 0;
}

int psfm_pose_grad_reduce_scaled(int ncalls, const psfm_params* const* calls,
                                 const psfm_workspace* const* ws, const float* grad_out,
                                 float* grad_T, int grad_stride, void* stream) {
    if (ncalls < 1 || ncalls > MAXS || !calls || !ws || !grad_T || !grad_out) return fail(-1, "bad pose reduce args");
    if (grad_stride != 12 && grad_stride != 16) return fail(-2, "grad_stride must be 12 or 16");
    PoseRedArgs r{};
    r.stride = grad_stride;
    r.ncalls = ncalls;
    r.N = calls[0]->N;
    r.B = calls[0]->B;
    r.grad_T = grad_T;
    r.grad_out = grad_out;
    for (int i = 0; i < ncalls; ++i) {
        if (calls[i]->N != r.N || calls[i]->B != r.B) return fail(-1, "calls disagree on N/B");
        r.c[i] = PoseRedCall{ws[i]->pose_part, calls[i]->S, calls[i]->N, calls[i]->B, bwd_units(calls[i])};
    }
    const int items = r.N * r.B * 12;
    hipLaunchKernelGGL(k_pose_reduce, dim3((items + 3) / 4), dim3(256), 0, (hipStream_t)stream, r);
    PSFM_LAUNCH_CHECK();
    return 0;
}

const char* psfm_last_error(void) { return g_err.c_str(); }
// the source hash is passed by __graft_entry__.build() (sha256 of csrc/ + include/): a run can
// prove which sources the library it mapped was built from (build() rebuilds on a mismatch)
#ifndef PSFM_SRC_HASH
#define PSFM_SRC_HASH "unstamped-build!"
#endif
const char* psfm_version(void) { return "psfm-gfx950 0.2 src=" PSFM_SRC_HASH; }

int psfm_k12_stamps(unsigned long long* buf, int capacity, void* stream) {
    if (capacity < 0 || (buf == nullptr) != (capacity == 0)) return fail(-1, "bad stamp buffer");
    const fused::StampBuf sb{buf, capacity};
    const hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(fused::g_k12_stamp), &sb, sizeof(sb), 0,
                                                hipMemcpyHostToDevice, (hipStream_t)stream);
    if (e != hipSuccess) return fail((int)e, "psfm_k12_stamps: hipMemcpyToSymbolAsync failed");
    // the host struct is pageable: the async copy is staged before this returns, but keep the
    // call synchronous with the stream so the next launch surely sees the new pointer
    return hipStreamSynchronize((hipStream_t)stream) == hipSuccess ? 0 : fail(-3, "stream sync failed");
}

}  // extern "C"
