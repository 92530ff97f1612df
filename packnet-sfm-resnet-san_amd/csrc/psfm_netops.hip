// psfm_netops.hip — fused BatchNorm / GroupNorm / bias + activation kernels of the depth and
// pose networks (include/psfm_netops.h), gfx950.
//
// An activation is a bf16 matrix [M, C] (NHWC storage).  A workgroup of 256 threads covers TR
// rows x C channels per row step: thread t owns the VEC consecutive channels (t % G)*VEC.. of
// row lane t / G (G = C/VEC; VEC = 8: one 16-byte load per thread, fully coalesced rows) and
// walks its workgroup's row range in steps of U*TR rows with U independent loads in flight.
//
// Column reductions (batch statistics, bias / affine gradients) are deterministic and need no
// device-scope synchronisation: each workgroup writes its partial row (fp32 column sums of its
// rows, LDS tree over its row lanes), and the NEXT launch sums the rows in a fixed order in fp64
// (a small finish kernel, or — GroupNorm — the apply pass's prologue).  The kernel boundary is
// the barrier: at these sizes it is cheaper than arrival counters through the non-coherent
// per-XCD L2s (two device-scope rounds of 3-5 us each).  No float atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "../../include/psfm_netops.h"
#include "psfm_knobs.h"

using namespace psfm;

namespace {

thread_local std::string g_err;
int fail(int code, const char* msg) {
    g_err = msg;
    return code;
}
#define NETOPS_LAUNCH_CHECK()                                        \
    do {                                                             \
        hipError_t e_ = hipGetLastError();                           \
        if (e_ != hipSuccess) {                                      \
            g_err = std::string("launch: ") + hipGetErrorString(e_); \
            return (int)e_;                                          \
        }                                                            \
    } while (0)

constexpr int NT = 256;           // threads per workgroup
constexpr int U = 4;              // row steps unrolled (independent loads in flight per thread)
constexpr int TARGET_BLOCKS = 512;
constexpr int MAX_KC = 1024;      // widest partial row (BN: 2*C, C <= 512)

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even (NaN stays NaN)
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bfround(float f) { return bf2f(f2bf(f)); }

template <int VEC>
struct Vec {
    float v[VEC];
};

template <int VEC>
__device__ __forceinline__ Vec<VEC> zero() {
    Vec<VEC> r;
#pragma unroll
    for (int i = 0; i < VEC; ++i) r.v[i] = 0.0f;
    return r;
}

template <int VEC>
__device__ __forceinline__ Vec<VEC> ld_bf(const uint16_t* __restrict__ p) {
    Vec<VEC> r;
    if constexpr (VEC == 8) {
        const uint4 q = *reinterpret_cast<const uint4*>(p);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            r.v[2 * i] = __uint_as_float(w[i] << 16);
            r.v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) r.v[i] = bf2f(p[i]);
    }
    return r;
}

template <int VEC>
__device__ __forceinline__ void st_bf(uint16_t* __restrict__ p, const Vec<VEC>& a) {
    if constexpr (VEC == 8) {
        uint4 q;
        q.x = (uint32_t)f2bf(a.v[0]) | ((uint32_t)f2bf(a.v[1]) << 16);
        q.y = (uint32_t)f2bf(a.v[2]) | ((uint32_t)f2bf(a.v[3]) << 16);
        q.z = (uint32_t)f2bf(a.v[4]) | ((uint32_t)f2bf(a.v[5]) << 16);
        q.w = (uint32_t)f2bf(a.v[6]) | ((uint32_t)f2bf(a.v[7]) << 16);
        *reinterpret_cast<uint4*>(p) = q;
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) p[i] = f2bf(a.v[i]);
    }
}

// v += the bf16 vector at p (the residual input of a fused GroupNorm)
template <int VEC>
__device__ __forceinline__ void add_bf(Vec<VEC>& v, const uint16_t* __restrict__ p) {
    const Vec<VEC> r = ld_bf<VEC>(p);
#pragma unroll
    for (int i = 0; i < VEC; ++i) v.v[i] += r.v[i];
}

template <int VEC>
__device__ __forceinline__ Vec<VEC> ld_f(const float* __restrict__ p) {
    Vec<VEC> r;
    if constexpr (VEC == 8) {
        const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
        r.v[0] = a.x, r.v[1] = a.y, r.v[2] = a.z, r.v[3] = a.w;
        r.v[4] = b.x, r.v[5] = b.y, r.v[6] = b.z, r.v[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) r.v[i] = p[i];
    }
    return r;
}

template <int VEC>
__device__ __forceinline__ void st_f(float* __restrict__ p, const Vec<VEC>& a) {
    if constexpr (VEC == 8) {
        *reinterpret_cast<float4*>(p) = make_float4(a.v[0], a.v[1], a.v[2], a.v[3]);
        *reinterpret_cast<float4*>(p + 4) = make_float4(a.v[4], a.v[5], a.v[6], a.v[7]);
    } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) p[i] = a.v[i];
    }
}

// per-channel parameter vector (bf16 or fp32 storage)
template <int VEC>
__device__ __forceinline__ Vec<VEC> ld_param(const void* p, int bf, int c0) {
    Vec<VEC> r;
#pragma unroll
    for (int i = 0; i < VEC; ++i)
        r.v[i] = bf ? bf2f(static_cast<const uint16_t*>(p)[c0 + i]) : static_cast<const float*>(p)[c0 + i];
    return r;
}

// ------------------------------------------------------------------------------------------
// Work geometry of an [M, C] pass: G = C / VEC vector columns, TR = row lanes per workgroup,
// rpb = rows per workgroup (a multiple of U*TR), nblk workgroups (<= TARGET_BLOCKS).
// ------------------------------------------------------------------------------------------
struct Geo {
    int G, TR, rpb, nblk;
};
inline Geo geometry(int M, int C, int vec, int target = TARGET_BLOCKS) {
    Geo g;
    g.G = C / vec;
    g.TR = std::max(1, NT / g.G);
    const int step = g.TR * U;
    const int per = (M + target - 1) / target;
    g.rpb = std::max(step, (per + step - 1) / step * step);
    g.nblk = (M + g.rpb - 1) / g.rpb;
    return g;
}
inline int pick_vec(int C) { return (C % 8 == 0 && C / 8 <= NT) ? 8 : 1; }
__host__ __device__ inline size_t align4(size_t n) { return (n + 3) / 4 * 4; }  // 16-byte alignment

// Block column reduction of K per-thread vectors; afterwards row lane 0 holds the block sums.
// red: LDS [K * NT * VEC] floats (TR * G <= NT).
template <int VEC, int K>
__device__ __forceinline__ void block_colsum(float (&acc)[K][VEC], float* red, int G, int TR) {
    const int t = threadIdx.x;
    const int cg = t % G, r = t / G;
    const bool active = r < TR;
    if (active) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int i = 0; i < VEC; ++i) red[((k * TR + r) * G + cg) * VEC + i] = acc[k][i];
    }
    __syncthreads();
    for (int s = 1; s < TR; s <<= 1) {  // fixed-order tree over the row lanes
        if (active && (r % (2 * s)) == 0 && r + s < TR) {
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int i = 0; i < VEC; ++i)
                    red[((k * TR + r) * G + cg) * VEC + i] += red[((k * TR + r + s) * G + cg) * VEC + i];
        }
        __syncthreads();
    }
    if (active && r == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[k][i] = red[(k * TR * G + cg) * VEC + i];
    }
}

__device__ __forceinline__ float act_fwd(float v, int act) {
    if (act == PSFM_ACT_RELU) return fmaxf(v, 0.0f);
    if (act == PSFM_ACT_SIGMOID) return 1.0f / (1.0f + expf(-v));
    return v;
}

#define ROW_LOOP_BEGIN(ROW0, ROW1, R, TR)                           \
    for (int base_ = (ROW0) + (R); base_ < (ROW1); base_ += U * (TR)) {
#define ROW_LOOP_END }

// ------------------------------------------------------------------------------------------
// bias + activation (decoder ConvBlock / disparity head)
// ------------------------------------------------------------------------------------------
struct BiasArgs {
    const uint16_t* x;
    const void* bias;
    const void* dy;
    const void* dy1;  // bwd (ReLU, bf16): a second gradient of y summed into dy (its other consumer); may be null
    const void* y;
    void* out;  // y (fwd) / dx (bwd)
    float* ws;  // bwd: per-workgroup partial rows of the bias gradient [nblk][C]
    int M, C, act, bias_bf16, G, TR, rpb, nblk;
};

template <int VEC>
__global__ __launch_bounds__(NT) void k_bias_act_fwd(BiasArgs a) {
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    if (r >= a.TR) return;
    const int c0 = cg * VEC;
    const Vec<VEC> b = ld_param<VEC>(a.bias, a.bias_bf16, c0);
    const int row0 = blockIdx.x * a.rpb, row1 = min(a.M, row0 + a.rpb);
    ROW_LOOP_BEGIN(row0, row1, r, a.TR)
    Vec<VEC> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int row = base_ + u * a.TR;
        v[u] = row < row1 ? ld_bf<VEC>(a.x + (size_t)row * a.C + c0) : zero<VEC>();
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int row = base_ + u * a.TR;
        if (row >= row1) break;
        const size_t o = (size_t)row * a.C + c0;
#pragma unroll
        for (int i = 0; i < VEC; ++i) v[u].v[i] = act_fwd(v[u].v[i] + b.v[i], a.act);
        if (a.act == PSFM_ACT_SIGMOID)
            st_f<VEC>(static_cast<float*>(a.out) + o, v[u]);
        else
            st_bf<VEC>(static_cast<uint16_t*>(a.out) + o, v[u]);
    }
    ROW_LOOP_END
}

template <int VEC>
__global__ __launch_bounds__(NT) void k_bias_act_bwd(BiasArgs a) {
    __shared__ float red[NT * VEC];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    float acc[1][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = 0.0f;
    if (r < a.TR) {
        const int row0 = blockIdx.x * a.rpb, row1 = min(a.M, row0 + a.rpb);
        const bool sig = a.act == PSFM_ACT_SIGMOID;
        ROW_LOOP_BEGIN(row0, row1, r, a.TR)
        Vec<VEC> dy[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = base_ + u * a.TR;
            const size_t o = (size_t)row * a.C + c0;
            if (row < row1) {
                dy[u] = sig ? ld_f<VEC>(static_cast<const float*>(a.dy) + o)
                            : ld_bf<VEC>(static_cast<const uint16_t*>(a.dy) + o);
                if (a.dy1) {   // autograd's bf16 accumulation of the two gradients, in the load
                    const Vec<VEC> d1 = ld_bf<VEC>(static_cast<const uint16_t*>(a.dy1) + o);
#pragma unroll
                    for (int i = 0; i < VEC; ++i) dy[u].v[i] = bfround(dy[u].v[i] + d1.v[i]);
                }
                y[u] = sig ? ld_f<VEC>(static_cast<const float*>(a.y) + o)
                           : ld_bf<VEC>(static_cast<const uint16_t*>(a.y) + o);
            } else {
                dy[u] = zero<VEC>();
                y[u] = zero<VEC>();
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = base_ + u * a.TR;
            if (row >= row1) break;
            Vec<VEC> g;
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                if (sig)
                    g.v[i] = dy[u].v[i] * ((1.0f - y[u].v[i]) * y[u].v[i]);
                else
                    g.v[i] = (a.act == PSFM_ACT_RELU && !(y[u].v[i] > 0.0f)) ? 0.0f : dy[u].v[i];
            }
            st_bf<VEC>(static_cast<uint16_t*>(a.out) + (size_t)row * a.C + c0, g);
            // the stored (bf16) gradient is the one the bias sums, as autograd's would
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[0][i] += bfround(g.v[i]);
        }
        ROW_LOOP_END
    }
    // this workgroup's column sums -> its partial row; k_cols_finish sums the rows (next launch)
    block_colsum<VEC, 1>(acc, red, a.G, a.TR);
    if (r == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) a.ws[(size_t)blockIdx.x * a.C + c0 + i] = acc[0][i];
    }
}

// ------------------------------------------------------------------------------------------
// Column totals of partial rows, the second launch of every reduction above and below (no
// arrival counters: the kernel boundary orders the partial rows before their readers).
// Job j: out_j[c] = sum over rows r < nrows of src_j[r * stride + off + c], c < ncols, in fp64:
// lane l of 64 sums rows l, l + 64, ... (8 loads in flight per thread), then a fixed tree over
// the lanes — deterministic.  Workgroup = 4 columns x 64 lanes; grid (ceil(cols / 4), jobs).
// ------------------------------------------------------------------------------------------
struct ColJob {
    const float* src;
    void* out;
    int stride, off, nrows, ncols, out_bf16;
};
struct FinishArgs {
    ColJob job[3];
};

__global__ __launch_bounds__(256) void k_cols_finish(FinishArgs a) {
    __shared__ double part[256];
    const ColJob j = a.job[blockIdx.y];
    const int t = threadIdx.x, cl = t & 3, lane = t >> 2;
    const int c = blockIdx.x * 4 + cl;
    double s = 0.0;
    if (c < j.ncols) {
        for (int r0 = lane; r0 < j.nrows; r0 += 8 * 64) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int rr = r0 + u * 64;
                v[u] = rr < j.nrows ? j.src[(size_t)rr * j.stride + j.off + c] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (double)v[u];
        }
    }
    part[t] = s;
    __syncthreads();
    for (int h = 32; h >= 1; h >>= 1) {
        if (lane < h) part[t] += part[t + 4 * h];
        __syncthreads();
    }
    if (lane == 0 && c < j.ncols) {
        if (j.out_bf16)
            static_cast<uint16_t*>(j.out)[c] = f2bf((float)part[t]);
        else
            static_cast<float*>(j.out)[c] = (float)part[t];
    }
}

inline hipError_t launch_finish(const ColJob* jobs, int njobs, hipStream_t st) {
    FinishArgs a{};
    int cols = 1;
    for (int k = 0; k < njobs; ++k) {
        a.job[k] = jobs[k];
        cols = std::max(cols, jobs[k].ncols);
    }
    hipLaunchKernelGGL(k_cols_finish, dim3((cols + 3) / 4, njobs), dim3(256), 0, st, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// BatchNorm (training) + residual + ReLU
// ------------------------------------------------------------------------------------------
__host__ __device__ inline size_t bn_coef_off(int nblk, int C) { return align4((size_t)nblk * 2 * C); }

// ------------------------------------------------------------------------------------------
// Resident BatchNorm: ONE launch each way for the small encoder layers (M = N*H*W rows up to the
// BN_RES_MAXM knob, 2048 by default = ResNet18 layer3 / layer4 at B = 4, 192x640; the kernels hold up
// to 8192, but at layer2's 7680 rows the 16-byte per-lane row loads of 16 workgroups lose to MIOpen,
// psfm_knobs.hip).  A workgroup owns 8 channels and ALL M rows of them: thread t
// holds rows t, t + NTH, ... (RPT 16-byte row vectors, <= 8 per tensor) in registers, so the batch
// statistics (two passes over the registers: mean, then sum (x - mean)^2 — no E[x^2] - mean^2
// cancellation), the running-stat update and the apply need no other workgroup, and the backward's
// dgamma / dbeta are complete in the workgroup (no partial rows, no finish kernel).  Reductions: xor
// butterflies within the wave, then the waves' rows in order in fp64 — fixed order, deterministic.
// The workgroup -> channel-block map is XCD-aware (workgroup w runs on XCD w % 8; an XCD gets a
// contiguous channel range, so the blocks sharing a 128-byte row line mostly share an L2).
// Replaces MIOpen's 3 + 3 BN kernels and the ReLU / add+ReLU / ReLU-mask passes around them.
// ------------------------------------------------------------------------------------------
constexpr int BNR_MAXT = 1024;  // threads per workgroup (<= 16 waves)
constexpr int BNR_MAXM = 8 * BNR_MAXT;

struct BNRArgs {
    const uint16_t* x;
    const uint16_t* res;
    const uint16_t* dy;
    const uint16_t* y;
    const float* gamma;
    const float* beta;
    float* run_mean;
    float* run_var;
    float* save_mean;
    float* save_invstd;
    uint16_t* out;   // y (fwd) / dx (bwd)
    uint16_t* dres;  // bwd, may be null
    const uint16_t* dy1;  // bwd: more gradients of the output (its other consumers), summed into dy; may be null
    const uint16_t* dy2;
    float* dgamma;
    float* dbeta;
    float momentum, eps;
    int M, C, relu, nb;  // nb = C / 8 channel blocks = workgroups
};

__device__ __forceinline__ int bnr_block(int w, int nb) { return (nb % 8 == 0) ? (w % 8) * (nb / 8) + w / 8 : w; }

// per-channel totals over the workgroup of K per-thread partials -> tot[K] (fp64, every thread
// reads them after the call).  Within a wave: xor butterflies 1 / 2 (DPP quad_perm), 4 (DPP
// row_half_mirror), 8 (DPP row_mirror) — every lane of a 16-lane row then holds the row sum — and
// 16 / 32 (lane shuffles); then the waves' sums in order in fp64.  Fixed order: deterministic.
// red: LDS [16][K] floats.
__device__ __forceinline__ float dpp_add(float v, int ctrl_sel) {
    switch (ctrl_sel) {  // compile-time after unrolling
        case 0: return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
        case 1: return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
        case 2: return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
        default: return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
    }
}

template <int K>
__device__ __forceinline__ void bnr_reduce(float (&v)[K], float* red, double* tot) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = dpp_add(v[k], st);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        v[k] += __shfl_xor(v[k], 16, 64);
        v[k] += __shfl_xor(v[k], 32, 64);
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) red[w * K + k] = v[k];
    }
    __syncthreads();
    if (t < K) {
        float part[BNR_MAXT / 64];
#pragma unroll
        for (int ww = 0; ww < BNR_MAXT / 64; ++ww) part[ww] = ww < nw ? red[ww * K + t] : 0.0f;
        double s = 0.0;
#pragma unroll
        for (int ww = 0; ww < BNR_MAXT / 64; ++ww) s += (double)part[ww];
        tot[t] = s;
    }
    __syncthreads();
}

// a + b of two packed bf16 row vectors, rounded to bf16: what autograd's accumulation of two bf16
// gradients of one tensor computes (CUDAFunctor_add<bf16>: fp32 sum, one rounding)
__device__ __forceinline__ uint4 add_bf16x8(const uint4 a, const uint4 b) {
    const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, bw[4] = {b.x, b.y, b.z, b.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float lo = __uint_as_float(aw[k] << 16) + __uint_as_float(bw[k] << 16);
        const float hi = __uint_as_float(aw[k] & 0xffff0000u) + __uint_as_float(bw[k] & 0xffff0000u);
        o[k] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// relu-mask a packed bf16 row vector by the forward output: ATen threshold_backward (y <= 0 -> 0)
__device__ __forceinline__ uint4 relu_mask4(uint4 g, uint4 y) {
    const uint32_t gw[4] = {g.x, g.y, g.z, g.w}, vw[4] = {y.x, y.y, y.z, y.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t lo = (__uint_as_float(vw[k] << 16) <= 0.0f) ? 0u : 0x0000ffffu;
        const uint32_t hi = (__uint_as_float(vw[k] & 0xffff0000u) <= 0.0f) ? 0u : 0xffff0000u;
        o[k] = gw[k] & (lo | hi);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

__device__ __forceinline__ void unpack8f(const uint4 q, float (&v)[8]) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}

template <int RPT, bool RES>
__global__ __launch_bounds__(BNR_MAXT) void k_bnr_fwd(BNRArgs a) {
    __shared__ float red[16 * 16];
    __shared__ double tot[16];
    const int t = threadIdx.x, NTH = blockDim.x;
    const int c0 = bnr_block(blockIdx.x, a.nb) * 8;
    uint4 xv[RPT], rv[RES ? RPT : 1];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {  // every load issued before the first use (clamped rows, masked below)
        const size_t o = (size_t)min(t + k * NTH, a.M - 1) * a.C + c0;
        xv[k] = *reinterpret_cast<const uint4*>(a.x + o);
        if constexpr (RES) rv[k] = *reinterpret_cast<const uint4*>(a.res + o);
    }
    // one reduction of sums shifted by the channel's first value K (sum (x - K), sum (x - K)^2): the
    // variance E[(x-K)^2] - E[x-K]^2 keeps no E[x^2] - mean^2 cancellation when |mean| >> std
    float kk[8];
    unpack8f(*reinterpret_cast<const uint4*>(a.x + c0), kk);
    float s[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = 0.0f;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (t + k * NTH >= a.M) break;
        float v[8];
        unpack8f(xv[k], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float d = v[i] - kk[i];
            s[i] += d;
            s[8 + i] += d * d;
        }
    }
    bnr_reduce<16>(s, red, tot);
    const double inv_m = 1.0 / (double)a.M;
    float mu[8];
    double var8[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double m1 = tot[i] * inv_m;
        mu[i] = (float)((double)kk[i] + m1);
        var8[i] = fmax(tot[8 + i] * inv_m - m1 * m1, 0.0);
    }
    float sc[8], sh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double var = var8[i];
        const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
        sc[i] = a.gamma[c0 + i] * invstd;
        sh[i] = a.beta[c0 + i] - mu[i] * sc[i];
        if (t == i) {
            a.save_mean[c0 + i] = mu[i];
            a.save_invstd[c0 + i] = invstd;
            if (a.run_mean) {  // torch: running = (1-m) running + m batch (unbiased var)
                const double unb = a.M > 1 ? var * (double)a.M / (double)(a.M - 1) : var;
                a.run_mean[c0 + i] = (float)((1.0 - a.momentum) * a.run_mean[c0 + i] + a.momentum * (double)mu[i]);
                a.run_var[c0 + i] = (float)((1.0 - a.momentum) * a.run_var[c0 + i] + a.momentum * unb);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int row = t + k * NTH;
        if (row >= a.M) break;
        float v[8];
        unpack8f(xv[k], v);
        float r[8];
        if constexpr (RES) unpack8f(rv[k], r);
        Vec<8> o;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float w = v[i] * sc[i] + sh[i];
            if constexpr (RES) w = bfround(w) + r[i];  // autocast: bn(x) is a bf16 tensor before the add
            if (a.relu) w = w <= 0.0f ? 0.0f : w;      // ATen relu (NaN propagates)
            o.v[i] = w;
        }
        st_bf<8>(a.out + (size_t)row * a.C + c0, o);
    }
}

// backward: x and the masked dy held (16 VGPRs per row vector pair): RPT >= 8 runs 512-thread
// workgroups (256 VGPRs; 1024 threads x RPT 8 spilled at the 128-VGPR limit)
constexpr int bnr_bwd_maxt(int rpt) { return rpt >= 8 ? BNR_MAXT / 2 : BNR_MAXT; }

template <int RPT>
__global__ __launch_bounds__(bnr_bwd_maxt(RPT)) void k_bnr_bwd(BNRArgs a) {
    __shared__ float red[16 * 16];
    __shared__ double tot[16];
    const int t = threadIdx.x, NTH = blockDim.x;
    const int c0 = bnr_block(blockIdx.x, a.nb) * 8;
    uint4 gv[RPT], xv[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const size_t o = (size_t)min(t + k * NTH, a.M - 1) * a.C + c0;
        gv[k] = *reinterpret_cast<const uint4*>(a.dy + o);
        xv[k] = *reinterpret_cast<const uint4*>(a.x + o);
        if (a.dy1) gv[k] = add_bf16x8(gv[k], *reinterpret_cast<const uint4*>(a.dy1 + o));   // wave-uniform
        if (a.dy2) gv[k] = add_bf16x8(gv[k], *reinterpret_cast<const uint4*>(a.dy2 + o));
        if (a.relu) gv[k] = relu_mask4(gv[k], *reinterpret_cast<const uint4*>(a.y + o));
    }
    float mu[8], is[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        mu[i] = a.save_mean[c0 + i];
        is[i] = a.save_invstd[c0 + i];
    }
    float acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (t + k * NTH >= a.M) break;
        float g[8], v[8];
        unpack8f(gv[k], g);
        unpack8f(xv[k], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            acc[i] += g[i];
            acc[8 + i] += g[i] * (v[i] - mu[i]);
        }
    }
    bnr_reduce<16>(acc, red, tot);
    // dx = k1 (g - k2 - (x - mu) k3) with k1 = gamma invstd, k2 = sum g / M, k3 = sum g (x - mu) invstd^2 / M,
    // folded (fp64) into dx = kg g + kx x + k0: three live coefficients per channel instead of five
    const double inv_m = 1.0 / (double)a.M;
    float kg[8], kx[8], k0[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double isd = is[i], k1 = (double)(a.gamma[c0 + i] * is[i]);
        const double k2 = tot[i] * inv_m, k3 = tot[8 + i] * isd * isd * inv_m;
        kg[i] = (float)k1;
        kx[i] = (float)(-k1 * k3);
        k0[i] = (float)(k1 * (k3 * (double)mu[i] - k2));
        if (t == i) {
            a.dbeta[c0 + i] = (float)tot[i];
            a.dgamma[c0 + i] = (float)(tot[8 + i] * isd);
        }
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int row = t + k * NTH;
        if (row >= a.M) break;
        const size_t o = (size_t)row * a.C + c0;
        float g[8], v[8];
        unpack8f(gv[k], g);
        unpack8f(xv[k], v);
        Vec<8> d;
#pragma unroll
        for (int i = 0; i < 8; ++i) d.v[i] = fmaf(kg[i], g[i], fmaf(kx[i], v[i], k0[i]));
        st_bf<8>(a.out + o, d);
        if (a.dres) *reinterpret_cast<uint4*>(a.dres + o) = gv[k];
    }
}

// resident geometry: RPT = the fewest row vectors per thread with RPT x (the direction's thread
// limit) >= M (forward RPT 1-8 at <= 1024 threads; backward RPT 1-4 at 1024, 8 / 16 at 512), NTH =
// ceil(M / RPT) rounded up to whole waves; false when the layer does not fit
struct BNRGeo {
    int rpt, nth;
};
// The forward applies the BN_RES_MAXM policy; the backward takes whatever the kernels hold (up to
// BNR_MAXM rows), so it follows the forward's decision even if the knob changed in between.
inline bool bnr_geometry(int M, int C, BNRGeo& g, bool bwd = false) {
    if (C % 8 || C > 512 || M < 1 || M > (bwd ? BNR_MAXM : std::min(BNR_MAXM, knob(KNOB_BN_RES_MAXM)))) return false;
    for (int r = 1; r <= (bwd ? 16 : 8); r *= 2) {
        const int maxt = bwd ? bnr_bwd_maxt(r) : BNR_MAXT;
        if ((long long)r * maxt >= M) {
            g.rpt = r;
            g.nth = std::max(64, ((M + r - 1) / r + 63) / 64 * 64);
            return true;
        }
    }
    return false;
}

#define BNR_FWD_CASE(R)                                                                                  \
    case R:                                                                                              \
        if (res) hipLaunchKernelGGL((k_bnr_fwd<R, true>), dim3(a.nb), dim3(g.nth), 0, st, a);           \
        else hipLaunchKernelGGL((k_bnr_fwd<R, false>), dim3(a.nb), dim3(g.nth), 0, st, a);              \
        break
#define BNR_BWD_CASE(R)                                                                                  \
    case R: hipLaunchKernelGGL((k_bnr_bwd<R>), dim3(a.nb), dim3(g.nth), 0, st, a); break


// ------------------------------------------------------------------------------------------
// GroupNorm(NG) of (x [+ res] + bias) + ReLU / ELU, per sample n over rows [n*HW, (n+1)*HW),
// bpn workgroups per sample.  No arrival counters: each pass writes per-workgroup partial rows
// and the NEXT launch reduces what it needs in a fixed order —
//   forward:  stats (rows of per-group sum / sum of squares, 2*NG floats) -> apply (every
//             workgroup sums its sample's bpn group rows in its prologue: mean / invstd);
//   backward: stats (rows of per-group A = sum gamma*dyr, Bq = sum gamma*dyr*xhat and
//             per-channel S1 = sum dyr, S2 = sum dyr*xhat, X = sum xhat) -> apply (prologue: A, Bq
//             of its sample -> dx coefficients) whose last ceil(C/4) workgroups finish the
//             parameter gradients from the same rows: dbeta = sum S1, dgamma = sum S2 and the conv
//             bias gradient in closed form, sum_hw dx = k1*S1 - HW*k2 - k3*X per sample.
// The apply passes issue their first activation loads before the prologue, so the per-sample
// reduction (bpn x 2*NG floats, L2-resident) overlaps them: two launches each way, no rounds.
// ------------------------------------------------------------------------------------------
// GroupNorm activations: ReLU (PoseNet conv_gn) or ELU(alpha = 1) (PackNet Conv2D / ResidualConv,
// layers01.py:10-37, :40-61: x > 0 ? x : expm1(x); backward from the result: y > 0 ? g : g (y + 1))
__device__ __forceinline__ float gn_act_f(float w, int act) {
    if (act == PSFM_ACT_RELU) return fmaxf(w, 0.0f);
    if (act == PSFM_ACT_ELU) return w > 0.0f ? w : expm1f(w);
    return w;
}
// backward of the activation from its input w (recomputed from x, mean / invstd, gamma / beta: the
// output y is not read back)
__device__ __forceinline__ float gn_act_g(float g, float w, int act) {
    if (act == PSFM_ACT_RELU) return w > 0.0f ? g : 0.0f;
    if (act == PSFM_ACT_ELU) return w > 0.0f ? g : g * expf(w);
    return g;
}

constexpr int MAX_C = 512;   // widest GroupNorm layer (PackNet encoder: 512)
constexpr int MAX_NG = 128;  // 2 * NG partial columns must fit one workgroup

struct GNArgs {
    const uint16_t* x;
    const uint16_t* res;  // optional second input summed with x (PackNet ResidualConv)
    const void* bias;     // optional (null = 0)
    const uint16_t* dy;
    const float* gamma;
    const float* beta;
    float* save_mean;    // [N*NG]
    float* save_invstd;  // [N*NG]
    uint16_t* out;
    uint16_t* out2;       // backward: dres (a second copy of dx) when res is given
    void* dbias;          // backward: conv-bias gradient (bias dtype) or null
    float* dgamma;
    float* dbeta;
    float* ws;            // stats rows [N*bpn][RW]
    float eps;
    int N, HW, C, NG, act, bias_bf16, G, TR, rpb, bpn, RW;  // act: PSFM_ACT_*; bpn: workgroups per sample
};

// tot[j] = sum over the sample's nrows partial rows (stride RW) of column j < KC, fp64, rows split
// over NT/KC lanes in a fixed order; every thread of the workgroup takes part (barriers inside).
__device__ void group_totals(const float* rows, int nrows, int RW, int KC, double* tot, double* scr) {
    const int t = threadIdx.x, L = NT / KC, j = t % KC, l = t / KC;
    if (l < L) {
        double s = 0.0;
        for (int r0 = l; r0 < nrows; r0 += 8 * L) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int rr = r0 + u * L;
                v[u] = rr < nrows ? rows[(size_t)rr * RW + j] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (double)v[u];
        }
        scr[l * KC + j] = s;
    }
    __syncthreads();
    if (t < KC) {
        double s = 0.0;
        for (int ll = 0; ll < L; ++ll) s += scr[ll * KC + t];
        tot[t] = s;
    }
    __syncthreads();
}

// per-channel column sums (row lane 0 of block_colsum) -> LDS chan[k][C]
template <int VEC, int K>
__device__ __forceinline__ void chan_to_lds(const float (&acc)[K][VEC], float* chan, int C, int c0, int r) {
    if (r == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int i = 0; i < VEC; ++i) chan[k * C + c0 + i] = acc[k][i];
    }
    __syncthreads();
}

// forward pass 1: per (workgroup, group) sum / sumsq of x (+ res) + bias -> partial row [2][NG]
template <int VEC>
__global__ __launch_bounds__(NT) void k_gn_fwd_stats(GNArgs a) {
    __shared__ float red[2 * NT * VEC];
    __shared__ float chan[2 * MAX_C];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    float acc[2][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = acc[1][i] = 0.0f;
    if (r < a.TR) {
        const Vec<VEC> b = a.bias ? ld_param<VEC>(a.bias, a.bias_bf16, c0) : zero<VEC>();
        const uint16_t* xs = a.x + (size_t)n * a.HW * a.C;
        const uint16_t* rs = a.res ? a.res + (size_t)n * a.HW * a.C : nullptr;
        const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
        ROW_LOOP_BEGIN(row0, row1, r, a.TR)
        Vec<VEC> v[U];
        bool in[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = base_ + u * a.TR;
            in[u] = row < row1;
            v[u] = in[u] ? ld_bf<VEC>(xs + (size_t)row * a.C + c0) : zero<VEC>();
            if (rs && in[u]) add_bf<VEC>(v[u], rs + (size_t)row * a.C + c0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const float w = in[u] ? v[u].v[i] + b.v[i] : 0.0f;
                acc[0][i] += w;
                acc[1][i] += w * w;
            }
        ROW_LOOP_END
    }
    block_colsum<VEC, 2>(acc, red, a.G, a.TR);
    chan_to_lds<VEC, 2>(acc, chan, a.C, c0, r);
    const int cpg = a.C / a.NG;
    float* row = a.ws + (size_t)blockIdx.x * a.RW;
    for (int j = t; j < 2 * a.NG; j += NT) {  // group sums in channel order
        const int k = j / a.NG, g = j - k * a.NG;
        float s = 0.0f;
        for (int u = 0; u < cpg; ++u) s += chan[k * a.C + g * cpg + u];
        row[j] = s;
    }
}

// forward pass 2: prologue = this sample's group statistics from the stats rows; y = act(...).
// The first U rows of every thread are loaded before the prologue (their latency overlaps it).
template <int VEC>
__global__ __launch_bounds__(NT) void k_gn_fwd_apply(GNArgs a) {
    __shared__ double tot[2 * MAX_NG];
    __shared__ double scr[NT];
    __shared__ float gmean[MAX_NG], ginv[MAX_NG];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const size_t so = (size_t)n * a.HW * a.C;
    const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
    const bool live = r < a.TR;
    Vec<VEC> v[U];
    auto load = [&](int base) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = base + u * a.TR;
            v[u] = row < row1 ? ld_bf<VEC>(a.x + so + (size_t)row * a.C + c0) : zero<VEC>();
            if (a.res && row < row1) add_bf<VEC>(v[u], a.res + so + (size_t)row * a.C + c0);
        }
    };
    if (live) load(row0 + r);
    group_totals(a.ws + (size_t)n * a.bpn * a.RW, a.bpn, a.RW, 2 * a.NG, tot, scr);
    const int cpg = a.C / a.NG;
    if (t < a.NG) {
        const double inv_cnt = 1.0 / ((double)a.HW * cpg);
        const double mean = tot[t] * inv_cnt;
        const double var = fmax(tot[a.NG + t] * inv_cnt - mean * mean, 0.0);
        const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
        gmean[t] = (float)mean;
        ginv[t] = invstd;
        if (bl == 0) {
            a.save_mean[n * a.NG + t] = (float)mean;
            a.save_invstd[n * a.NG + t] = invstd;
        }
    }
    __syncthreads();
    if (!live) return;
    Vec<VEC> sc, sh;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
        const int g = (c0 + i) / cpg;
        sc.v[i] = a.gamma[c0 + i] * ginv[g];
        sh.v[i] = a.beta[c0 + i] - gmean[g] * sc.v[i];
    }
    const Vec<VEC> b = a.bias ? ld_param<VEC>(a.bias, a.bias_bf16, c0) : zero<VEC>();
    for (int base = row0 + r; base < row1; base += U * a.TR) {
        if (base != row0 + r) load(base);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = base + u * a.TR;
            if (row >= row1) break;
#pragma unroll
            for (int i = 0; i < VEC; ++i) v[u].v[i] = gn_act_f((v[u].v[i] + b.v[i]) * sc.v[i] + sh.v[i], a.act);
            st_bf<VEC>(a.out + so + (size_t)row * a.C + c0, v[u]);
        }
    }
}

// backward pass 1: per workgroup: S1 = sum dyr, S2 = sum dyr*xhat, X = sum xhat per channel, and
// per group A = sum_{c in g} gamma S1, Bq = sum_{c in g} gamma S2
// -> row [A(NG) | Bq(NG) | S1(C) | S2(C) | X(C)]
template <int VEC>
__global__ __launch_bounds__(NT) void k_gn_bwd_stats(GNArgs a) {
    __shared__ float red[3 * NT * VEC];
    __shared__ float chan[3 * MAX_C];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const int cpg = a.C / a.NG;
    float acc[3][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = acc[1][i] = acc[2][i] = 0.0f;
    if (r < a.TR) {
        const Vec<VEC> b = a.bias ? ld_param<VEC>(a.bias, a.bias_bf16, c0) : zero<VEC>();
        float mu[VEC], is[VEC];
        float ga[VEC], be[VEC];
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            mu[i] = a.save_mean[n * a.NG + (c0 + i) / cpg];
            is[i] = a.save_invstd[n * a.NG + (c0 + i) / cpg];
            ga[i] = a.gamma[c0 + i];
            be[i] = a.beta[c0 + i];
        }
        const size_t so = (size_t)n * a.HW * a.C;
        const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
        ROW_LOOP_BEGIN(row0, row1, r, a.TR)
        Vec<VEC> g[U], x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = base_ + u * a.TR;
            const size_t o = so + (size_t)row * a.C + c0;
            const bool in = row < row1;
            g[u] = in ? ld_bf<VEC>(a.dy + o) : zero<VEC>();
            x[u] = in ? ld_bf<VEC>(a.x + o) : zero<VEC>();
            if (a.res && in) add_bf<VEC>(x[u], a.res + o);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in_u = base_ + u * a.TR < row1;
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const float xh = (x[u].v[i] + b.v[i] - mu[i]) * is[i];
                const float gg = gn_act_g(g[u].v[i], xh * ga[i] + be[i], a.act);
                acc[0][i] += gg;
                acc[1][i] += gg * xh;
                acc[2][i] += in_u ? xh : 0.0f;
            }
        }
        ROW_LOOP_END
    }
    block_colsum<VEC, 3>(acc, red, a.G, a.TR);
    chan_to_lds<VEC, 3>(acc, chan, a.C, c0, r);
    float* row = a.ws + (size_t)blockIdx.x * a.RW;
    for (int j = t; j < 2 * a.NG; j += NT) {
        const int k = j / a.NG, g = j - k * a.NG;
        float s = 0.0f;
        for (int u = 0; u < cpg; ++u) s += a.gamma[g * cpg + u] * chan[k * a.C + g * cpg + u];
        row[j] = s;
    }
    for (int j = t; j < 3 * a.C; j += NT) row[2 * a.NG + j] = chan[j];
}

// parameter gradients from the backward stats rows (the last ceil(C/4) workgroups of the apply
// launch): workgroup = 4 channels x 64 lanes, lane l works on sample l / (64 / N) (N <= 64) and sums
// its share of that sample's rows (fp64, fixed order) -> per (sample, channel) S1, S2, X and the
// sample's group totals A, Bq -> dbeta = sum_n S1, dgamma = sum_n S2,
// dbias = sum_n (k1 S1 - HW k2 - k3 X) (k as in the apply pass, in fp64).
__device__ void gn_bwd_params(const GNArgs& a, int f) {
    __shared__ double part[5][NT];
    __shared__ double nt[5][64][4];
    const int t = threadIdx.x, cl = t & 3, lane = t >> 2;
    const int c = f * 4 + cl;
    const int lpn = 64 / a.N, n = lane / lpn, li = lane % lpn;
    const int cpg = a.C / a.NG;
    double s[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    if (c < a.C && n < a.N) {
        const int g = c / cpg;
        const int col[5] = {2 * a.NG + c, 2 * a.NG + a.C + c, 2 * a.NG + 2 * a.C + c, g, a.NG + g};
        for (int r0 = li; r0 < a.bpn; r0 += 2 * lpn) {
            float v[2][5];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int rr = r0 + u * lpn;
                const float* row = a.ws + (size_t)(n * a.bpn + (rr < a.bpn ? rr : 0)) * a.RW;
#pragma unroll
                for (int k = 0; k < 5; ++k) v[u][k] = rr < a.bpn ? row[col[k]] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int k = 0; k < 5; ++k) s[k] += (double)v[u][k];
        }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) part[k][t] = s[k];
    __syncthreads();
    if (t < 4 * a.N) {   // per (sample, channel): lanes in order
        const int cc = t & 3, nn = t >> 2;
        for (int k = 0; k < 5; ++k) {
            double q = 0.0;
            for (int l = 0; l < lpn; ++l) q += part[k][((nn * lpn + l) << 2) | cc];
            nt[k][nn][cc] = q;
        }
    }
    __syncthreads();
    if (t < 4 && c < a.C) {
        const int g = c / cpg;
        const double cnt = (double)a.HW * cpg, ga = a.gamma[c];
        double db = 0.0, dg = 0.0, dbias = 0.0;
        for (int nn = 0; nn < a.N; ++nn) {
            const double S1 = nt[0][nn][t], S2 = nt[1][nn][t], X = nt[2][nn][t];
            const double is = a.save_invstd[nn * a.NG + g];
            db += S1;
            dg += S2;
            dbias += ga * is * S1 - (double)a.HW * (nt[3][nn][t] / cnt * is) - (nt[4][nn][t] / cnt * is) * X;
        }
        a.dbeta[c] = (float)db;
        a.dgamma[c] = (float)dg;
        if (a.dbias) {
            if (a.bias_bf16)
                static_cast<uint16_t*>(a.dbias)[c] = f2bf((float)dbias);
            else
                static_cast<float*>(a.dbias)[c] = (float)dbias;
        }
    }
}

// backward pass 2: prologue = A, Bq of this sample -> dx = k1*dyr - k2 - xhat*k3 with
// k1 = gamma*invstd, k2 = A/cnt*invstd, k3 = Bq/cnt*invstd, xhat = (x + bias - mean)*invstd.
// Workgroups past N*bpn compute the parameter gradients (gn_bwd_params).
template <int VEC>
__global__ __launch_bounds__(NT) void k_gn_bwd_apply(GNArgs a) {
    if ((int)blockIdx.x >= a.N * a.bpn) {
        gn_bwd_params(a, blockIdx.x - a.N * a.bpn);
        return;
    }
    __shared__ double tot[2 * MAX_NG];
    __shared__ double scr[NT];
    __shared__ float gk2[MAX_NG], gk3[MAX_NG];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const int cpg = a.C / a.NG;
    const size_t so = (size_t)n * a.HW * a.C;
    const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
    const bool live = r < a.TR;
    Vec<VEC> g[U], x[U];
    auto load = [&](int base) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = base + u * a.TR;
            const size_t o = so + (size_t)row * a.C + c0;
            const bool in = row < row1;
            g[u] = in ? ld_bf<VEC>(a.dy + o) : zero<VEC>();
            x[u] = in ? ld_bf<VEC>(a.x + o) : zero<VEC>();
            if (a.res && in) add_bf<VEC>(x[u], a.res + o);
        }
    };
    if (live) load(row0 + r);
    group_totals(a.ws + (size_t)n * a.bpn * a.RW, a.bpn, a.RW, 2 * a.NG, tot, scr);
    if (t < a.NG) {
        const double cnt = (double)a.HW * cpg;
        const double is = a.save_invstd[n * a.NG + t];
        gk2[t] = (float)(tot[t] / cnt * is);
        gk3[t] = (float)(tot[a.NG + t] / cnt * is);
    }
    __syncthreads();
    if (!live) return;
    const Vec<VEC> b = a.bias ? ld_param<VEC>(a.bias, a.bias_bf16, c0) : zero<VEC>();
    float mu[VEC], is[VEC], ga[VEC], be[VEC], k1[VEC], k2[VEC], k3[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
        const int gi = (c0 + i) / cpg;
        mu[i] = a.save_mean[n * a.NG + gi];
        is[i] = a.save_invstd[n * a.NG + gi];
        ga[i] = a.gamma[c0 + i];
        be[i] = a.beta[c0 + i];
        k1[i] = ga[i] * is[i];
        k2[i] = gk2[gi];
        k3[i] = gk3[gi];
    }
    for (int base = row0 + r; base < row1; base += U * a.TR) {
        if (base != row0 + r) load(base);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = base + u * a.TR;
            if (row >= row1) break;
            Vec<VEC> d;
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const float xh = (x[u].v[i] + b.v[i] - mu[i]) * is[i];
                const float gg = gn_act_g(g[u].v[i], xh * ga[i] + be[i], a.act);
                d.v[i] = k1[i] * gg - k2[i] - xh * k3[i];
            }
            st_bf<VEC>(a.out + so + (size_t)row * a.C + c0, d);
            if (a.out2) st_bf<VEC>(a.out2 + so + (size_t)row * a.C + c0, d);
        }
    }
}

// ------------------------------------------------------------------------------------------
// One-pass ("resident") GroupNorm for the layers whose (sample, channel block) fits the registers
// of one workgroup — every PackNet / PoseNet layer below 96x320 (layers01.py:10-72, PoseNet.py:15-19):
// a workgroup owns sample n and CB consecutive channels = gpw whole groups (CB = cpg, or 8 channels
// = 8 / cpg groups when cpg < 8, so every pixel run is one or more 16-byte vectors), holds its
// RPT row vectors per thread in registers, reduces the group statistics in-workgroup (fixed-order
// wave butterflies, then fp64 over the waves) and applies them from the registers:
//   forward  ONE launch (read x [+ res] once, write y)        instead of stats + apply (2 reads);
//   backward ONE data launch (read dy, x [+ res] once, write dx [+ dres]) + a one-workgroup
//            parameter finish (per-(sample, channel) partial rows -> dgamma, dbeta, dbias),
//            instead of stats + apply (2 reads of dy and x).
// Same arithmetic as the two-pass kernels (fp32 per thread, fp64 totals; the conv-bias gradient
// in the closed form sum_hw dx = k1 S1 - HW k2 - k3 X per sample, fp64); deterministic.
// ------------------------------------------------------------------------------------------
constexpr int RNT = 256;  // threads per workgroup

struct GNRArgs {
    const uint16_t* x;
    const uint16_t* res;
    const void* bias;
    const uint16_t* dy;
    const float* gamma;
    const float* beta;
    float* save_mean;
    float* save_invstd;
    uint16_t* out;
    uint16_t* out2;
    float* part;      // backward: [N][3][C] per-sample S1 | S2 | conv-bias partials
    void* dbias;
    float* dgamma;
    float* dbeta;
    float eps;
    int N, HW, C, NG, act, bias_bf16;
    int cpg, CB, CV, gpw, nblk;  // channels per group / per workgroup, 16-byte columns, groups per workgroup,
                                 // workgroups per sample
};

// sum over the lanes of this wave that share t % CV (CV = 1, 2, 4): xor butterflies CV..32, fixed order
template <int K>
__device__ __forceinline__ void wave_colsum(float (&v)[K], int CV) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        if (off < CV) break;
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] += __shfl_xor(v[k], off, 64);
    }
}

// per-channel totals of K per-thread accumulators [K][8] over the workgroup -> tot[k * CB + c] (fp64)
// red: LDS [waves][CV][K*8] floats
template <int K>
__device__ __forceinline__ void wg_chan_totals(float (&acc)[K * 8], float* red, double* tot, int CV, int CB) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, nw = blockDim.x >> 6;
    wave_colsum<K * 8>(acc, CV);
    if (lane < CV) {
#pragma unroll
        for (int k = 0; k < K * 8; ++k) red[(w * CV + lane) * (K * 8) + k] = acc[k];
    }
    __syncthreads();
    for (int j = t; j < K * CB; j += blockDim.x) {
        const int k = j / CB, c = j - k * CB, cv = c >> 3, i = c & 7;
        double s = 0.0;
        for (int ww = 0; ww < nw; ++ww) s += (double)red[(ww * CV + cv) * (K * 8) + k * 8 + i];
        tot[j] = s;
    }
    __syncthreads();
}

// the held row vectors become opaque across the reduction: the apply pass re-unpacks them from the
// packed bf16 registers instead of the compiler keeping every unpacked fp32 value live (2x VGPRs)
__device__ __forceinline__ void opaque4(uint4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }

template <int RPT, bool RES>
__global__ __launch_bounds__(RNT) void k_gnr_fwd(GNRArgs a) {
    __shared__ float red[(RNT / 64) * 4 * 16];
    __shared__ double tot[2 * 32];
    __shared__ float gsc[32], gsh[32];
    const int t = threadIdx.x, cv = t % a.CV, r = t / a.CV, RL = blockDim.x / a.CV;
    const int n = blockIdx.x / a.nblk, blk = blockIdx.x - n * a.nblk;
    const int c0 = blk * a.CB + cv * 8;  // this thread's 8 channels
    const size_t so = (size_t)n * a.HW * a.C;
    uint4 xv[RPT], rv[RES ? RPT : 1];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int row = r + k * RL;
        const size_t o = so + (size_t)min(row, a.HW - 1) * a.C + c0;
        xv[k] = *reinterpret_cast<const uint4*>(a.x + o);
        if constexpr (RES) rv[k] = *reinterpret_cast<const uint4*>(a.res + o);
    }
    const Vec<8> b = a.bias ? ld_param<8>(a.bias, a.bias_bf16, c0) : zero<8>();
    float acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (r + k * RL >= a.HW) break;
        const uint32_t w4[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = __uint_as_float(w4[i] << 16);
            v[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
        }
        if constexpr (RES) {
            const uint32_t q4[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                v[2 * i] += __uint_as_float(q4[i] << 16);
                v[2 * i + 1] += __uint_as_float(q4[i] & 0xffff0000u);
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float u = v[i] + b.v[i];
            acc[i] += u;
            acc[8 + i] += u * u;
        }
    }
    wg_chan_totals<2>(acc, red, tot, a.CV, a.CB);
    if (t < a.gpw) {  // group statistics (fp64, channel order)
        const int g = blk * a.gpw + t;
        double s1 = 0.0, s2 = 0.0;
        for (int u = 0; u < a.cpg; ++u) {
            s1 += tot[t * a.cpg + u];
            s2 += tot[a.CB + t * a.cpg + u];
        }
        const double inv_cnt = 1.0 / ((double)a.HW * a.cpg);
        const double mean = s1 * inv_cnt;
        const double var = fmax(s2 * inv_cnt - mean * mean, 0.0);
        const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
        gsc[t] = (float)mean;
        gsh[t] = invstd;
        a.save_mean[n * a.NG + g] = (float)mean;
        a.save_invstd[n * a.NG + g] = invstd;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        opaque4(xv[k]);
        if constexpr (RES) opaque4(rv[k]);
    }
    float sc[8], sh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int gl = (cv * 8 + i) / a.cpg;  // group within the block
        sc[i] = a.gamma[c0 + i] * gsh[gl];
        sh[i] = a.beta[c0 + i] - gsc[gl] * sc[i];
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int row = r + k * RL;
        if (row >= a.HW) break;
        const uint32_t w4[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
        Vec<8> v;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v.v[2 * i] = __uint_as_float(w4[i] << 16);
            v.v[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
        }
        if constexpr (RES) {
            const uint32_t q4[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                v.v[2 * i] += __uint_as_float(q4[i] << 16);
                v.v[2 * i + 1] += __uint_as_float(q4[i] & 0xffff0000u);
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) v.v[i] = gn_act_f((v.v[i] + b.v[i]) * sc[i] + sh[i], a.act);
        st_bf<8>(a.out + so + (size_t)row * a.C + c0, v);
    }
}

template <int RPT, bool RES>
__global__ __launch_bounds__(RNT) void k_gnr_bwd(GNRArgs a) {
    __shared__ float red[(RNT / 64) * 4 * 24];
    __shared__ double tot[3 * 32];
    __shared__ float gk2[32], gk3[32];
    const int t = threadIdx.x, cv = t % a.CV, r = t / a.CV, RL = blockDim.x / a.CV;
    const int n = blockIdx.x / a.nblk, blk = blockIdx.x - n * a.nblk;
    const int c0 = blk * a.CB + cv * 8;
    const size_t so = (size_t)n * a.HW * a.C;
    uint4 gv[RPT], xv[RPT], rv[RES ? RPT : 1];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int row = r + k * RL;
        const size_t o = so + (size_t)min(row, a.HW - 1) * a.C + c0;
        gv[k] = *reinterpret_cast<const uint4*>(a.dy + o);
        xv[k] = *reinterpret_cast<const uint4*>(a.x + o);
        if constexpr (RES) rv[k] = *reinterpret_cast<const uint4*>(a.res + o);
    }
    const Vec<8> b = a.bias ? ld_param<8>(a.bias, a.bias_bf16, c0) : zero<8>();
    float mu[8], is[8], ga[8], be[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int g = (c0 + i) / a.cpg;
        mu[i] = a.save_mean[n * a.NG + g];
        is[i] = a.save_invstd[n * a.NG + g];
        ga[i] = a.gamma[c0 + i];
        be[i] = a.beta[c0 + i];
    }
    // xhat and the activation-masked gradient of one row vector
    auto row_vals = [&](int k, float (&xh)[8], float (&gg)[8]) {
        const uint32_t w4[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
        const uint32_t d4[4] = {gv[k].x, gv[k].y, gv[k].z, gv[k].w};
        float v[8], d[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = __uint_as_float(w4[i] << 16);
            v[2 * i + 1] = __uint_as_float(w4[i] & 0xffff0000u);
            d[2 * i] = __uint_as_float(d4[i] << 16);
            d[2 * i + 1] = __uint_as_float(d4[i] & 0xffff0000u);
        }
        if constexpr (RES) {
            const uint32_t q4[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                v[2 * i] += __uint_as_float(q4[i] << 16);
                v[2 * i + 1] += __uint_as_float(q4[i] & 0xffff0000u);
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            xh[i] = (v[i] + b.v[i] - mu[i]) * is[i];
            gg[i] = gn_act_g(d[i], xh[i] * ga[i] + be[i], a.act);
        }
    };
    float acc[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) acc[i] = 0.0f;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (r + k * RL >= a.HW) break;
        float xh[8], gg[8];
        row_vals(k, xh, gg);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            acc[i] += gg[i];
            acc[8 + i] += gg[i] * xh[i];
            acc[16 + i] += xh[i];
        }
    }
    wg_chan_totals<3>(acc, red, tot, a.CV, a.CB);   // tot = [S1 | S2 | X][CB]
    const double cnt = (double)a.HW * a.cpg;
    if (t < a.gpw) {
        const int g = blk * a.gpw + t;
        double A = 0.0, Bq = 0.0;
        for (int u = 0; u < a.cpg; ++u) {
            const int c = t * a.cpg + u;
            const double gc = a.gamma[blk * a.CB + c];
            A += gc * tot[c];
            Bq += gc * tot[a.CB + c];
        }
        const double isg = a.save_invstd[n * a.NG + g];
        gk2[t] = (float)(A / cnt * isg);
        gk3[t] = (float)(Bq / cnt * isg);
    }
    __syncthreads();
    // per-(sample, channel) partial rows of the parameter gradients (the closed-form conv-bias term
    // with the same fp32 k2 / k3 the dx below uses)
    for (int c = t; c < a.CB; c += blockDim.x) {
        const int cg = blk * a.CB + c, gl = c / a.cpg;
        const double isg = a.save_invstd[n * a.NG + cg / a.cpg], gc = a.gamma[cg];
        float* pr = a.part + (size_t)n * 3 * a.C;
        pr[cg] = (float)tot[c];
        pr[a.C + cg] = (float)tot[a.CB + c];
        pr[2 * a.C + cg] = (float)(gc * isg * tot[c] - (double)a.HW * (double)gk2[gl] -
                                   (double)gk3[gl] * tot[2 * a.CB + c]);
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        opaque4(xv[k]);
        opaque4(gv[k]);
        if constexpr (RES) opaque4(rv[k]);
    }
    float k1[8], k2[8], k3[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int gl = (cv * 8 + i) / a.cpg;
        k1[i] = ga[i] * is[i];
        k2[i] = gk2[gl];
        k3[i] = gk3[gl];
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int row = r + k * RL;
        if (row >= a.HW) break;
        float xh[8], gg[8];
        row_vals(k, xh, gg);
        Vec<8> d;
#pragma unroll
        for (int i = 0; i < 8; ++i) d.v[i] = k1[i] * gg[i] - k2[i] - xh[i] * k3[i];
        st_bf<8>(a.out + so + (size_t)row * a.C + c0, d);
        if (a.out2) st_bf<8>(a.out2 + so + (size_t)row * a.C + c0, d);
    }
}

// parameter gradients from the per-sample rows: thread = channel, samples in order (fp64)
__global__ __launch_bounds__(256) void k_gnr_params(GNRArgs a) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= a.C) return;
    double s1 = 0.0, s2 = 0.0, sb = 0.0;
    for (int n = 0; n < a.N; ++n) {
        const float* pr = a.part + (size_t)n * 3 * a.C;
        s1 += (double)pr[c];
        s2 += (double)pr[a.C + c];
        sb += (double)pr[2 * a.C + c];
    }
    a.dbeta[c] = (float)s1;
    a.dgamma[c] = (float)s2;
    if (a.dbias) {
        if (a.bias_bf16)
            static_cast<uint16_t*>(a.dbias)[c] = f2bf((float)sb);
        else
            static_cast<float*>(a.dbias)[c] = (float)sb;
    }
}

// resident-path geometry: CB channels per workgroup (whole groups, a multiple of 8 with CV = CB / 8
// in {1, 2, 4}), nthr threads, RPT row vectors per thread (a template value) — false when the layer
// does not fit (cap = row vectors per thread the register budget allows)
struct GNRGeo {
    int CB, CV, gpw, nthr, rpt;
};
inline bool gnr_geometry(int HW, int C, int G, int cap, GNRGeo& g) {
    if (C % G) return false;
    const int cpg = C / G;
    if (cpg >= 8) {
        // CV = cpg / 8 row vectors of a pixel must be a power of two (1, 2, 4): the row-per-thread
        // mapping (RL = 256 / CV) and the XOR butterflies of wave_colsum group lanes by lane & (CV - 1)
        if (cpg != 8 && cpg != 16 && cpg != 32) return false;
        g.CB = cpg, g.gpw = 1;
    } else {
        if (8 % cpg || G % (8 / cpg)) return false;
        g.CB = 8, g.gpw = 8 / cpg;
    }
    if (C % g.CB || g.gpw > 32) return false;
    g.CV = g.CB / 8;
    // 256-thread workgroups only: in the PackNet step the 512 / 1024-thread forms were slower than
    // the two-pass kernels (a whole-CU workgroup waits for a CU to drain beside the concurrent pose
    // branch, and RPT row vectors per thread are one long latency chain; profiles/r04/gn)
    static const int tmpl[] = {1, 2, 4, 8};
    const int nthr = 256, RL = nthr / g.CV;
    const int need = (HW + RL - 1) / RL;
    for (int r : tmpl) {
        if (r > cap) break;
        if (r >= need) {
            g.nthr = nthr, g.rpt = r;
            return true;
        }
    }
    return false;
}
// row vectors per thread: the GN_RES_RPT knob, 4 by default (the resident path only pays for
// small layers, see gnr_geometry; RPT 8 — PackNetSAN01's 24x80 layers — lost the step A/B,
// psfm_knobs.hip); backward with res at most 2 (RPT 4 + res spills: compiler resource report,
// -Rpass-analysis=kernel-resource-usage)
inline int gnr_cap_fwd(bool res) { (void)res; return knob(KNOB_GN_RES_RPT); }
inline int gnr_cap_bwd(bool res) { return res ? std::min(2, knob(KNOB_GN_RES_RPT)) : knob(KNOB_GN_RES_RPT); }

// RPT instantiations: forward 1, 2, 4, 8, backward 1, 2, 4, 8 (res <= 2), see gnr_cap_*
#define GNR_CASE(KERNEL, R, RES_, grid, nthr, st, a)                                   \
    case R:                                                                          \
        if (RES_) hipLaunchKernelGGL((KERNEL<R, true>), grid, dim3(nthr), 0, st, a);   \
        else hipLaunchKernelGGL((KERNEL<R, false>), grid, dim3(nthr), 0, st, a);       \
        break
#define GNR_LAUNCH_FWD(RPT_, RES_, grid, nthr, st, a)                                  \
    do {                                                                             \
        switch (RPT_) {                                                              \
            GNR_CASE(k_gnr_fwd, 1, RES_, grid, nthr, st, a);                         \
            GNR_CASE(k_gnr_fwd, 2, RES_, grid, nthr, st, a);                         \
            GNR_CASE(k_gnr_fwd, 4, RES_, grid, nthr, st, a);                         \
            GNR_CASE(k_gnr_fwd, 8, RES_, grid, nthr, st, a);                         \
        }                                                                            \
    } while (0)
#define GNR_LAUNCH_BWD(RPT_, RES_, grid, nthr, st, a)                                  \
    do {                                                                             \
        switch (RPT_) {                                                              \
            GNR_CASE(k_gnr_bwd, 1, RES_, grid, nthr, st, a);                         \
            GNR_CASE(k_gnr_bwd, 2, RES_, grid, nthr, st, a);                         \
            case 4: hipLaunchKernelGGL((k_gnr_bwd<4, false>), grid, dim3(nthr), 0, st, a); break; \
            default: hipLaunchKernelGGL((k_gnr_bwd<8, false>), grid, dim3(nthr), 0, st, a); break; \
        }                                                                            \
    } while (0)

// ------------------------------------------------------------------------------------------
// BasicBlock tail (resnet_encoder.py:61-98 -> torchvision BasicBlock: out = relu(bn2(conv2(.)) +
// identity)) after MIOpen's BatchNorm: y = relu(a + b) in ONE pass (bf16 in, fp32 add, one rounding —
// what autocast's bf16 add followed by relu produces: the add rounds to bf16 and relu keeps it), and
// its backward dz = dy * (y > 0), written once and handed to both inputs.  16-byte vectors, one per
// thread, a grid over the tensor (no row loops: these run at the launch floor).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_add_relu_fwd(const uint4* __restrict__ a, const uint4* __restrict__ b,
                                                       uint4* __restrict__ y, long long n8) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n8) return;
    const Vec<8> va = ld_bf<8>(reinterpret_cast<const uint16_t*>(a + i));
    const Vec<8> vb = b ? ld_bf<8>(reinterpret_cast<const uint16_t*>(b + i)) : zero<8>();   // b null: relu(a)
    Vec<8> o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {   // ATen relu: NaN propagates (fmaxf would drop it)
        const float sum = bfround(va.v[k] + vb.v[k]);
        o.v[k] = sum <= 0.0f ? 0.0f : sum;
    }
    st_bf<8>(reinterpret_cast<uint16_t*>(y + i), o);
}
// dz = (y <= 0) ? 0 : dy [+ dy1 [+ dy2]] (each sum rounded to bf16, as autograd accumulates the
// gradients of a tensor with several consumers; dy1 / dy2 may be null)
__global__ __launch_bounds__(256) void k_relu_mask_bwd(const uint4* __restrict__ dy, const uint4* __restrict__ dy1,
                                                        const uint4* __restrict__ dy2, const uint4* __restrict__ y,
                                                        uint4* __restrict__ dz, long long n8) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n8) return;
    uint4 g = dy[i];
    if (dy1) g = add_bf16x8(g, dy1[i]);
    if (dy2) g = add_bf16x8(g, dy2[i]);
    dz[i] = relu_mask4(g, y[i]);
}

// ------------------------------------------------------------------------------------------
// Two-pass GroupNorm, software-pipelined (VEC = 8): the large layers (PackNet 192x640 / 96x320) run
// from HBM in the step, where one row step's loads then its arithmetic left each thread waiting a
// full memory latency per step (2.1-2.8 TB/s in the step, profiles/r04/gn).  Here every thread keeps
// the NEXT row step's loads in flight while it works on the current one (two register buffers,
// raw 16-byte words: no conversion may sit between a load and the next step's compute).  The loads
// are unconditional (rows clamped into the range, masked at use) and the trip count is uniform, so
// no branch around a load makes the wait counts conservative.  Same arithmetic and order as
// k_gn_*<8> (bitwise equal results).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ Vec<8> unpack8(const uint4 q) {
    Vec<8> r;
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        r.v[2 * i] = __uint_as_float(w[i] << 16);
        r.v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
    return r;
}
__device__ __forceinline__ uint4 ldq(const uint16_t* p) { return *reinterpret_cast<const uint4*>(p); }

// x (+ res) of row step `it` of this thread: rows row0 + r + it*U*TR + u*TR, clamped to row1 - 1
template <bool RES>
struct RowsX {
    uint4 x[U], q[RES ? U : 1];
    __device__ __forceinline__ void load(const GNArgs& a, size_t so, int c0, int first, int TR, int row1) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t o = so + (size_t)min(first + u * TR, row1 - 1) * a.C + c0;
            x[u] = ldq(a.x + o);
            if constexpr (RES) q[u] = ldq(a.res + o);
        }
    }
    __device__ __forceinline__ Vec<8> val(int u) const {
        Vec<8> v = unpack8(x[u]);
        if constexpr (RES) {
            const Vec<8> w = unpack8(q[u]);
#pragma unroll
            for (int i = 0; i < 8; ++i) v.v[i] += w.v[i];
        }
        return v;
    }
};
template <bool RES>
struct RowsGX : RowsX<RES> {
    uint4 g[U];
    __device__ __forceinline__ void load(const GNArgs& a, size_t so, int c0, int first, int TR, int row1) {
        RowsX<RES>::load(a, so, c0, first, TR, row1);
#pragma unroll
        for (int u = 0; u < U; ++u) g[u] = ldq(a.dy + so + (size_t)min(first + u * TR, row1 - 1) * a.C + c0);
    }
};

// drive body(rows, first_row) over the row steps with the next step's loads in flight
#define GNP_PIPELINE(ROWS_T, ROW0, ROW1, R, TR, SO, C0, BODY)                      \
    do {                                                                       \
        const int step_ = U * (TR);                                            \
        const int niter_ = ((ROW1) - (ROW0) + step_ - 1) / step_;              \
        ROWS_T A_, B_;                                                         \
        if (niter_ > 0) A_.load(a, SO, C0, (ROW0) + (R), TR, ROW1);            \
        for (int it_ = 0; it_ < niter_; it_ += 2) {                            \
            B_.load(a, SO, C0, (ROW0) + (R) + (it_ + 1) * step_, TR, ROW1);    \
            BODY(A_, (ROW0) + (R) + it_ * step_);                              \
            if (it_ + 1 >= niter_) break;                                      \
            A_.load(a, SO, C0, (ROW0) + (R) + (it_ + 2) * step_, TR, ROW1);    \
            BODY(B_, (ROW0) + (R) + (it_ + 1) * step_);                        \
        }                                                                      \
    } while (0)

template <bool RES>
__global__ __launch_bounds__(NT) void k_gnp_fwd_stats(GNArgs a) {
    __shared__ float red[2 * NT * 8];
    __shared__ float chan[2 * MAX_C];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * 8;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    float acc[2][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[0][i] = acc[1][i] = 0.0f;
    if (r < a.TR) {
        const Vec<8> b = a.bias ? ld_param<8>(a.bias, a.bias_bf16, c0) : zero<8>();
        const size_t so = (size_t)n * a.HW * a.C;
        const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
#define GNP_FWD_STATS_BODY(RW, FIRST)                                          \
        _Pragma("unroll") for (int u = 0; u < U; ++u) {                        \
            const bool in = (FIRST) + u * a.TR < row1;                         \
            const Vec<8> v = RW.val(u);                                        \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) {                    \
                const float w = in ? v.v[i] + b.v[i] : 0.0f;                   \
                acc[0][i] += w;                                                \
                acc[1][i] += w * w;                                            \
            }                                                                  \
        }
        GNP_PIPELINE(RowsX<RES>, row0, row1, r, a.TR, so, c0, GNP_FWD_STATS_BODY);
#undef GNP_FWD_STATS_BODY
    }
    block_colsum<8, 2>(acc, red, a.G, a.TR);
    chan_to_lds<8, 2>(acc, chan, a.C, c0, r);
    const int cpg = a.C / a.NG;
    float* row = a.ws + (size_t)blockIdx.x * a.RW;
    for (int j = t; j < 2 * a.NG; j += NT) {
        const int k = j / a.NG, g = j - k * a.NG;
        float s = 0.0f;
        for (int u = 0; u < cpg; ++u) s += chan[k * a.C + g * cpg + u];
        row[j] = s;
    }
}

template <bool RES>
__global__ __launch_bounds__(NT) void k_gnp_fwd_apply(GNArgs a) {
    __shared__ double tot[2 * MAX_NG];
    __shared__ double scr[NT];
    __shared__ float gmean[MAX_NG], ginv[MAX_NG];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * 8;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const size_t so = (size_t)n * a.HW * a.C;
    const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
    const bool live = r < a.TR;
    const int step = U * a.TR, niter = (row1 - row0 + step - 1) / step;
    RowsX<RES> A, B;
    // the first two row steps go out before the prologue (their latency overlaps the reduction)
    if (live && niter > 0) A.load(a, so, c0, row0 + r, a.TR, row1);
    if (live && niter > 0) B.load(a, so, c0, row0 + r + step, a.TR, row1);
    group_totals(a.ws + (size_t)n * a.bpn * a.RW, a.bpn, a.RW, 2 * a.NG, tot, scr);
    const int cpg = a.C / a.NG;
    if (t < a.NG) {
        const double inv_cnt = 1.0 / ((double)a.HW * cpg);
        const double mean = tot[t] * inv_cnt;
        const double var = fmax(tot[a.NG + t] * inv_cnt - mean * mean, 0.0);
        const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
        gmean[t] = (float)mean;
        ginv[t] = invstd;
        if (bl == 0) {
            a.save_mean[n * a.NG + t] = (float)mean;
            a.save_invstd[n * a.NG + t] = invstd;
        }
    }
    __syncthreads();
    if (!live) return;
    Vec<8> sc, sh;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int g = (c0 + i) / cpg;
        sc.v[i] = a.gamma[c0 + i] * ginv[g];
        sh.v[i] = a.beta[c0 + i] - gmean[g] * sc.v[i];
    }
    const Vec<8> b = a.bias ? ld_param<8>(a.bias, a.bias_bf16, c0) : zero<8>();
    auto body = [&](const RowsX<RES>& RW, int first) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = first + u * a.TR;
            Vec<8> v = RW.val(u);
#pragma unroll
            for (int i = 0; i < 8; ++i) v.v[i] = gn_act_f((v.v[i] + b.v[i]) * sc.v[i] + sh.v[i], a.act);
            if (row < row1) st_bf<8>(a.out + so + (size_t)row * a.C + c0, v);
        }
    };
    for (int it = 0; it < niter; it += 2) {
        body(A, row0 + r + it * step);
        if (it + 1 >= niter) break;
        A.load(a, so, c0, row0 + r + (it + 2) * step, a.TR, row1);
        body(B, row0 + r + (it + 1) * step);
        B.load(a, so, c0, row0 + r + (it + 3) * step, a.TR, row1);
    }
}

template <bool RES>
__global__ __launch_bounds__(NT) void k_gnp_bwd_stats(GNArgs a) {
    __shared__ float red[3 * NT * 8];
    __shared__ float chan[3 * MAX_C];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * 8;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const int cpg = a.C / a.NG;
    float acc[3][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[0][i] = acc[1][i] = acc[2][i] = 0.0f;
    if (r < a.TR) {
        const Vec<8> b = a.bias ? ld_param<8>(a.bias, a.bias_bf16, c0) : zero<8>();
        float mu[8], is[8], ga[8], be[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            mu[i] = a.save_mean[n * a.NG + (c0 + i) / cpg];
            is[i] = a.save_invstd[n * a.NG + (c0 + i) / cpg];
            ga[i] = a.gamma[c0 + i];
            be[i] = a.beta[c0 + i];
        }
        const size_t so = (size_t)n * a.HW * a.C;
        const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
#define GNP_BWD_STATS_BODY(RW, FIRST)                                          \
        _Pragma("unroll") for (int u = 0; u < U; ++u) {                        \
            const bool in_u = (FIRST) + u * a.TR < row1;                       \
            const Vec<8> x = RW.val(u), g = unpack8(RW.g[u]);                  \
            _Pragma("unroll") for (int i = 0; i < 8; ++i) {                    \
                const float gv = in_u ? g.v[i] : 0.0f, xv = in_u ? x.v[i] : 0.0f; \
                const float xh = (xv + b.v[i] - mu[i]) * is[i];                \
                const float gg = gn_act_g(gv, xh * ga[i] + be[i], a.act);      \
                acc[0][i] += gg;                                               \
                acc[1][i] += gg * xh;                                          \
                acc[2][i] += in_u ? xh : 0.0f;                                 \
            }                                                                  \
        }
        GNP_PIPELINE(RowsGX<RES>, row0, row1, r, a.TR, so, c0, GNP_BWD_STATS_BODY);
#undef GNP_BWD_STATS_BODY
    }
    block_colsum<8, 3>(acc, red, a.G, a.TR);
    chan_to_lds<8, 3>(acc, chan, a.C, c0, r);
    float* row = a.ws + (size_t)blockIdx.x * a.RW;
    for (int j = t; j < 2 * a.NG; j += NT) {
        const int k = j / a.NG, g = j - k * a.NG;
        float s = 0.0f;
        for (int u = 0; u < cpg; ++u) s += a.gamma[g * cpg + u] * chan[k * a.C + g * cpg + u];
        row[j] = s;
    }
    for (int j = t; j < 3 * a.C; j += NT) row[2 * a.NG + j] = chan[j];
}

template <bool RES>
__global__ __launch_bounds__(NT) void k_gnp_bwd_apply(GNArgs a) {
    if ((int)blockIdx.x >= a.N * a.bpn) {
        gn_bwd_params(a, blockIdx.x - a.N * a.bpn);
        return;
    }
    __shared__ double tot[2 * MAX_NG];
    __shared__ double scr[NT];
    __shared__ float gk2[MAX_NG], gk3[MAX_NG];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * 8;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const int cpg = a.C / a.NG;
    const size_t so = (size_t)n * a.HW * a.C;
    const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
    const bool live = r < a.TR;
    const int step = U * a.TR, niter = (row1 - row0 + step - 1) / step;
    RowsGX<RES> A, B;
    if (live && niter > 0) A.load(a, so, c0, row0 + r, a.TR, row1);
    if (live && niter > 0) B.load(a, so, c0, row0 + r + step, a.TR, row1);
    group_totals(a.ws + (size_t)n * a.bpn * a.RW, a.bpn, a.RW, 2 * a.NG, tot, scr);
    if (t < a.NG) {
        const double cnt = (double)a.HW * cpg;
        const double is = a.save_invstd[n * a.NG + t];
        gk2[t] = (float)(tot[t] / cnt * is);
        gk3[t] = (float)(tot[a.NG + t] / cnt * is);
    }
    __syncthreads();
    if (!live) return;
    const Vec<8> b = a.bias ? ld_param<8>(a.bias, a.bias_bf16, c0) : zero<8>();
    float mu[8], is[8], ga[8], be[8], k1[8], k2[8], k3[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int gi = (c0 + i) / cpg;
        mu[i] = a.save_mean[n * a.NG + gi];
        is[i] = a.save_invstd[n * a.NG + gi];
        ga[i] = a.gamma[c0 + i];
        be[i] = a.beta[c0 + i];
        k1[i] = ga[i] * is[i];
        k2[i] = gk2[gi];
        k3[i] = gk3[gi];
    }
    auto body = [&](const RowsGX<RES>& RW, int first) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int row = first + u * a.TR;
            const Vec<8> x = RW.val(u), g = unpack8(RW.g[u]);
            Vec<8> d;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float xh = (x.v[i] + b.v[i] - mu[i]) * is[i];
                const float gg = gn_act_g(g.v[i], xh * ga[i] + be[i], a.act);
                d.v[i] = k1[i] * gg - k2[i] - xh * k3[i];
            }
            if (row < row1) {
                st_bf<8>(a.out + so + (size_t)row * a.C + c0, d);
                if (a.out2) st_bf<8>(a.out2 + so + (size_t)row * a.C + c0, d);
            }
        }
    };
    for (int it = 0; it < niter; it += 2) {
        body(A, row0 + r + it * step);
        if (it + 1 >= niter) break;
        A.load(a, so, c0, row0 + r + (it + 2) * step, a.TR, row1);
        body(B, row0 + r + (it + 1) * step);
        B.load(a, so, c0, row0 + r + (it + 3) * step, a.TR, row1);
    }
}

// the software-pipelined two-pass GroupNorm (k_gnp_*) is the product's form for VEC = 8; the
// unpipelined k_gn_*<VEC> kernels run only VEC = 1 (the unpipelined VEC = 8 form, bitwise the same
// results, lost 208 vs 211 img/s on PackNet01, profiles/r04/gn, and was removed in round 6)

template <typename A>
void set_geo(A& a, const Geo& g) {
    a.G = g.G;
    a.TR = g.TR;
    a.rpb = g.rpb;
}

// host mirror of the GN workspace: stats rows [N*bpn][RW] (RW = 2NG + 3C covers both passes)
inline int gn_rw_bwd(int C, int G) { return 2 * G + 3 * C; }
size_t gn_ws(int N, int bpn, int C, int G) { return align4((size_t)N * bpn * gn_rw_bwd(C, G)); }

inline int check_vec(int C, const char* what) {
    if (pick_vec(C) == 1 && C > NT) return fail(-2, (std::string(what) + ": C must be a multiple of 8 or <= 256").c_str());
    if (2 * C > MAX_KC) return fail(-2, (std::string(what) + ": C must be <= 512").c_str());
    return 0;
}

// GN geometry: the grid stays <= TARGET_BLOCKS workgroups over the N samples
inline Geo gn_geometry(int N, int HW, int C) {
    return geometry(HW, C, pick_vec(C), std::max(1, TARGET_BLOCKS / N));
}

// ---------------------------------------------------------------------------------------------
// Decoder up-stage input: out = cat([nearest_up2(x), skip], channels), NHWC bf16, 16-byte
// vectors (depth_decoder.py:48-57).  One launch each way instead of the upsample, cat and the
// backward's strided copy + two-pass block-sum reduction.
// ---------------------------------------------------------------------------------------------
struct UpcatArgs {
    const uint4* x;     // [N, h, w, C1/8]
    const uint4* skip;  // [N, 2h, 2w, C2/8] or null
    uint4* out;         // [N, 2h, 2w, (C1+C2)/8]
    const uint4* dout;
    uint4* dx;
    uint4* dskip;
    const void* bias;   // RELU variant: conv bias [C1] (bf16 / fp32)
    float* rows;        // RELU backward: per-workgroup partial rows of the bias gradient [nbx][C1]
    int N, h, w, V1, V2;  // V = channels / 8
    int bias_bf16;
    uint32_t nfwd, ndx, ndskip, nbx;  // nbx: workgroups of the dx part (the dskip part follows)
};

__device__ __forceinline__ uint4 pack8(const float (&v)[8]) {
    uint4 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
    o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
    return o;
}
__device__ __forceinline__ void unpack8(uint4 q, float (&v)[8]) {
    const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[2 * k] = __uint_as_float(u[k] << 16);
        v[2 * k + 1] = __uint_as_float(u[k] & 0xffff0000u);
    }
}

// RELU = true: the x part is relu(x + bias) of the up-stage's first ConvBlock (layers.py:25-41:
// Conv3x3 + ReLU), computed on the fly — the block's output is never written on its own.
template <bool RELU>
__global__ __launch_bounds__(256) void k_upcat_fwd(UpcatArgs a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= a.nfwd) return;
    const uint32_t Vt = (uint32_t)(a.V1 + a.V2);
    const uint32_t pix = i / Vt, v = i - pix * Vt;   // output pixel (n, Y, X), vector in the row
    const uint32_t W2 = 2u * (uint32_t)a.w, H2 = 2u * (uint32_t)a.h;
    const uint32_t X = pix % W2, nY = pix / W2, Y = nY % H2, n = nY / H2;
    if (v < (uint32_t)a.V1) {
        const uint4 q = a.x[(((size_t)n * a.h + (Y >> 1)) * a.w + (X >> 1)) * a.V1 + v];
        if constexpr (RELU) {
            float f[8];
            unpack8(q, f);
            const Vec<8> b = ld_param<8>(a.bias, a.bias_bf16, (int)v * 8);
#pragma unroll
            for (int k = 0; k < 8; ++k) f[k] = fmaxf(f[k] + b.v[k], 0.0f);
            a.out[i] = pack8(f);
        } else {
            a.out[i] = q;
        }
    } else {
        a.out[i] = a.skip[(size_t)pix * a.V2 + (v - a.V1)];
    }
}

__device__ __forceinline__ void add8(float (&acc)[8], uint4 q) {
    const uint32_t u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        acc[2 * k] += __uint_as_float(u[k] << 16);
        acc[2 * k + 1] += __uint_as_float(u[k] & 0xffff0000u);
    }
}

// workgroups [0, nbx): one 8-channel vector of dx per thread (sum of its 2x2 block, rows then
// columns, fp32, one bf16 rounding; RELU: masked where the block's output relu(x + bias) — read
// back from the forward output — is 0, and the workgroup's column sums of the stored dx written as
// its partial bias-gradient row); workgroups [nbx, ..): one vector of dskip per thread (copy)
template <bool RELU>
__global__ __launch_bounds__(256) void k_upcat_bwd(UpcatArgs a) {
    const uint32_t Vt = (uint32_t)(a.V1 + a.V2);
    if (blockIdx.x < a.nbx) {
        const uint32_t i = blockIdx.x * 256u + threadIdx.x;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (i < a.ndx) {
            const uint32_t pix = i / (uint32_t)a.V1, v = i - pix * (uint32_t)a.V1;  // input pixel (n, y, x)
            const uint32_t x = pix % (uint32_t)a.w, ny = pix / (uint32_t)a.w;
            const uint32_t y = ny % (uint32_t)a.h, n = ny / (uint32_t)a.h;
            const uint32_t W2 = 2u * (uint32_t)a.w;
            const size_t r0 = ((size_t)n * 2u * a.h + 2u * y) * W2 + 2u * x;  // top-left output pixel
            add8(acc, a.dout[r0 * Vt + v]);
            add8(acc, a.dout[(r0 + 1) * Vt + v]);
            add8(acc, a.dout[(r0 + W2) * Vt + v]);
            add8(acc, a.dout[(r0 + W2 + 1) * Vt + v]);
            if constexpr (RELU) {
                float y0[8];
                unpack8(a.out[r0 * Vt + v], y0);
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[k] = y0[k] > 0.0f ? bfround(acc[k]) : 0.0f;
            }
            a.dx[i] = pack8(acc);
        }
        if constexpr (RELU) {   // partial row: pixels of this workgroup summed per channel (fixed tree)
            __shared__ float red[256][8];
            const int t = threadIdx.x, V1 = a.V1;
#pragma unroll
            for (int k = 0; k < 8; ++k) red[t][k] = acc[k];
            __syncthreads();
            for (int st = (256 / V1) / 2; st >= 1; st >>= 1) {
                if (t / V1 < st)
#pragma unroll
                    for (int k = 0; k < 8; ++k) red[t][k] += red[t + st * V1][k];
                __syncthreads();
            }
            if (t < V1)
#pragma unroll
                for (int k = 0; k < 8; ++k) a.rows[(size_t)blockIdx.x * V1 * 8 + t * 8 + k] = red[t][k];
        }
        return;
    }
    const uint32_t j = (blockIdx.x - a.nbx) * 256u + threadIdx.x;
    if (j >= a.ndskip) return;
    const uint32_t pix = j / (uint32_t)a.V2, v = j - pix * (uint32_t)a.V2;
    a.dskip[j] = a.dout[(size_t)pix * Vt + a.V1 + v];
}

// ------------------------------------------------------------------------------------------
// The ResNet stem's ReLU + MaxPool2d(3, stride 2, pad 1) (torchvision ResNet via resnet_encoder.py:
// relu(bn1(conv1(x))) feeds maxpool and the decoder's first skip): ONE pass each way on bf16
// channels_last, H and W even.  A thread owns one output pixel's 8-channel vector and the 2 x 2
// input block it tiles (stride 2): it loads the 3 x 3 window once, writes the ReLU output of its own
// block (the decoder skip), the pooled value and the window position of the maximum (uint8 per
// channel: kh * 3 + kw).  ATen semantics: max with NaN propagation (`v > m || isnan(v)`, first
// maximum kept on ties).  Backward: per input pixel, the pooled gradients of the <= 4 windows whose
// maximum it is, in (oh, ow) order in fp32, one bf16 rounding (max_pool_backward_nhwc), plus the
// skip gradient (autograd's bf16 add), then the ReLU mask of the output — and the pooled output's
// two consumers' gradients summed first (fused._fork): one kernel for max-pool backward, two adds and
// the ReLU backward.
// ------------------------------------------------------------------------------------------
struct PoolArgs {
    const uint16_t* x;     // fwd: the BatchNorm output [N, H, W, C]
    uint16_t* relu;        // [N, H, W, C] relu(x)
    uint16_t* pool;        // [N, H/2, W/2, C]
    uint8_t* arg;          // [N, H/2, W/2, C] window position of the maximum
    const uint16_t* dpool;   // bwd
    const uint16_t* dpool1;  // may be null
    const uint16_t* dskip;   // may be null
    uint16_t* dx;
    int N, H, W, C, Ho, Wo, CV;   // CV = C / 8
    long long n;                  // N * Ho * Wo * CV threads
};

__global__ __launch_bounds__(256) void k_relu_maxpool_fwd(PoolArgs a) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int cv = (int)(i % a.CV);
    const long long opix = i / a.CV;
    const int ow = (int)(opix % a.Wo), oh = (int)((opix / a.Wo) % a.Ho), nb = (int)(opix / ((long long)a.Wo * a.Ho));
    const int c0 = cv * 8;
    float m[8];
    uint32_t idx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = -INFINITY, idx[k] = 0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
        const int ih = 2 * oh - 1 + kh;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int iw = 2 * ow - 1 + kw;
            if (ih < 0 || ih >= a.H || iw < 0 || iw >= a.W) continue;
            const size_t o = (((size_t)nb * a.H + ih) * a.W + iw) * a.C + c0;
            const uint4 q = *reinterpret_cast<const uint4*>(a.x + o);
            float v[8];
            unpack8f(q, v);
            Vec<8> rv;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float r = v[k] <= 0.0f ? 0.0f : v[k];   // ATen relu (NaN propagates)
                rv.v[k] = r;
                if (r > m[k] || r != r) {   // max_pool_forward_nhwc's test (r >= 0 > -inf: the first sets it)
                    m[k] = r;
                    idx[k] = kh * 3 + kw;
                }
            }
            if (kh >= 1 && kw >= 1) st_bf<8>(a.relu + o, rv);   // this thread's own 2 x 2 block
        }
    }
    Vec<8> pv;
#pragma unroll
    for (int k = 0; k < 8; ++k) pv.v[k] = m[k];
    const size_t po = (size_t)opix * a.C + c0;
    st_bf<8>(a.pool + po, pv);
    uint2 packed;
    packed.x = idx[0] | (idx[1] << 8) | (idx[2] << 16) | (idx[3] << 24);
    packed.y = idx[4] | (idx[5] << 8) | (idx[6] << 16) | (idx[7] << 24);
    *reinterpret_cast<uint2*>(a.arg + po) = packed;
}

__global__ __launch_bounds__(256) void k_relu_maxpool_bwd(PoolArgs a) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const int cv = (int)(i % a.CV);
    const long long opix = i / a.CV;
    const int ow = (int)(opix % a.Wo), oh = (int)((opix / a.Wo) % a.Ho), nb = (int)(opix / ((long long)a.Wo * a.Ho));
    const int c0 = cv * 8;
    // the (up to) 4 windows touching this thread's 2 x 2 block: (oh + wy, ow + wx), wy, wx in {0, 1}
    float g[2][2][8];
    uint32_t ar[2][2][2];
    bool ok[2][2];
#pragma unroll
    for (int wy = 0; wy < 2; ++wy)
#pragma unroll
        for (int wx = 0; wx < 2; ++wx) {
            const int ph = oh + wy, pw = ow + wx;
            ok[wy][wx] = ph < a.Ho && pw < a.Wo;
            const size_t po = (((size_t)nb * a.Ho + min(ph, a.Ho - 1)) * a.Wo + min(pw, a.Wo - 1)) * a.C + c0;
            uint4 d = *reinterpret_cast<const uint4*>(a.dpool + po);
            if (a.dpool1) d = add_bf16x8(d, *reinterpret_cast<const uint4*>(a.dpool1 + po));
            unpack8f(d, g[wy][wx]);
            const uint2 q = *reinterpret_cast<const uint2*>(a.arg + po);
            ar[wy][wx][0] = q.x;
            ar[wy][wx][1] = q.y;
        }
#pragma unroll
    for (int by = 0; by < 2; ++by)
#pragma unroll
        for (int bx = 0; bx < 2; ++bx) {
            const int ih = 2 * oh + by, iw = 2 * ow + bx;
            const size_t o = (((size_t)nb * a.H + ih) * a.W + iw) * a.C + c0;
            float acc[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] = 0.0f;
            // windows containing (ih, iw): row oh (+ oh + 1 when by == 1), column ow (+ ow + 1 when bx == 1),
            // in (oh, ow) order; the pixel's position in window (oh + wy, ow + wx)
#pragma unroll
            for (int wy = 0; wy < 2; ++wy) {
                if (wy > by) continue;
#pragma unroll
                for (int wx = 0; wx < 2; ++wx) {
                    if (wx > bx || !ok[wy][wx]) continue;
                    const uint32_t pos = (uint32_t)((1 + by - 2 * wy) * 3 + (1 + bx - 2 * wx));
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const uint32_t am = (ar[wy][wx][k >> 2] >> (8 * (k & 3))) & 0xffu;
                        if (am == pos) acc[k] += g[wy][wx][k];
                    }
                }
            }
            Vec<8> d;
#pragma unroll
            for (int k = 0; k < 8; ++k) d.v[k] = bfround(acc[k]);   // max_pool backward's bf16 gradient
            if (a.dskip) {
                const Vec<8> sk = ld_bf<8>(a.dskip + o);
#pragma unroll
                for (int k = 0; k < 8; ++k) d.v[k] = bfround(d.v[k] + sk.v[k]);
            }
            const Vec<8> r = ld_bf<8>(a.relu + o);
#pragma unroll
            for (int k = 0; k < 8; ++k) d.v[k] = r.v[k] <= 0.0f ? 0.0f : d.v[k];   // threshold_backward
            st_bf<8>(a.dx + o, d);
        }
}

// ------------------------------------------------------------------------------------------
// The nets' input images in bf16, in one pass each: the depth encoder's (x - 0.45) / 0.225
// (resnet_encoder.py:89) and PoseNet's channel concatenation of target + contexts (PoseNet.py:
// torch.cat([image, *context], 1)), each followed by autocast's bf16 cast for the first convolution
// — ATen runs sub, div, cast / cat, cast as separate passes over the fp32 images.  Same arithmetic:
// ATen's sub with a scalar is x + (-1 * a) = x - a in fp32, and its true division by a CPU scalar
// multiplies by the fp32 reciprocal (BinaryDivTrueKernel.cu), so y = bf16((x - a) * m) with m =
// 1.0f / b computed by the caller; the cast rounds to nearest even.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_normalize_bf16(const float* __restrict__ x, long long n, float a, float m,
                                                        uint16_t* __restrict__ y) {
    const long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (i + 4 <= n) {
        const float4 v = *reinterpret_cast<const float4*>(x + i);
        uint2 o;
        o.x = (uint32_t)f2bf((v.x - a) * m) | ((uint32_t)f2bf((v.y - a) * m) << 16);
        o.y = (uint32_t)f2bf((v.z - a) * m) | ((uint32_t)f2bf((v.w - a) * m) << 16);
        *reinterpret_cast<uint2*>(y + i) = o;
    } else {
        for (long long j = i; j < n; ++j) y[j] = f2bf((x[j] - a) * m);
    }
}

struct CatArgs {
    const float* x[4];
    int c[4];
    int k, ctot, pixels;
};

// NHWC: a workgroup per CAT_PX pixels.  Each input's slice of them (CAT_PX * c[q] consecutive floats)
// is read coalesced, converted and scattered into the block's output rows in LDS, then the block's
// CAT_PX * ctot bf16 values leave as coalesced 4-byte words (32-bit indexing: the host checks
// pixels * ctot < 2^31, ctot <= CAT_MAXC).
constexpr int CAT_PX = 256, CAT_MAXC = 32;

__global__ __launch_bounds__(256) void k_cat_channels_bf16(CatArgs a, uint16_t* __restrict__ y) {
    __shared__ uint16_t tile[CAT_PX * CAT_MAXC];
    const int t = threadIdx.x, p0 = blockIdx.x * CAT_PX, npx = min(CAT_PX, a.pixels - p0);
    int off = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (q >= a.k) break;
        const int cq = a.c[q], ne = npx * cq;
        const float* xi = a.x[q] + (size_t)p0 * cq;
        for (int e = t; e < ne; e += 256) {
            const int pp = e / cq;
            tile[pp * a.ctot + off + (e - pp * cq)] = f2bf(xi[e]);
        }
        off += cq;
    }
    __syncthreads();
    const int nout = npx * a.ctot;
    uint16_t* o = y + (size_t)p0 * a.ctot;
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(tile);
    for (int w = t; w < nout / 2; w += 256) reinterpret_cast<uint32_t*>(o)[w] = t32[w];
    if ((nout & 1) && t == 0) o[nout - 1] = tile[nout - 1];
}

}  // namespace

extern "C" {

static int pool_setup(PoolArgs& a, int N, int H, int W, int C, const char* who) {
    if (N < 1 || H < 2 || W < 2 || (H & 1) || (W & 1) || C < 8 || (C % 8)) return fail(-1, who);
    a.N = N, a.H = H, a.W = W, a.C = C, a.Ho = H / 2, a.Wo = W / 2, a.CV = C / 8;
    a.n = (long long)N * a.Ho * a.Wo * a.CV;
    return 0;
}

int psfm_normalize_bf16(const float* x, long long n, float sub, float mul, void* y, void* stream) {
    if (!x || !y || n < 1 || (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y) & 7))
        return fail(-1, "normalize_bf16: bad arguments (16-byte aligned x, 8-byte aligned y)");
    const long long threads = (n + 3) / 4;
    hipLaunchKernelGGL(k_normalize_bf16, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       x, n, sub, mul, static_cast<uint16_t*>(y));
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_cat_channels_bf16(int k, const float* const* xs, const int* channels, long long pixels, void* y,
                           void* stream) {
    if (k < 1 || k > 4 || !xs || !channels || !y || pixels < 1) return fail(-1, "cat_channels_bf16: bad arguments");
    CatArgs a{};
    a.k = k;
    long long ctot = 0;
    for (int q = 0; q < k; ++q) {
        if (!xs[q] || channels[q] < 1) return fail(-1, "cat_channels_bf16: bad input");
        a.x[q] = xs[q], a.c[q] = channels[q];
        ctot += channels[q];
    }
    if (pixels * ctot >= (1LL << 31) || ctot > CAT_MAXC || (reinterpret_cast<uintptr_t>(y) & 3))
        return fail(-1, "cat_channels_bf16: too large (pixels * channels < 2^31, <= 32 channels) or y not 4-byte aligned");
    a.ctot = (int)ctot;
    a.pixels = (int)pixels;
    hipLaunchKernelGGL(k_cat_channels_bf16, dim3((unsigned)((pixels + CAT_PX - 1) / CAT_PX)), dim3(256), 0,
                       (hipStream_t)stream, a, static_cast<uint16_t*>(y));
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_relu_maxpool_fwd(const void* x, int N, int H, int W, int C, void* relu_out, void* pool_out, void* argmax,
                          void* stream) {
    PoolArgs a{};
    if (!x || !relu_out || !pool_out || !argmax) return fail(-1, "relu_maxpool_fwd: bad arguments");
    if (int e = pool_setup(a, N, H, W, C, "relu_maxpool_fwd: H, W even, C % 8 == 0")) return e;
    a.x = static_cast<const uint16_t*>(x);
    a.relu = static_cast<uint16_t*>(relu_out);
    a.pool = static_cast<uint16_t*>(pool_out);
    a.arg = static_cast<uint8_t*>(argmax);
    hipLaunchKernelGGL(k_relu_maxpool_fwd, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_relu_maxpool_bwd(const void* dpool, const void* dpool1, const void* dskip, const void* relu_out,
                          const void* argmax, int N, int H, int W, int C, void* dx, void* stream) {
    PoolArgs a{};
    if (!dpool || !relu_out || !argmax || !dx) return fail(-1, "relu_maxpool_bwd: bad arguments");
    if (int e = pool_setup(a, N, H, W, C, "relu_maxpool_bwd: H, W even, C % 8 == 0")) return e;
    a.dpool = static_cast<const uint16_t*>(dpool);
    a.dpool1 = static_cast<const uint16_t*>(dpool1);
    a.dskip = static_cast<const uint16_t*>(dskip);
    a.relu = const_cast<uint16_t*>(static_cast<const uint16_t*>(relu_out));
    a.arg = const_cast<uint8_t*>(static_cast<const uint8_t*>(argmax));
    a.dx = static_cast<uint16_t*>(dx);
    hipLaunchKernelGGL(k_relu_maxpool_bwd, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

static int upcat_check(int N, int h, int w, int C1, int C2, const char* who) {
    if (N < 1 || h < 1 || w < 1 || C1 < 8 || C2 < 0 || (C1 % 8) || (C2 % 8)) return fail(-1, who);
    if ((long long)N * 4 * h * w * (C1 + C2) / 8 >= (1LL << 32)) return fail(-1, who);
    return 0;
}

static UpcatArgs upcat_args(int N, int h, int w, int C1, int C2) {
    UpcatArgs a{};
    a.N = N, a.h = h, a.w = w, a.V1 = C1 / 8, a.V2 = C2 / 8;
    a.nfwd = (uint32_t)((size_t)N * 4 * h * w * (a.V1 + a.V2));
    a.ndx = (uint32_t)((size_t)N * h * w * a.V1);
    a.ndskip = (uint32_t)((size_t)N * 4 * h * w * a.V2);
    a.nbx = (a.ndx + 255) / 256;
    return a;
}

int psfm_upcat_fwd(const void* x, const void* skip, int N, int h, int w, int C1, int C2, void* out, void* stream) {
    if (int e = upcat_check(N, h, w, C1, C2, "upcat_fwd: bad shape (C1 >= 8, C1 and C2 multiples of 8)")) return e;
    if (!x || !out || (C2 > 0 && !skip)) return fail(-1, "upcat_fwd: null pointer");
    UpcatArgs a = upcat_args(N, h, w, C1, C2);
    a.x = static_cast<const uint4*>(x);
    a.skip = static_cast<const uint4*>(skip);
    a.out = static_cast<uint4*>(out);
    hipLaunchKernelGGL(k_upcat_fwd<false>, dim3((a.nfwd + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_upcat_bwd(const void* dout, int N, int h, int w, int C1, int C2, void* dx, void* dskip, void* stream) {
    if (int e = upcat_check(N, h, w, C1, C2, "upcat_bwd: bad shape (C1 >= 8, C1 and C2 multiples of 8)")) return e;
    if (!dout || !dx || (C2 > 0 && !dskip)) return fail(-1, "upcat_bwd: null pointer");
    UpcatArgs a = upcat_args(N, h, w, C1, C2);
    a.dout = static_cast<const uint4*>(dout);
    a.dx = static_cast<uint4*>(dx);
    a.dskip = static_cast<uint4*>(dskip);
    const uint32_t nb = a.nbx + (a.ndskip + 255) / 256;
    hipLaunchKernelGGL(k_upcat_bwd<false>, dim3(nb), dim3(256), 0, (hipStream_t)stream, a);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

static int upcat_relu_check(int C1, const char* who) {
    if (256 % (C1 / 8) != 0) return fail(-2, (std::string(who) + ": C1 / 8 must divide 256").c_str());
    return 0;
}

size_t psfm_upcat_ws_floats(int N, int h, int w, int C1) {
    return (size_t)upcat_args(N, h, w, C1, 0).nbx * (size_t)C1;
}

int psfm_upcat_bias_relu_fwd(const void* x, const void* bias, int bias_bf16, const void* skip, int N, int h, int w,
                             int C1, int C2, void* out, void* stream) {
    if (int e = upcat_check(N, h, w, C1, C2, "upcat_bias_relu_fwd: bad shape (C1 >= 8, C1 and C2 multiples of 8)"))
        return e;
    if (int e = upcat_relu_check(C1, "upcat_bias_relu_fwd")) return e;
    if (!x || !bias || !out || (C2 > 0 && !skip)) return fail(-1, "upcat_bias_relu_fwd: null pointer");
    UpcatArgs a = upcat_args(N, h, w, C1, C2);
    a.x = static_cast<const uint4*>(x);
    a.skip = static_cast<const uint4*>(skip);
    a.out = static_cast<uint4*>(out);
    a.bias = bias, a.bias_bf16 = bias_bf16;
    hipLaunchKernelGGL(k_upcat_fwd<true>, dim3((a.nfwd + 255) / 256), dim3(256), 0, (hipStream_t)stream, a);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_upcat_bias_relu_bwd(const void* dout, const void* out, int N, int h, int w, int C1, int C2, void* dx,
                             void* dskip, void* dbias, int bias_bf16, float* ws, void* stream) {
    if (int e = upcat_check(N, h, w, C1, C2, "upcat_bias_relu_bwd: bad shape (C1 >= 8, C1 and C2 multiples of 8)"))
        return e;
    if (int e = upcat_relu_check(C1, "upcat_bias_relu_bwd")) return e;
    if (!dout || !out || !dx || !dbias || !ws || (C2 > 0 && !dskip)) return fail(-1, "upcat_bias_relu_bwd: null pointer");
    UpcatArgs a = upcat_args(N, h, w, C1, C2);
    a.dout = static_cast<const uint4*>(dout);
    a.out = static_cast<uint4*>(const_cast<void*>(out));
    a.dx = static_cast<uint4*>(dx);
    a.dskip = static_cast<uint4*>(dskip);
    a.rows = ws;
    hipStream_t st = (hipStream_t)stream;
    const uint32_t nb = a.nbx + (a.ndskip + 255) / 256;
    hipLaunchKernelGGL(k_upcat_bwd<true>, dim3(nb), dim3(256), 0, st, a);
    NETOPS_LAUNCH_CHECK();
    const ColJob job{ws, dbias, C1, 0, (int)a.nbx, C1, bias_bf16};
    if (hipError_t e = launch_finish(&job, 1, st)) return fail((int)e, "upcat_bias_relu_bwd: finish launch");
    return 0;
}

size_t psfm_netops_ws_floats(int M, int C) {   // partial rows [nblk][2C] + coefficients [3][C]
    const Geo g = geometry(M, C, pick_vec(C));
    return bn_coef_off(g.nblk, C) + 3 * (size_t)C;
}

size_t psfm_gn_ws_floats(int N, int HW, int C, int G) {
    // two-pass statistics rows, or the resident backward's per-sample parameter rows [N][3][C]
    return std::max(gn_ws(N, gn_geometry(N, HW, C).nblk, C, G), align4((size_t)3 * N * C));
}

int psfm_add_relu_fwd(const void* a, const void* b, long long n, void* y, void* stream) {
    if (!a || !y || n < 0 || n % 8 || (((uintptr_t)a | (uintptr_t)b | (uintptr_t)y) & 15))
        return fail(-1, "add_relu_fwd: n a multiple of 8, 16-byte aligned bf16 buffers");
    const long long n8 = n / 8;
    if (n8) hipLaunchKernelGGL(k_add_relu_fwd, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                               static_cast<const uint4*>(a), static_cast<const uint4*>(b), static_cast<uint4*>(y), n8);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_relu_mask_bwd_sum(const void* dy, const void* dy1, const void* dy2, const void* y, long long n, void* dz,
                           void* stream) {
    if (!dy || !y || !dz || n < 0 || n % 8 ||
        (((uintptr_t)dy | (uintptr_t)dy1 | (uintptr_t)dy2 | (uintptr_t)y | (uintptr_t)dz) & 15))
        return fail(-1, "relu_mask_bwd: n a multiple of 8, 16-byte aligned bf16 buffers");
    const long long n8 = n / 8;
    if (n8) hipLaunchKernelGGL(k_relu_mask_bwd, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                               static_cast<const uint4*>(dy), static_cast<const uint4*>(dy1),
                               static_cast<const uint4*>(dy2), static_cast<const uint4*>(y), static_cast<uint4*>(dz), n8);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_relu_mask_bwd(const void* dy, const void* y, long long n, void* dz, void* stream) {
    return psfm_relu_mask_bwd_sum(dy, nullptr, nullptr, y, n, dz, stream);
}

int psfm_bias_act_fwd(const void* x, const void* bias, int bias_bf16, int M, int C, int act, void* y, void* stream) {
    if (!x || !bias || !y || M < 1 || C < 1) return fail(-1, "bias_act_fwd: bad arguments");
    if (int e = check_vec(C, "bias_act_fwd")) return e;
    const int vec = pick_vec(C);
    const Geo g = geometry(M, C, vec);
    BiasArgs a{};
    a.x = static_cast<const uint16_t*>(x);
    a.bias = bias;
    a.out = y;
    a.M = M, a.C = C, a.act = act, a.bias_bf16 = bias_bf16, a.nblk = g.nblk;
    set_geo(a, g);
    if (vec == 8)
        hipLaunchKernelGGL(k_bias_act_fwd<8>, dim3(g.nblk), dim3(NT), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(k_bias_act_fwd<1>, dim3(g.nblk), dim3(NT), 0, (hipStream_t)stream, a);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_bias_act_bwd(const void* dy, const void* y, int M, int C, int act, void* dx, void* dbias, int bias_bf16,
                      float* ws, void* stream) {
    return psfm_bias_act_bwd_sum(dy, nullptr, y, M, C, act, dx, dbias, bias_bf16, ws, stream);
}

int psfm_bias_act_bwd_sum(const void* dy, const void* dy1, const void* y, int M, int C, int act, void* dx, void* dbias,
                          int bias_bf16, float* ws, void* stream) {
    if (!dy || !y || !dx || !dbias || !ws || M < 1 || C < 1 || (dy1 && act == PSFM_ACT_SIGMOID))
        return fail(-1, "bias_act_bwd: bad arguments");
    if (int e = check_vec(C, "bias_act_bwd")) return e;
    const int vec = pick_vec(C);
    const Geo g = geometry(M, C, vec);
    BiasArgs a{};
    a.dy = dy;
    a.dy1 = dy1;
    a.y = y;
    a.out = dx;
    a.ws = ws;
    a.M = M, a.C = C, a.act = act, a.bias_bf16 = bias_bf16, a.nblk = g.nblk;
    set_geo(a, g);
    hipStream_t st = (hipStream_t)stream;
    if (vec == 8)
        hipLaunchKernelGGL(k_bias_act_bwd<8>, dim3(g.nblk), dim3(NT), 0, st, a);
    else
        hipLaunchKernelGGL(k_bias_act_bwd<1>, dim3(g.nblk), dim3(NT), 0, st, a);
    NETOPS_LAUNCH_CHECK();
    const ColJob job{ws, dbias, C, 0, g.nblk, C, bias_bf16};
    if (hipError_t e = launch_finish(&job, 1, st)) return fail((int)e, "bias_act_bwd: finish launch");
    return 0;
}

// BatchNorm form: 0 the resident kernels (forward: up to BN_RES_MAXM rows; backward: any shape they
// hold), -1 none (MIOpen's BatchNorm runs there).  The ticket / three-pass forms were removed in round 6.
static int bn_form(int M, int C, BNRGeo& rg, bool bwd) {
    if (bnr_geometry(M, C, rg, bwd)) return 0;
    return -1;
}
int psfm_bn_act_resident(int M, int C) {
    BNRGeo g;
    return bnr_geometry(M, C, g) ? 1 : 0;
}

int psfm_bn_act_fused(int M, int C) {
    BNRGeo g;
    const int f = bn_form(M, C, g, false);
    return f == 0 || f == 1 ? 1 : 0;
}


int psfm_bn_act_fwd(const void* x, const void* res, const float* gamma, const float* beta, float* run_mean,
                    float* run_var, float momentum, float eps, int M, int C, int relu, void* y, float* save_mean,
                    float* save_invstd, float* ws, void* stream) {
    if (!x || !gamma || !beta || !y || !save_mean || !save_invstd || M < 1 || C < 1)
        return fail(-1, "bn_act_fwd: bad arguments");
    if ((run_mean == nullptr) != (run_var == nullptr)) return fail(-1, "bn_act_fwd: running stats must pair");
    if (int e = check_vec(C, "bn_act_fwd")) return e;
    BNRGeo rgeo;
    const int form = bn_form(M, C, rgeo, false);
    if (form == 0) {  // one launch (resident)
        BNRArgs a{};
        a.x = static_cast<const uint16_t*>(x);
        a.res = static_cast<const uint16_t*>(res);
        a.gamma = gamma, a.beta = beta, a.run_mean = run_mean, a.run_var = run_var;
        a.save_mean = save_mean, a.save_invstd = save_invstd;
        a.out = static_cast<uint16_t*>(y);
        a.momentum = momentum, a.eps = eps, a.M = M, a.C = C, a.relu = relu, a.nb = C / 8;
        hipStream_t st = (hipStream_t)stream;
        const BNRGeo& g = rgeo;
        switch (g.rpt) { BNR_FWD_CASE(1); BNR_FWD_CASE(2); BNR_FWD_CASE(4); BNR_FWD_CASE(8); }
        NETOPS_LAUNCH_CHECK();
        return 0;
    }
    (void)ws;
    return fail(-3, "bn_act_fwd: no fused BatchNorm for this shape (psfm_bn_act_fused: C % 8 == 0, C <= 512, M <= "
                    "BN_RES_MAXM)");
}

int psfm_bn_act_bwd(const void* dy, const void* y, const void* x, const float* gamma, const float* save_mean,
                    const float* save_invstd, int M, int C, int relu, void* dx, void* dres, float* dgamma,
                    float* dbeta, float* ws, void* stream) {
    return psfm_bn_act_bwd_sum(dy, nullptr, nullptr, y, x, gamma, save_mean, save_invstd, M, C, relu, dx, dres, dgamma,
                               dbeta, ws, stream);
}

int psfm_bn_act_bwd_sum(const void* dy, const void* dy1, const void* dy2, const void* y, const void* x,
                        const float* gamma, const float* save_mean, const float* save_invstd, int M, int C, int relu,
                        void* dx, void* dres, float* dgamma, float* dbeta, float* ws, void* stream) {
    if (!dy || !x || !gamma || !save_mean || !save_invstd || !dx || !dgamma || !dbeta ||
        M < 1 || C < 1 || (relu && !y))
        return fail(-1, "bn_act_bwd: bad arguments");
    if (int e = check_vec(C, "bn_act_bwd")) return e;
    BNRGeo rgeo;
    const int form = bn_form(M, C, rgeo, true);
    if (form == 0) {  // one launch (resident)
        BNRArgs a{};
        a.dy = static_cast<const uint16_t*>(dy);
        a.y = static_cast<const uint16_t*>(y);
        a.x = static_cast<const uint16_t*>(x);
        a.gamma = gamma, a.save_mean = const_cast<float*>(save_mean), a.save_invstd = const_cast<float*>(save_invstd);
        a.out = static_cast<uint16_t*>(dx);
        a.dres = static_cast<uint16_t*>(dres);
        a.dy1 = static_cast<const uint16_t*>(dy1), a.dy2 = static_cast<const uint16_t*>(dy2);
        a.dgamma = dgamma, a.dbeta = dbeta, a.M = M, a.C = C, a.relu = relu, a.nb = C / 8;
        hipStream_t st = (hipStream_t)stream;
        const BNRGeo& g = rgeo;
        switch (g.rpt) { BNR_BWD_CASE(1); BNR_BWD_CASE(2); BNR_BWD_CASE(4); BNR_BWD_CASE(8); BNR_BWD_CASE(16); }
        NETOPS_LAUNCH_CHECK();
        return 0;
    }
    (void)ws;
    return fail(-3, "bn_act_bwd: no fused BatchNorm for this shape (C % 8 == 0, C <= 512, M <= 8192)");
}

// the resident path is the default; the GN_PATH knob = 1 forces the two-pass kernels (A/B, tests)
static bool gnr_enabled() { return knob(KNOB_GN_PATH) == 0; }
static void gnr_common(GNRArgs& r, const GNRGeo& rg, const GNArgs& a) {
    r.x = a.x, r.res = a.res, r.bias = a.bias, r.bias_bf16 = a.bias_bf16, r.gamma = a.gamma, r.beta = a.beta;
    r.save_mean = a.save_mean, r.save_invstd = a.save_invstd, r.out = a.out, r.eps = a.eps;
    r.N = a.N, r.HW = a.HW, r.C = a.C, r.NG = a.NG, r.act = a.act;
    r.cpg = a.C / a.NG, r.CB = rg.CB, r.CV = rg.CV, r.gpw = rg.gpw, r.nblk = a.C / rg.CB;
}

static int gn_setup(GNArgs& a, int N, int HW, int C, int G, Geo& g, int& vec) {
    if (N < 1 || HW < 1 || C < 1 || G < 1 || C % G != 0) return fail(-1, "groupnorm: bad shape");
    if (int e = check_vec(C, "groupnorm")) return e;
    if (C > MAX_C || G > MAX_NG || N > 64) return fail(-2, "groupnorm: C <= 512, G <= 128, N <= 64");
    vec = pick_vec(C);
    g = gn_geometry(N, HW, C);
    a.N = N, a.HW = HW, a.C = C, a.NG = G, a.bpn = g.nblk;
    set_geo(a, g);
    return 0;
}

int psfm_gn_act_fwd(const void* x, const void* res, const void* bias, int bias_bf16, const float* gamma,
                    const float* beta, float eps, int N, int HW, int C, int G, int act, void* y, float* save_mean,
                    float* save_invstd, float* ws, void* stream) {
    if (!x || !gamma || !beta || !y || !save_mean || !save_invstd || !ws ||
        (act != PSFM_ACT_NONE && act != PSFM_ACT_RELU && act != PSFM_ACT_ELU))
        return fail(-1, "gn_act_fwd: bad arguments");
    GNArgs a{};
    Geo g;
    int vec;
    if (int e = gn_setup(a, N, HW, C, G, g, vec)) return e;
    a.x = static_cast<const uint16_t*>(x);
    a.res = static_cast<const uint16_t*>(res);
    a.bias = bias, a.bias_bf16 = bias_bf16, a.gamma = gamma, a.beta = beta, a.eps = eps;
    a.save_mean = save_mean, a.save_invstd = save_invstd;
    a.out = static_cast<uint16_t*>(y);
    a.ws = ws, a.act = act, a.RW = 2 * G;
    hipStream_t st = (hipStream_t)stream;
    GNRGeo rg;
    if (vec == 8 && gnr_enabled() && gnr_geometry(HW, C, G, gnr_cap_fwd(res != nullptr), rg)) {
        GNRArgs r{};
        gnr_common(r, rg, a);
        const dim3 rgrid(N * r.nblk);
        GNR_LAUNCH_FWD(rg.rpt, res != nullptr, rgrid, rg.nthr, st, r);
        NETOPS_LAUNCH_CHECK();
        return 0;
    }
    const dim3 grid(N * g.nblk);
    if (vec == 8) {
        if (res) {
            hipLaunchKernelGGL(k_gnp_fwd_stats<true>, grid, dim3(NT), 0, st, a);
            hipLaunchKernelGGL(k_gnp_fwd_apply<true>, grid, dim3(NT), 0, st, a);
        } else {
            hipLaunchKernelGGL(k_gnp_fwd_stats<false>, grid, dim3(NT), 0, st, a);
            hipLaunchKernelGGL(k_gnp_fwd_apply<false>, grid, dim3(NT), 0, st, a);
        }
    } else {
        hipLaunchKernelGGL(k_gn_fwd_stats<1>, grid, dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_gn_fwd_apply<1>, grid, dim3(NT), 0, st, a);
    }
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_gn_act_bwd(const void* dy, const void* x, const void* res, const void* bias, int bias_bf16,
                    const float* gamma, const float* beta, const float* save_mean, const float* save_invstd, int N,
                    int HW, int C, int G, int act, void* dx, void* dres, void* dbias, float* dgamma, float* dbeta,
                    float* ws, void* stream) {
    if (!dy || !x || !gamma || !beta || !save_mean || !save_invstd || !dx || !dgamma || !dbeta || !ws ||
        (act != PSFM_ACT_NONE && act != PSFM_ACT_RELU && act != PSFM_ACT_ELU) || (res && !dres) || (bias && !dbias))
        return fail(-1, "gn_act_bwd: bad arguments");
    GNArgs a{};
    Geo g;
    int vec;
    if (int e = gn_setup(a, N, HW, C, G, g, vec)) return e;
    a.dy = static_cast<const uint16_t*>(dy);
    a.x = static_cast<const uint16_t*>(x);
    a.res = static_cast<const uint16_t*>(res);
    a.bias = bias, a.bias_bf16 = bias_bf16, a.gamma = gamma, a.beta = beta;
    a.save_mean = const_cast<float*>(save_mean), a.save_invstd = const_cast<float*>(save_invstd);
    a.out = static_cast<uint16_t*>(dx);
    a.out2 = static_cast<uint16_t*>(dres);
    a.ws = ws, a.act = act, a.RW = gn_rw_bwd(C, G);
    a.dbias = dbias, a.dgamma = dgamma, a.dbeta = dbeta;
    hipStream_t st = (hipStream_t)stream;
    GNRGeo rg;
    if (vec == 8 && gnr_enabled() && gnr_geometry(HW, C, G, gnr_cap_bwd(res != nullptr), rg)) {
        GNRArgs r{};
        gnr_common(r, rg, a);
        r.dy = a.dy, r.out2 = a.out2, r.part = ws, r.dbias = dbias, r.dgamma = dgamma, r.dbeta = dbeta;
        const dim3 rgrid(N * r.nblk);
        GNR_LAUNCH_BWD(rg.rpt, res != nullptr, rgrid, rg.nthr, st, r);
        hipLaunchKernelGGL(k_gnr_params, dim3((C + 255) / 256), dim3(256), 0, st, r);
        NETOPS_LAUNCH_CHECK();
        return 0;
    }
    const dim3 grid(N * g.nblk), grid_apply(N * g.nblk + (C + 3) / 4);
    if (vec == 8) {
        if (res) {
            hipLaunchKernelGGL(k_gnp_bwd_stats<true>, grid, dim3(NT), 0, st, a);
            hipLaunchKernelGGL(k_gnp_bwd_apply<true>, grid_apply, dim3(NT), 0, st, a);
        } else {
            hipLaunchKernelGGL(k_gnp_bwd_stats<false>, grid, dim3(NT), 0, st, a);
            hipLaunchKernelGGL(k_gnp_bwd_apply<false>, grid_apply, dim3(NT), 0, st, a);
        }
    } else {
        hipLaunchKernelGGL(k_gn_bwd_stats<1>, grid, dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_gn_bwd_apply<1>, grid_apply, dim3(NT), 0, st, a);
    }
    NETOPS_LAUNCH_CHECK();
    return 0;
}

const char* psfm_netops_last_error(void) { return g_err.c_str(); }

}  // extern "C"
