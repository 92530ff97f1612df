// psfm_netops.hip — fused BatchNorm / GroupNorm / bias + activation kernels of the depth and
// pose networks (include/psfm_netops.h), gfx950.
//
// An activation is a bf16 matrix [M, C] (NHWC storage).  A workgroup of 256 threads covers TR
// rows x C channels per iteration: thread t owns the VEC consecutive channels (t % G)*VEC.. of
// row lane t / G (G = C/VEC; VEC = 8: one 16-byte load per thread, fully coalesced rows) and
// walks its workgroup's row range with stride TR.  Column reductions: per-thread fp32 sums ->
// LDS tree over the TR row lanes -> per-workgroup partials in `ws` -> the last workgroup to
// arrive (device-scope int counter) sums the partials in a fixed order (fp64) and writes the
// per-channel results.  Deterministic; no float atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>

#include "../../include/psfm_netops.h"

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

constexpr int NT = 256;
constexpr int TARGET_BLOCKS = 512;  // ~2 workgroups per CU for the streaming passes

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even (NaN stays NaN)
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

template <int VEC>
struct Vec {
    float v[VEC];
};

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

template <int VEC>
__device__ __forceinline__ Vec<VEC> ld_f(const float* __restrict__ p) {
    Vec<VEC> r;
#pragma unroll
    for (int i = 0; i < VEC; ++i) r.v[i] = p[i];
    return r;
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

// Work geometry of an [M, C] pass: G = C / VEC vector columns, TR = row lanes per workgroup.
struct Geo {
    int G, TR, rpb, nblk;
};
// Reduction passes use fewer, fuller workgroups (>= MIN_ITERS rows per row lane): the partials
// the last workgroup sums stay few.
constexpr int RED_BLOCKS = 256;
constexpr int MIN_ITERS = 8;
inline Geo geometry(int M, int C, int vec, int target = TARGET_BLOCKS, int min_iters = 1) {
    Geo g;
    g.G = C / vec;
    g.TR = std::max(1, NT / g.G);
    int rpb = (M + target - 1) / target;
    rpb = std::max(g.TR * min_iters, (rpb + g.TR - 1) / g.TR * g.TR);
    rpb = std::min(rpb, (M + g.TR - 1) / g.TR * g.TR);
    g.rpb = rpb;
    g.nblk = (M + rpb - 1) / rpb;
    return g;
}
inline int pick_vec(int C) { return (C % 8 == 0 && C / 8 <= NT) ? 8 : 1; }

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

// Cross-XCD visibility without cache-wide fences: the L2 of an XCD is not coherent with the
// others, and a device-scope release fence would write back the whole L2 (buffer_wbl2) in every
// workgroup.  Instead the partials are written with device-scope relaxed atomic stores and read
// back with device-scope atomic loads (both bypass the non-coherent L2 level, sc1), their
// completion is awaited explicitly (s_waitcnt) before the counter increment, and the counter is
// a device-scope RMW (performed at the coherent memory side).
__device__ __forceinline__ void st_part(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_part(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Last-workgroup election after this workgroup's partials are stored (st_part): true (in every
// thread) only in the last workgroup, which then reads every other workgroup's partials with
// ld_part.  The counter is re-armed to 0 for the next launch (graph replays included).
__device__ __forceinline__ bool last_block(int* counter, int nblk) {
    __shared__ int is_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        const int prev = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (prev == nblk - 1);
        if (is_last) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return is_last;
}

// Fixed-order sum of the K partial arrays ws[b*stride + k*C + c] over b in [b0, b0+nb) for the
// channels [cbeg, cbeg+nc) (nc <= NT): threads split channels x block ranges, combined through
// LDS in fixed order.  out[k*nc + i] (fp64, LDS), valid after the call in every thread.
template <int K>
__device__ void final_colsum(const float* __restrict__ ws, size_t stride, int b0, int nb, int C, int cbeg, int nc,
                             double* out, double* scratch /* LDS [NT*K] */) {
    const int t = threadIdx.x;
    const int tpc = NT / nc;
    const int c = cbeg + t % nc, sub = t / nc;
    double s[K];
#pragma unroll
    for (int k = 0; k < K; ++k) s[k] = 0.0;
    if (sub < tpc) {
        constexpr int U = 8;  // independent loads in flight per thread, summed in order after
        for (int b = sub; b < nb; b += U * tpc) {
            float v[U][K];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int bb = b + u * tpc;
#pragma unroll
                for (int k = 0; k < K; ++k)
                    v[u][k] = bb < nb ? ld_part(&ws[(size_t)(b0 + bb) * stride + (size_t)k * C + c]) : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int k = 0; k < K; ++k) s[k] += (double)v[u][k];
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) scratch[t * K + k] = s[k];
    __syncthreads();
    if (t < nc) {
        for (int u = 1; u < tpc; ++u)
#pragma unroll
            for (int k = 0; k < K; ++k) s[k] += scratch[(u * nc + t) * K + k];
#pragma unroll
        for (int k = 0; k < K; ++k) out[k * nc + t] = s[k];
    }
    __syncthreads();
}

__device__ __forceinline__ float act_fwd(float v, int act) {
    if (act == PSFM_ACT_RELU) return fmaxf(v, 0.0f);
    if (act == PSFM_ACT_SIGMOID) return 1.0f / (1.0f + expf(-v));
    return v;
}

// ------------------------------------------------------------------------------------------
// bias + activation (decoder ConvBlock / disparity head)
// ------------------------------------------------------------------------------------------
struct BiasArgs {
    const uint16_t* x;
    const void* bias;
    const void* dy;
    const void* y;
    void* out;  // y (fwd) / dx (bwd)
    void* dbias;
    float* ws;
    int* counter;
    int M, C, act, bias_bf16, G, TR, rpb, nblk;
};

template <int VEC>
__global__ __launch_bounds__(NT) void k_bias_act_fwd(BiasArgs a) {
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    if (r >= a.TR) return;
    const int c0 = cg * VEC;
    const Vec<VEC> b = ld_param<VEC>(a.bias, a.bias_bf16, c0);
    const int row0 = blockIdx.x * a.rpb, row1 = min(a.M, row0 + a.rpb);
    for (int row = row0 + r; row < row1; row += a.TR) {
        const size_t o = (size_t)row * a.C + c0;
        Vec<VEC> v = ld_bf<VEC>(a.x + o);
#pragma unroll
        for (int i = 0; i < VEC; ++i) v.v[i] = act_fwd(v.v[i] + b.v[i], a.act);
        if (a.act == PSFM_ACT_SIGMOID) {
            float* y = static_cast<float*>(a.out) + o;
#pragma unroll
            for (int i = 0; i < VEC; ++i) y[i] = v.v[i];
        } else {
            st_bf<VEC>(static_cast<uint16_t*>(a.out) + o, v);
        }
    }
}

template <int VEC>
__global__ __launch_bounds__(NT) void k_bias_act_bwd(BiasArgs a) {
    __shared__ float red[NT * VEC];
    __shared__ double fin[NT];
    __shared__ double scratch[NT];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    float acc[1][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = 0.0f;
    if (r < a.TR) {
        const int row0 = blockIdx.x * a.rpb, row1 = min(a.M, row0 + a.rpb);
        for (int row = row0 + r; row < row1; row += a.TR) {
            const size_t o = (size_t)row * a.C + c0;
            Vec<VEC> g;
            if (a.act == PSFM_ACT_SIGMOID) {
                const Vec<VEC> dy = ld_f<VEC>(static_cast<const float*>(a.dy) + o);
                const Vec<VEC> y = ld_f<VEC>(static_cast<const float*>(a.y) + o);
#pragma unroll
                for (int i = 0; i < VEC; ++i) g.v[i] = dy.v[i] * ((1.0f - y.v[i]) * y.v[i]);
            } else {
                const Vec<VEC> dy = ld_bf<VEC>(static_cast<const uint16_t*>(a.dy) + o);
                const Vec<VEC> y = ld_bf<VEC>(static_cast<const uint16_t*>(a.y) + o);
#pragma unroll
                for (int i = 0; i < VEC; ++i)
                    g.v[i] = (a.act == PSFM_ACT_RELU && !(y.v[i] > 0.0f)) ? 0.0f : dy.v[i];
            }
            Vec<VEC> gq;  // the stored (bf16) gradient is the one the bias sums, as autograd's would
            st_bf<VEC>(static_cast<uint16_t*>(a.out) + o, g);
#pragma unroll
            for (int i = 0; i < VEC; ++i) gq.v[i] = bf2f(f2bf(g.v[i]));
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[0][i] += gq.v[i];
        }
    }
    block_colsum<VEC, 1>(acc, red, a.G, a.TR);
    if (r == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) st_part(&a.ws[(size_t)blockIdx.x * a.C + c0 + i], acc[0][i]);
    }
    if (!last_block(a.counter, a.nblk)) return;
    for (int cb = 0; cb < a.C; cb += NT) {
        const int nc = min(NT, a.C - cb);
        final_colsum<1>(a.ws, a.C, 0, a.nblk, a.C, cb, nc, fin, scratch);
        if (t < nc) {
            if (a.bias_bf16)
                static_cast<uint16_t*>(a.dbias)[cb + t] = f2bf((float)fin[t]);
            else
                static_cast<float*>(a.dbias)[cb + t] = (float)fin[t];
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------
// BatchNorm (training) + residual + ReLU
// ------------------------------------------------------------------------------------------
struct BNArgs {
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
    uint16_t* dres;  // bwd
    float* dgamma;
    float* dbeta;
    float* ws;       // [nblk][2][C] partials, then [2][C] coefficients
    int* counter;
    float momentum, eps;
    int M, C, relu, G, TR, rpb, nblk;
};

// pass 1: per-channel sum / sum of squares; last block -> mean, invstd, running stats and the
// affine coefficients scale = gamma*invstd, shift = beta - mean*scale (ws tail).
template <int VEC>
__global__ __launch_bounds__(NT) void k_bn_fwd_stats(BNArgs a) {
    __shared__ float red[2 * NT * VEC];
    __shared__ double fin[2 * NT];
    __shared__ double scratch[2 * NT];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    float acc[2][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = acc[1][i] = 0.0f;
    if (r < a.TR) {
        const int row0 = blockIdx.x * a.rpb, row1 = min(a.M, row0 + a.rpb);
        for (int row = row0 + r; row < row1; row += a.TR) {
            const Vec<VEC> v = ld_bf<VEC>(a.x + (size_t)row * a.C + c0);
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                acc[0][i] += v.v[i];
                acc[1][i] += v.v[i] * v.v[i];
            }
        }
    }
    block_colsum<VEC, 2>(acc, red, a.G, a.TR);
    if (r == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            st_part(&a.ws[((size_t)blockIdx.x * 2 + 0) * a.C + c0 + i], acc[0][i]);
            st_part(&a.ws[((size_t)blockIdx.x * 2 + 1) * a.C + c0 + i], acc[1][i]);
        }
    }
    if (!last_block(a.counter, a.nblk)) return;
    float* coef = a.ws + (size_t)a.nblk * 2 * a.C;  // [2][C]: scale, shift
    const double inv_m = 1.0 / (double)a.M;
    for (int cb = 0; cb < a.C; cb += NT) {
        const int nc = min(NT, a.C - cb);
        final_colsum<2>(a.ws, 2 * (size_t)a.C, 0, a.nblk, a.C, cb, nc, fin, scratch);
        if (t < nc) {
            const int c = cb + t;
            const double mean = fin[t] * inv_m;
            const double var = fmax(fin[nc + t] * inv_m - mean * mean, 0.0);
            const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
            a.save_mean[c] = (float)mean;
            a.save_invstd[c] = invstd;
            if (a.run_mean) {  // torch: running = (1-m) running + m batch (unbiased var)
                const double unb = a.M > 1 ? var * (double)a.M / (double)(a.M - 1) : var;
                a.run_mean[c] = (float)((1.0 - a.momentum) * a.run_mean[c] + a.momentum * mean);
                a.run_var[c] = (float)((1.0 - a.momentum) * a.run_var[c] + a.momentum * unb);
            }
            const float scale = a.gamma[c] * invstd;
            coef[c] = scale;
            coef[a.C + c] = a.beta[c] - (float)mean * scale;
        }
        __syncthreads();
    }
}

// pass 2: y = act(x*scale + shift [+ res])
template <int VEC>
__global__ __launch_bounds__(NT) void k_bn_fwd_apply(BNArgs a) {
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    if (r >= a.TR) return;
    const int c0 = cg * VEC;
    const float* coef = a.ws + (size_t)a.nblk * 2 * a.C;
    const Vec<VEC> sc = ld_f<VEC>(coef + c0), sh = ld_f<VEC>(coef + a.C + c0);
    const int row0 = blockIdx.x * a.rpb, row1 = min(a.M, row0 + a.rpb);
    for (int row = row0 + r; row < row1; row += a.TR) {
        const size_t o = (size_t)row * a.C + c0;
        Vec<VEC> v = ld_bf<VEC>(a.x + o);
#pragma unroll
        for (int i = 0; i < VEC; ++i) v.v[i] = v.v[i] * sc.v[i] + sh.v[i];
        if (a.res) {
            // the reference rounds bn(x) to bf16 before the residual add (both operands bf16)
            const Vec<VEC> rv = ld_bf<VEC>(a.res + o);
#pragma unroll
            for (int i = 0; i < VEC; ++i) v.v[i] = bf2f(f2bf(v.v[i])) + rv.v[i];
        }
        if (a.relu) {
#pragma unroll
            for (int i = 0; i < VEC; ++i) v.v[i] = fmaxf(v.v[i], 0.0f);
        }
        st_bf<VEC>(a.out + o, v);
    }
}

// backward pass 1: per channel sum(dyr), sum(dyr * (x - mean)); last block -> dgamma, dbeta and
// dx coefficients k1 = gamma*invstd, k2 = sum(dyr)/M, k3 = sum(dyr*xc)*invstd^2/M.
template <int VEC>
__global__ __launch_bounds__(NT) void k_bn_bwd_stats(BNArgs a) {
    __shared__ float red[2 * NT * VEC];
    __shared__ double fin[2 * NT];
    __shared__ double scratch[2 * NT];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    float acc[2][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = acc[1][i] = 0.0f;
    if (r < a.TR) {
        const Vec<VEC> mu = ld_f<VEC>(a.save_mean + c0);
        const int row0 = blockIdx.x * a.rpb, row1 = min(a.M, row0 + a.rpb);
        for (int row = row0 + r; row < row1; row += a.TR) {
            const size_t o = (size_t)row * a.C + c0;
            Vec<VEC> g = ld_bf<VEC>(a.dy + o);
            if (a.relu) {
                const Vec<VEC> y = ld_bf<VEC>(a.y + o);
#pragma unroll
                for (int i = 0; i < VEC; ++i) g.v[i] = y.v[i] > 0.0f ? g.v[i] : 0.0f;
            }
            const Vec<VEC> x = ld_bf<VEC>(a.x + o);
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                acc[0][i] += g.v[i];
                acc[1][i] += g.v[i] * (x.v[i] - mu.v[i]);
            }
        }
    }
    block_colsum<VEC, 2>(acc, red, a.G, a.TR);
    if (r == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            st_part(&a.ws[((size_t)blockIdx.x * 2 + 0) * a.C + c0 + i], acc[0][i]);
            st_part(&a.ws[((size_t)blockIdx.x * 2 + 1) * a.C + c0 + i], acc[1][i]);
        }
    }
    if (!last_block(a.counter, a.nblk)) return;
    float* coef = a.ws + (size_t)a.nblk * 2 * a.C;  // [3][C]
    const double inv_m = 1.0 / (double)a.M;
    for (int cb = 0; cb < a.C; cb += NT) {
        const int nc = min(NT, a.C - cb);
        final_colsum<2>(a.ws, 2 * (size_t)a.C, 0, a.nblk, a.C, cb, nc, fin, scratch);
        if (t < nc) {
            const int c = cb + t;
            const double is = a.save_invstd[c];
            a.dbeta[c] = (float)fin[t];
            a.dgamma[c] = (float)(fin[nc + t] * is);
            coef[c] = a.gamma[c] * (float)is;
            coef[a.C + c] = (float)(fin[t] * inv_m);
            coef[2 * a.C + c] = (float)(fin[nc + t] * is * is * inv_m);
        }
        __syncthreads();
    }
}

// backward pass 2: dx = k1 * (dyr - k2 - (x - mean) * k3); dres = dyr
template <int VEC>
__global__ __launch_bounds__(NT) void k_bn_bwd_apply(BNArgs a) {
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    if (r >= a.TR) return;
    const int c0 = cg * VEC;
    const float* coef = a.ws + (size_t)a.nblk * 2 * a.C;
    const Vec<VEC> k1 = ld_f<VEC>(coef + c0), k2 = ld_f<VEC>(coef + a.C + c0), k3 = ld_f<VEC>(coef + 2 * a.C + c0);
    const Vec<VEC> mu = ld_f<VEC>(a.save_mean + c0);
    const int row0 = blockIdx.x * a.rpb, row1 = min(a.M, row0 + a.rpb);
    for (int row = row0 + r; row < row1; row += a.TR) {
        const size_t o = (size_t)row * a.C + c0;
        Vec<VEC> g = ld_bf<VEC>(a.dy + o);
        if (a.relu) {
            const Vec<VEC> y = ld_bf<VEC>(a.y + o);
#pragma unroll
            for (int i = 0; i < VEC; ++i) g.v[i] = y.v[i] > 0.0f ? g.v[i] : 0.0f;
        }
        if (a.dres) st_bf<VEC>(a.dres + o, g);
        const Vec<VEC> x = ld_bf<VEC>(a.x + o);
        Vec<VEC> d;
#pragma unroll
        for (int i = 0; i < VEC; ++i) d.v[i] = k1.v[i] * ((g.v[i] - k2.v[i]) - (x.v[i] - mu.v[i]) * k3.v[i]);
        st_bf<VEC>(a.out + o, d);
    }
}

// ------------------------------------------------------------------------------------------
// GroupNorm(G) of (x + bias) + ReLU, per sample n over rows [n*HW, (n+1)*HW)
// ------------------------------------------------------------------------------------------
struct GNArgs {
    const uint16_t* x;
    const void* bias;
    const uint16_t* dy;
    const uint16_t* y;
    const float* gamma;
    const float* beta;
    float* save_mean;    // [N*G]
    float* save_invstd;  // [N*G]
    uint16_t* out;
    void* dbias;
    float* dgamma;
    float* dbeta;
    float* ws;  // [N][bpn][K][C] partials, then coefficients
    int* counter;
    float eps;
    int N, HW, C, NG, relu, bias_bf16, G, TR, rpb, bpn;  // bpn: workgroups per sample
};

// forward pass 1: per (n, c) sum / sumsq of x+bias; last block -> per (n, g) mean / invstd and
// per (n, c) affine coefficients scale = gamma*invstd, shift = beta - mean*scale (bias folded:
// y = (x + bias)*scale + shift).
template <int VEC>
__global__ __launch_bounds__(NT) void k_gn_fwd_stats(GNArgs a) {
    __shared__ float red[2 * NT * VEC];
    __shared__ double fin[2 * NT];
    __shared__ double scratch[2 * NT];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    float acc[2][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = acc[1][i] = 0.0f;
    if (r < a.TR) {
        const Vec<VEC> b = ld_param<VEC>(a.bias, a.bias_bf16, c0);
        const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
        for (int row = row0 + r; row < row1; row += a.TR) {
            const Vec<VEC> v = ld_bf<VEC>(a.x + ((size_t)n * a.HW + row) * a.C + c0);
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const float u = v.v[i] + b.v[i];
                acc[0][i] += u;
                acc[1][i] += u * u;
            }
        }
    }
    block_colsum<VEC, 2>(acc, red, a.G, a.TR);
    if (r == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            st_part(&a.ws[((size_t)blockIdx.x * 2 + 0) * a.C + c0 + i], acc[0][i]);
            st_part(&a.ws[((size_t)blockIdx.x * 2 + 1) * a.C + c0 + i], acc[1][i]);
        }
    }
    if (!last_block(a.counter, a.N * a.bpn)) return;
    // per (n, c) totals, then per group (fixed channel order)
    __shared__ double gsum[2 * NT];
    float* coef = a.ws + (size_t)a.N * a.bpn * 2 * a.C;  // [N][2][C]
    const int cpg = a.C / a.NG;
    const double inv_cnt = 1.0 / ((double)a.HW * cpg);
    for (int nn = 0; nn < a.N; ++nn) {
        for (int cb = 0; cb < a.C; cb += NT) {  // C <= NT for every PoseNet layer; general anyway
            const int nc = min(NT, a.C - cb);
            final_colsum<2>(a.ws, 2 * (size_t)a.C, nn * a.bpn, a.bpn, a.C, cb, nc, fin, scratch);
            if (t < nc) {
                gsum[t] = fin[t];
                gsum[NT + t] = fin[nc + t];
            }
            __syncthreads();
            if (t < nc) {
                const int c = cb + t, g = c / cpg;
                const int first = g * cpg - cb;  // groups never straddle a chunk: NT % cpg == 0
                double s = 0.0, q = 0.0;
                for (int u = 0; u < cpg; ++u) {
                    s += gsum[first + u];
                    q += gsum[NT + first + u];
                }
                const double mean = s * inv_cnt;
                const double var = fmax(q * inv_cnt - mean * mean, 0.0);
                const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
                if (c % cpg == 0) {
                    a.save_mean[nn * a.NG + g] = (float)mean;
                    a.save_invstd[nn * a.NG + g] = invstd;
                }
                const float scale = a.gamma[c] * invstd;
                coef[((size_t)nn * 2 + 0) * a.C + c] = scale;
                coef[((size_t)nn * 2 + 1) * a.C + c] = a.beta[c] - (float)mean * scale;
            }
            __syncthreads();
        }
    }
}

template <int VEC>
__global__ __launch_bounds__(NT) void k_gn_fwd_apply(GNArgs a) {
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    if (r >= a.TR) return;
    const int c0 = cg * VEC;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const float* coef = a.ws + (size_t)a.N * a.bpn * 2 * a.C + (size_t)n * 2 * a.C;
    const Vec<VEC> sc = ld_f<VEC>(coef + c0), sh = ld_f<VEC>(coef + a.C + c0);
    const Vec<VEC> b = ld_param<VEC>(a.bias, a.bias_bf16, c0);
    const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
    for (int row = row0 + r; row < row1; row += a.TR) {
        const size_t o = ((size_t)n * a.HW + row) * a.C + c0;
        Vec<VEC> v = ld_bf<VEC>(a.x + o);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            v.v[i] = (v.v[i] + b.v[i]) * sc.v[i] + sh.v[i];
            if (a.relu) v.v[i] = fmaxf(v.v[i], 0.0f);
        }
        st_bf<VEC>(a.out + o, v);
    }
}

// backward pass 1: per (n, c): S1 = sum dyr, S2 = sum dyr*xhat.  Last block: dbeta[c] = sum_n
// S1, dgamma[c] = sum_n S2, per (n, g): A = sum_{c in g} gamma S1, Bq = sum_{c in g} gamma S2;
// dx = invstd (gamma dyr - A/cnt - xhat Bq/cnt) (coefficients for pass 2).
template <int VEC>
__global__ __launch_bounds__(NT) void k_gn_bwd_stats(GNArgs a) {
    __shared__ float red[2 * NT * VEC];
    __shared__ double fin[2 * NT];
    __shared__ double scratch[2 * NT];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const int cpg = a.C / a.NG;
    float acc[2][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = acc[1][i] = 0.0f;
    if (r < a.TR) {
        const Vec<VEC> b = ld_param<VEC>(a.bias, a.bias_bf16, c0);
        float mu[VEC], is[VEC];
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            mu[i] = a.save_mean[n * a.NG + (c0 + i) / cpg];
            is[i] = a.save_invstd[n * a.NG + (c0 + i) / cpg];
        }
        const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
        for (int row = row0 + r; row < row1; row += a.TR) {
            const size_t o = ((size_t)n * a.HW + row) * a.C + c0;
            Vec<VEC> g = ld_bf<VEC>(a.dy + o);
            if (a.relu) {
                const Vec<VEC> y = ld_bf<VEC>(a.y + o);
#pragma unroll
                for (int i = 0; i < VEC; ++i) g.v[i] = y.v[i] > 0.0f ? g.v[i] : 0.0f;
            }
            const Vec<VEC> x = ld_bf<VEC>(a.x + o);
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const float xh = (x.v[i] + b.v[i] - mu[i]) * is[i];
                acc[0][i] += g.v[i];
                acc[1][i] += g.v[i] * xh;
            }
        }
    }
    block_colsum<VEC, 2>(acc, red, a.G, a.TR);
    if (r == 0) {
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int i = 0; i < VEC; ++i) st_part(&a.ws[((size_t)blockIdx.x * 2 + k) * a.C + c0 + i], acc[k][i]);
    }
    if (!last_block(a.counter, a.N * a.bpn)) return;
    __shared__ double gs[2 * NT];
    float* coef = a.ws + (size_t)a.N * a.bpn * 2 * a.C;  // [N][3][C]: k1 = gamma*invstd, k2 = A/cnt*invstd, k3 = Bq/cnt*invstd
    const double cnt = (double)a.HW * cpg;
    for (int cb = 0; cb < a.C; cb += NT) {
        const int nc = min(NT, a.C - cb);
        double db = 0.0, dg = 0.0;
        for (int nn = 0; nn < a.N; ++nn) {
            final_colsum<2>(a.ws, 2 * (size_t)a.C, nn * a.bpn, a.bpn, a.C, cb, nc, fin, scratch);
            if (t < nc) {
                const float gam = a.gamma[cb + t];
                gs[t] = gam * fin[t];
                gs[NT + t] = gam * fin[nc + t];
            }
            __syncthreads();
            if (t < nc) {
                const int c = cb + t, g = c / cpg, first = g * cpg - cb;
                double A = 0.0, Bq = 0.0;
                for (int u = 0; u < cpg; ++u) {
                    A += gs[first + u];
                    Bq += gs[NT + first + u];
                }
                const double is = a.save_invstd[nn * a.NG + g];
                db += fin[t];
                dg += fin[nc + t];
                coef[((size_t)nn * 3 + 0) * a.C + c] = a.gamma[c] * (float)is;
                coef[((size_t)nn * 3 + 1) * a.C + c] = (float)(A / cnt * is);
                coef[((size_t)nn * 3 + 2) * a.C + c] = (float)(Bq / cnt * is);
            }
            __syncthreads();
        }
        if (t < nc) {
            a.dbeta[cb + t] = (float)db;
            a.dgamma[cb + t] = (float)dg;
        }
        __syncthreads();
    }
}

// backward pass 2: dx = k1*dyr - k2 - xhat*k3 with xhat = (x + bias - mean)*invstd, and the conv
// bias gradient as autograd forms it: the column sum of the stored (bf16) dx over n, hw.
template <int VEC>
__global__ __launch_bounds__(NT) void k_gn_bwd_apply(GNArgs a) {
    __shared__ float red[NT * VEC];
    __shared__ double fin[NT];
    __shared__ double scratch[NT];
    const int t = threadIdx.x, cg = t % a.G, r = t / a.G;
    const int c0 = cg * VEC;
    const int n = blockIdx.x / a.bpn, bl = blockIdx.x % a.bpn;
    const int cpg = a.C / a.NG;
    float acc[1][VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[0][i] = 0.0f;
    float* part = a.ws + (size_t)a.N * a.bpn * 2 * a.C + (size_t)a.N * 3 * a.C;  // [N*bpn][C]
    if (r < a.TR) {
        const float* coef = a.ws + (size_t)a.N * a.bpn * 2 * a.C + (size_t)n * 3 * a.C;
        const Vec<VEC> k1 = ld_f<VEC>(coef + c0), k2 = ld_f<VEC>(coef + a.C + c0), k3 = ld_f<VEC>(coef + 2 * a.C + c0);
        const Vec<VEC> b = ld_param<VEC>(a.bias, a.bias_bf16, c0);
        float mu[VEC], is[VEC];
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
            mu[i] = a.save_mean[n * a.NG + (c0 + i) / cpg];
            is[i] = a.save_invstd[n * a.NG + (c0 + i) / cpg];
        }
        const int row0 = bl * a.rpb, row1 = min(a.HW, row0 + a.rpb);
        for (int row = row0 + r; row < row1; row += a.TR) {
            const size_t o = ((size_t)n * a.HW + row) * a.C + c0;
            Vec<VEC> g = ld_bf<VEC>(a.dy + o);
            if (a.relu) {
                const Vec<VEC> y = ld_bf<VEC>(a.y + o);
#pragma unroll
                for (int i = 0; i < VEC; ++i) g.v[i] = y.v[i] > 0.0f ? g.v[i] : 0.0f;
            }
            const Vec<VEC> x = ld_bf<VEC>(a.x + o);
            Vec<VEC> d;
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
                const float xh = (x.v[i] + b.v[i] - mu[i]) * is[i];
                d.v[i] = k1.v[i] * g.v[i] - k2.v[i] - xh * k3.v[i];
            }
            st_bf<VEC>(a.out + o, d);
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[0][i] += bf2f(f2bf(d.v[i]));
        }
    }
    block_colsum<VEC, 1>(acc, red, a.G, a.TR);
    if (r == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) st_part(&part[(size_t)blockIdx.x * a.C + c0 + i], acc[0][i]);
    }
    if (!last_block(a.counter + 1, a.N * a.bpn)) return;
    for (int cb = 0; cb < a.C; cb += NT) {
        const int nc = min(NT, a.C - cb);
        final_colsum<1>(part, a.C, 0, a.N * a.bpn, a.C, cb, nc, fin, scratch);
        if (t < nc) {
            if (a.bias_bf16)
                static_cast<uint16_t*>(a.dbias)[cb + t] = f2bf((float)fin[t]);
            else
                static_cast<float*>(a.dbias)[cb + t] = (float)fin[t];
        }
        __syncthreads();
    }
}

template <typename A>
void set_geo(A& a, const Geo& g) {
    a.G = g.G;
    a.TR = g.TR;
    a.rpb = g.rpb;
}

}  // namespace

extern "C" {

size_t psfm_netops_ws_floats(int M, int C) {
    const Geo g = geometry(M, C, pick_vec(C), RED_BLOCKS, MIN_ITERS);
    return (size_t)g.nblk * 2 * C + 3 * (size_t)C;
}

size_t psfm_gn_ws_floats(int N, int HW, int C, int G) {
    (void)G;
    const Geo g = geometry(HW, C, pick_vec(C), std::max(1, RED_BLOCKS / std::max(N, 1)), MIN_ITERS);
    return (size_t)N * g.nblk * 2 * C + (size_t)N * 3 * C + (size_t)N * g.nblk * C;
}

int psfm_bias_act_fwd(const void* x, const void* bias, int bias_bf16, int M, int C, int act, void* y, void* stream) {
    if (!x || !bias || !y || M < 1 || C < 1) return fail(-1, "bias_act_fwd: bad arguments");
    const int vec = pick_vec(C);
    const Geo g = geometry(M, C, vec);
    if (vec == 1 && C > NT) return fail(-2, "bias_act_fwd: C must be a multiple of 8 or <= 256");
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
                      float* ws, int* counter, void* stream) {
    if (!dy || !y || !dx || !dbias || !ws || !counter || M < 1 || C < 1)
        return fail(-1, "bias_act_bwd: bad arguments");
    const int vec = pick_vec(C);
    if (vec == 1 && C > NT) return fail(-2, "bias_act_bwd: C must be a multiple of 8 or <= 256");
    const Geo g = geometry(M, C, vec, RED_BLOCKS, MIN_ITERS);
    BiasArgs a{};
    a.dy = dy;
    a.y = y;
    a.out = dx;
    a.dbias = dbias;
    a.ws = ws;
    a.counter = counter;
    a.M = M, a.C = C, a.act = act, a.bias_bf16 = bias_bf16, a.nblk = g.nblk;
    set_geo(a, g);
    if (vec == 8)
        hipLaunchKernelGGL(k_bias_act_bwd<8>, dim3(g.nblk), dim3(NT), 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(k_bias_act_bwd<1>, dim3(g.nblk), dim3(NT), 0, (hipStream_t)stream, a);
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_bn_act_fwd(const void* x, const void* res, const float* gamma, const float* beta, float* run_mean,
                    float* run_var, float momentum, float eps, int M, int C, int relu, void* y, float* save_mean,
                    float* save_invstd, float* ws, int* counter, void* stream) {
    if (!x || !gamma || !beta || !y || !save_mean || !save_invstd || !ws || !counter || M < 1 || C < 1)
        return fail(-1, "bn_act_fwd: bad arguments");
    if ((run_mean == nullptr) != (run_var == nullptr)) return fail(-1, "bn_act_fwd: running stats must pair");
    const int vec = pick_vec(C);
    if (vec == 1 && C > NT) return fail(-2, "bn_act_fwd: C must be a multiple of 8 or <= 256");
    const Geo g = geometry(M, C, vec, RED_BLOCKS, MIN_ITERS);
    BNArgs a{};
    a.x = static_cast<const uint16_t*>(x);
    a.res = static_cast<const uint16_t*>(res);
    a.gamma = gamma, a.beta = beta, a.run_mean = run_mean, a.run_var = run_var;
    a.save_mean = save_mean, a.save_invstd = save_invstd;
    a.out = static_cast<uint16_t*>(y);
    a.ws = ws, a.counter = counter, a.momentum = momentum, a.eps = eps;
    a.M = M, a.C = C, a.relu = relu, a.nblk = g.nblk;
    set_geo(a, g);
    hipStream_t st = (hipStream_t)stream;
    if (vec == 8) {
        hipLaunchKernelGGL(k_bn_fwd_stats<8>, dim3(g.nblk), dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_bn_fwd_apply<8>, dim3(g.nblk), dim3(NT), 0, st, a);
    } else {
        hipLaunchKernelGGL(k_bn_fwd_stats<1>, dim3(g.nblk), dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_bn_fwd_apply<1>, dim3(g.nblk), dim3(NT), 0, st, a);
    }
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_bn_act_bwd(const void* dy, const void* y, const void* x, const float* gamma, const float* save_mean,
                    const float* save_invstd, int M, int C, int relu, void* dx, void* dres, float* dgamma,
                    float* dbeta, float* ws, int* counter, void* stream) {
    if (!dy || !x || !gamma || !save_mean || !save_invstd || !dx || !dgamma || !dbeta || !ws || !counter ||
        M < 1 || C < 1 || (relu && !y))
        return fail(-1, "bn_act_bwd: bad arguments");
    const int vec = pick_vec(C);
    if (vec == 1 && C > NT) return fail(-2, "bn_act_bwd: C must be a multiple of 8 or <= 256");
    const Geo g = geometry(M, C, vec, RED_BLOCKS, MIN_ITERS);
    BNArgs a{};
    a.dy = static_cast<const uint16_t*>(dy);
    a.y = static_cast<const uint16_t*>(y);
    a.x = static_cast<const uint16_t*>(x);
    a.gamma = gamma, a.save_mean = const_cast<float*>(save_mean), a.save_invstd = const_cast<float*>(save_invstd);
    a.out = static_cast<uint16_t*>(dx);
    a.dres = static_cast<uint16_t*>(dres);
    a.dgamma = dgamma, a.dbeta = dbeta, a.ws = ws, a.counter = counter;
    a.M = M, a.C = C, a.relu = relu, a.nblk = g.nblk;
    set_geo(a, g);
    hipStream_t st = (hipStream_t)stream;
    if (vec == 8) {
        hipLaunchKernelGGL(k_bn_bwd_stats<8>, dim3(g.nblk), dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_bn_bwd_apply<8>, dim3(g.nblk), dim3(NT), 0, st, a);
    } else {
        hipLaunchKernelGGL(k_bn_bwd_stats<1>, dim3(g.nblk), dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_bn_bwd_apply<1>, dim3(g.nblk), dim3(NT), 0, st, a);
    }
    NETOPS_LAUNCH_CHECK();
    return 0;
}

static int gn_setup(GNArgs& a, int N, int HW, int C, int G, Geo& g, int& vec) {
    if (N < 1 || HW < 1 || C < 1 || G < 1 || C % G != 0) return fail(-1, "groupnorm: bad shape");
    vec = pick_vec(C);
    if (vec == 1 && C > NT) return fail(-2, "groupnorm: C must be a multiple of 8 or <= 256");
    if (C > NT && NT % (C / G) != 0) return fail(-2, "groupnorm: channels per group must divide 256");
    g = geometry(HW, C, vec, std::max(1, RED_BLOCKS / N), MIN_ITERS);
    a.N = N, a.HW = HW, a.C = C, a.NG = G, a.bpn = g.nblk;
    set_geo(a, g);
    return 0;
}

int psfm_gn_act_fwd(const void* x, const void* bias, int bias_bf16, const float* gamma, const float* beta, float eps,
                    int N, int HW, int C, int G, int relu, void* y, float* save_mean, float* save_invstd, float* ws,
                    int* counter, void* stream) {
    if (!x || !bias || !gamma || !beta || !y || !save_mean || !save_invstd || !ws || !counter)
        return fail(-1, "gn_act_fwd: bad arguments");
    GNArgs a{};
    Geo g;
    int vec;
    if (int e = gn_setup(a, N, HW, C, G, g, vec)) return e;
    a.x = static_cast<const uint16_t*>(x);
    a.bias = bias, a.bias_bf16 = bias_bf16, a.gamma = gamma, a.beta = beta, a.eps = eps;
    a.save_mean = save_mean, a.save_invstd = save_invstd;
    a.out = static_cast<uint16_t*>(y);
    a.ws = ws, a.counter = counter, a.relu = relu;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(N * g.nblk);
    if (vec == 8) {
        hipLaunchKernelGGL(k_gn_fwd_stats<8>, grid, dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_gn_fwd_apply<8>, grid, dim3(NT), 0, st, a);
    } else {
        hipLaunchKernelGGL(k_gn_fwd_stats<1>, grid, dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_gn_fwd_apply<1>, grid, dim3(NT), 0, st, a);
    }
    NETOPS_LAUNCH_CHECK();
    return 0;
}

int psfm_gn_act_bwd(const void* dy, const void* y, const void* x, const void* bias, int bias_bf16, const float* gamma,
                    const float* save_mean, const float* save_invstd, int N, int HW, int C, int G, int relu, void* dx,
                    void* dbias, float* dgamma, float* dbeta, float* ws, int* counter, void* stream) {
    if (!dy || !x || !bias || !gamma || !save_mean || !save_invstd || !dx || !dbias || !dgamma || !dbeta || !ws ||
        !counter || (relu && !y))
        return fail(-1, "gn_act_bwd: bad arguments");
    GNArgs a{};
    Geo g;
    int vec;
    if (int e = gn_setup(a, N, HW, C, G, g, vec)) return e;
    a.dy = static_cast<const uint16_t*>(dy);
    a.y = static_cast<const uint16_t*>(y);
    a.x = static_cast<const uint16_t*>(x);
    a.bias = bias, a.bias_bf16 = bias_bf16, a.gamma = gamma;
    a.save_mean = const_cast<float*>(save_mean), a.save_invstd = const_cast<float*>(save_invstd);
    a.out = static_cast<uint16_t*>(dx);
    a.dbias = dbias, a.dgamma = dgamma, a.dbeta = dbeta, a.ws = ws, a.counter = counter, a.relu = relu;
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid(N * g.nblk);
    if (vec == 8) {
        hipLaunchKernelGGL(k_gn_bwd_stats<8>, grid, dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_gn_bwd_apply<8>, grid, dim3(NT), 0, st, a);
    } else {
        hipLaunchKernelGGL(k_gn_bwd_stats<1>, grid, dim3(NT), 0, st, a);
        hipLaunchKernelGGL(k_gn_bwd_apply<1>, grid, dim3(NT), 0, st, a);
    }
    NETOPS_LAUNCH_CHECK();
    return 0;
}

const char* psfm_netops_last_error(void) { return g_err.c_str(); }

}  // extern "C"
