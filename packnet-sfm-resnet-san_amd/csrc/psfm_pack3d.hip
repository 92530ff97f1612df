// psfm_pack3d.hip — fused PackNet packing / unpacking 3-D convolution for MI355X (gfx950), behind
// include/psfm_pack3d.h.
//
// Reference: packnet_sfm/networks/layers/packnet/layers01.py:126-146 (packing), :189-223
// (PackLayerConv3d), :226-282 (UnpackLayerConv3d).  The Conv3d(1 -> d=8, 3x3x3, pad 1) is a small
// stencil (216 FMAs per voxel) whose output is 8x its input: it is HBM-bound on the write, so
// the kernels stream the volume through LDS tiles (with a 1-voxel halo in k, y, x), keep the 216
// weights in LDS ([tap][o]: two b128 broadcast reads per tap), and write every folded /
// pixel-shuffled output element exactly once, straight into the caller's layout (strides).
//   k_p3d_fwd      y  = conv3d(V)            4 x 16 pixels x 32 k per chunk, thread = pixel x 8 k
//                                            (d x 8 register outputs, 16-byte stores)
//   k_p3d_bwd_x_cl dV = conv3d^T(dy)         pack layers, channels_last dy: one 4 x 16 pixel x 16 k
//                                            chunk per workgroup (XCD-aware order), o in passes
//                                            of 4, thread = 4 pixels x a k pair (packed f32)
//   k_p3d_bwd_x_mfma dV = conv3d^T(dy)       bf16 channels_last, r = 2 (default for unpack layers):
//                                            channel mix on the matrix cores (9 shifts x (8 k, 2
//                                            pixels) x (dz, o, hi/lo weight)), fp32 shift-sum in LDS
//   k_p3d_bwd_x    dV = conv3d^T(dy)         any other layout: 4 x 8 pixels x 16 k
//   k_p3d_bwd_w    per-workgroup dw / db partials (thread = (spatial shift, pixel group), ND x 3
//                  register partials; 16-byte dy staging for channels_last pack layers), fixed-order
//                  fp64 reduce
// V is the virtual volume: pack = space-to-depth view of x (channel k = c r^2 + i r + j),
// unpack = x itself; the output channel o K + k is folded (pack) or pixel-shuffled (unpack).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "../../include/psfm_pack3d.h"
#include "psfm_knobs.h"

using namespace psfm;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

constexpr int NTH = 256;
typedef float f2 __attribute__((ext_vector_type(2)));   // packed f32 pair (v_pk_fma_f32)
constexpr int P3D_WAVES = 2;
#ifndef P3D_FWD_MFMA_DEFAULT
#define P3D_FWD_MFMA_DEFAULT 0   // 1: the matrix-core forward for d = 4 pack layers too
#endif
#ifndef P3D_DX_MFMA_DEFAULT
#define P3D_DX_MFMA_DEFAULT 0   // 1: dx of bf16 channels_last PACK layers on the matrix cores by default too
#endif
#ifndef MFMA_DW
#define MFMA_DW 1   // weight gradient of bf16 channels_last pack layers on the matrix cores
#endif
// ND: Conv3d output features d — 8 (PackNet01) or 4 (PackNetSAN01, num_3d_feat = 4)

struct P3 {
    int B, C, Hv, Wv, r, K, KG;  // K volume channels, KG channel groups (workgroups per pixel tile)
    int lin, gxn, gyn;           // lin: 1-D XCD-grouped grid over gxn x gyn tiles (wg_coords)
    int dy32;                    // every in-image element offset of dy fits int32 (host-checked)
    int64_t xs[4], ys[4];
    const void* x;
    const void* dy;
    void* y;
    void* dx;
    const float* w;
    const float* bias;
    float* ws;
};

// storage types: fp32, or bf16 as raw 16-bit words (round to nearest even, as torch does)
template <typename T>
__device__ __forceinline__ float ld(const void* p, int64_t i);
template <>
__device__ __forceinline__ float ld<float>(const void* p, int64_t i) {
    return static_cast<const float*>(p)[i];
}
template <>
__device__ __forceinline__ float ld<uint16_t>(const void* p, int64_t i) {
    return __uint_as_float((uint32_t)static_cast<const uint16_t*>(p)[i] << 16);
}
template <typename T>
__device__ __forceinline__ void st(void* p, int64_t i, float v);
template <>
__device__ __forceinline__ void st<float>(void* p, int64_t i, float v) {
    static_cast<float*>(p)[i] = v;
}
template <>
__device__ __forceinline__ void st<uint16_t>(void* p, int64_t i, float v) {
    uint32_t u = __float_as_uint(v);
    u += 0x7fffu + ((u >> 16) & 1u);  // RNE (finite values)
    static_cast<uint16_t*>(p)[i] = (uint16_t)(u >> 16);
}

template <typename T>
__device__ __forceinline__ float ldi(const T* p, int i);
template <>
__device__ __forceinline__ float ldi<float>(const float* p, int i) {
    return p[i];
}
template <>
__device__ __forceinline__ float ldi<uint16_t>(const uint16_t* p, int i) {
    return __uint_as_float((uint32_t)p[i] << 16);
}

// element offset of volume voxel (b, k, y, x) in x
template <int MODE>
__device__ __forceinline__ int64_t vaddr(const P3& a, int b, int k, int y, int x) {
    if (MODE == PSFM_P3D_PACK) {
        if (a.r == 2) {   // every PackNet layer (wave-uniform): shifts instead of integer divisions
            const int c = k >> 2, i = (k >> 1) & 1, j = k & 1;
            return b * a.xs[0] + c * a.xs[1] + (int64_t)(2 * y + i) * a.xs[2] + (int64_t)(2 * x + j) * a.xs[3];
        }
        const int rr = a.r * a.r, c = k / rr, q = k - c * rr, i = q / a.r, j = q - i * a.r;
        return b * a.xs[0] + c * a.xs[1] + (int64_t)(y * a.r + i) * a.xs[2] + (int64_t)(x * a.r + j) * a.xs[3];
    }
    return b * a.xs[0] + k * a.xs[1] + (int64_t)y * a.xs[2] + (int64_t)x * a.xs[3];
}
// element offset of output feature (b, o, k, y, x) in y (folded channel o K + k)
template <int MODE>
__device__ __forceinline__ int64_t yaddr(const P3& a, int b, int o, int k, int y, int x) {
    const int q = o * a.K + k;
    if (MODE == PSFM_P3D_PACK)
        return b * a.ys[0] + q * a.ys[1] + (int64_t)y * a.ys[2] + (int64_t)x * a.ys[3];
    if (a.r == 2) {
        const int c = q >> 2, i = (q >> 1) & 1, j = q & 1;
        return b * a.ys[0] + c * a.ys[1] + (int64_t)(2 * y + i) * a.ys[2] + (int64_t)(2 * x + j) * a.ys[3];
    }
    const int rr = a.r * a.r, c = q / rr, s = q - c * rr, i = s / a.r, j = s - i * a.r;
    return b * a.ys[0] + c * a.ys[1] + (int64_t)(y * a.r + i) * a.ys[2] + (int64_t)(x * a.r + j) * a.ys[3];
}

// (tile x, tile y, b * KG + kg) of this workgroup.  lin = 0: the 3-D grid.  lin = 1: a 1-D grid
// dealt round-robin to the 8 XCDs (workgroup w -> XCD w % 8); the logical index runs contiguously
// within each XCD with the channel group fastest, so the KG workgroups of one pixel tile run side
// by side on ONE XCD: the x lines they all read (each group uses 16-32 bytes of a pixel's 128-byte
// channels_last line) and the dy lines shared by neighbouring groups are fetched into that XCD's
// L2 once instead of once per group (profiles/r03/p3d: the 3-D grid fetched 7.6x / 3.2x the
// forward / weight-gradient operand bytes).
struct WG {
    int bx, by, bz;
};
__device__ __forceinline__ WG wg_coords(const P3& a) {
    if (!a.lin) return WG{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
    const int n = gridDim.x, w = blockIdx.x, q = n / 8, rm = n % 8, xcd = w % 8, idx = w / 8;
    const int L = xcd < rm ? xcd * (q + 1) + idx : rm * (q + 1) + (xcd - rm) * q + idx;
    const int kg = L % a.KG, rest = L / a.KG, nt = a.gxn * a.gyn, tile = rest % nt, b = rest / nt;
    return WG{tile % a.gxn, tile / a.gxn, b * a.KG + kg};
}

template <int ND>
__device__ __forceinline__ void load_weights(const P3& a, float* sw) {
    // sw[tap * 8 + o] = w[o][tap]; sw[216 + o] = bias[o]
    for (int i = threadIdx.x; i < 27 * ND; i += NTH) sw[i] = a.w[(i % ND) * 27 + i / ND];
    if (threadIdx.x < ND) sw[27 * ND + threadIdx.x] = a.bias ? a.bias[threadIdx.x] : 0.0f;
}

// --------------------------------------------------------------------------------------------
// forward: y[o, k, p] = bias[o] + sum_taps w[o, tap] V[k + dz - 1, p + (dy, dx) - 1].  Per 4 x 16
// pixel x 32 k chunk the V halo tile is staged in LDS; a thread owns one pixel and 8 consecutive k
// and keeps all d x 8 outputs in registers: per (dy, dx) one 10-channel V run (16-byte aligned LDS
// reads) serves the three dz and the 8 k (27 LDS reads per 27 x 8 x d FMAs), weights are LDS
// broadcasts.  Channels_last pack outputs (the folded channel o K + k innermost) are written as
// one 16-byte store of 8 bf16 (two of 4 fp32) per o; other layouts element by element.
template <typename T, int MODE, int ND>
__device__ __forceinline__ void fwd_body(const P3& a) {
    constexpr int TY = 4, TX = 16, DC = 32, LY = TY + 2, LX = TX + 2, LK = DC + 4;  // LK: 16-B rows
    constexpr int KB = 8;                                                          // k per thread
    __shared__ __attribute__((aligned(16))) float sv[LY * LX * LK];
    __shared__ __attribute__((aligned(16))) float sw[27 * ND + ND];
    load_weights<ND>(a, sw);
    const WG g = wg_coords(a);
    const int x0 = g.bx * TX, y0 = g.by * TY;
    const int b = g.bz / a.KG, kg = g.bz - b * a.KG;
    const int nch = (a.K + DC - 1) / DC, c_lo = kg * nch / a.KG, c_hi = (kg + 1) * nch / a.KG;
    const int kq = threadIdx.x % (DC / KB), p = threadIdx.x / (DC / KB), py = p / TX, px = p % TX;
    const int gy = y0 + py, gx = x0 + px;
    for (int ch = c_lo; ch < c_hi; ++ch) {
        const int k0 = ch * DC;
        __syncthreads();
        for (int e = threadIdx.x; e < LY * LX * LK; e += NTH) {
            const int kk = e % LK, rest = e / LK, xx = rest % LX, yy = rest / LX;
            const int gk = k0 - 1 + kk, gy2 = y0 - 1 + yy, gx2 = x0 - 1 + xx;
            const bool in = kk < DC + 2 && gk >= 0 && gk < a.K && gy2 >= 0 && gy2 < a.Hv && gx2 >= 0 && gx2 < a.Wv;
            sv[e] = in ? ld<T>(a.x, vaddr<MODE>(a, b, gk, gy2, gx2)) : 0.0f;
        }
        __syncthreads();
        const int kb = k0 + kq * KB;
        if (gy >= a.Hv || gx >= a.Wv || kb >= a.K) continue;
        float acc[ND][KB];
#pragma unroll
        for (int o = 0; o < ND; ++o)
#pragma unroll
            for (int j = 0; j < KB; ++j) acc[o][j] = sw[27 * ND + o];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                const float4* vr = reinterpret_cast<const float4*>(sv + ((py + dy) * LX + (px + dx)) * LK + kq * KB);
                float v[KB + 4];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const float4 q = vr[i];
                    v[4 * i] = q.x, v[4 * i + 1] = q.y, v[4 * i + 2] = q.z, v[4 * i + 3] = q.w;
                }
#pragma unroll
                for (int dz = 0; dz < 3; ++dz) {
                    const float4* w4 = reinterpret_cast<const float4*>(sw + ((dz * 3 + dy) * 3 + dx) * ND);
#pragma unroll
                    for (int h = 0; h < ND / 4; ++h) {
                        const float4 wv = w4[h];
                        const float wo[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int j = 0; j < KB; ++j) acc[4 * h + u][j] += wo[u] * v[j + dz];
                    }
                }
            }
        if (kb + KB <= a.K) {
#pragma unroll
            for (int o = 0; o < ND; ++o) {
                T* dst = static_cast<T*>(a.y) + yaddr<MODE>(a, b, o, kb, gy, gx);
                if constexpr (sizeof(T) == 2) {
                    uint32_t w[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        uint32_t lo = __float_as_uint(acc[o][2 * i]), hi = __float_as_uint(acc[o][2 * i + 1]);
                        lo += 0x7fffu + ((lo >> 16) & 1u);
                        hi += 0x7fffu + ((hi >> 16) & 1u);
                        w[i] = (lo >> 16) | (hi & 0xffff0000u);
                    }
                    *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
                } else {
                    reinterpret_cast<float4*>(dst)[0] = make_float4(acc[o][0], acc[o][1], acc[o][2], acc[o][3]);
                    reinterpret_cast<float4*>(dst)[1] = make_float4(acc[o][4], acc[o][5], acc[o][6], acc[o][7]);
                }
            }
        } else {
#pragma unroll
            for (int o = 0; o < ND; ++o)
#pragma unroll
                for (int j = 0; j < KB; ++j)
                    if (kb + j < a.K) st<T>(a.y, yaddr<MODE>(a, b, o, kb + j, gy, gx), acc[o][j]);
        }
    }
}

template <typename T, int MODE, int ND>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(P3D_WAVES))) void k_p3d_fwd(P3 a) {
    fwd_body<T, MODE, ND>(a);
}
// Forward of a PACK layer with channels_last x AND y (every PackNet encoder pack layer).  Same
// arithmetic per output as fwd_body (the same 27 fp32 FMAs per (o, k, pixel) in the same order),
// three changes measured against it (profiles/r03/p3d):
//  * staging by 16-byte loads: V[k = 4c + 2i + j, y, x] = x[b, 2y + i, 2x + j, c], so one (pixel,
//    i, j) gives 8 (bf16) / 4 (fp32) consecutive c of the chunk at once (fwd_body: one 2-byte load
//    and a 64-bit address per element); the chunk halo k0 - 1 / k0 + 32 is one element each;
//  * thread = (wave = 8-k group, lane = pixel): a 16-lane quarter of a b128 LDS read covers 16
//    consecutive pixels of one tile row, whose 144-byte (LK = 36) runs start on 16 distinct 4-bank
//    groups — conflict-free (fwd_body's (pixel, k-group) lanes hit 2-way conflicts);
//  * CPW chunks per workgroup, the next chunk's loads in flight (registers) during this one's FMAs.
template <typename T, int ND>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(ND == 8 ? 3 : 4))) void k_p3d_fwd_cl(P3 a) {
    constexpr int TY = 4, TX = 16, DC = 32, LY = TY + 2, LX = TX + 2, LK = DC + 4, KB = 8;
    constexpr int VEC = 16 / sizeof(T);               // channels c per 16-byte load
    constexpr int NQ = LY * LX * 4 * (8 / VEC);       // 16-byte loads per chunk: (pixel, i, j, c half)
    constexpr int NV = (NQ + NTH - 1) / NTH;
    static_assert(LY * LX * 2 <= NTH, "halo staging slots");
    __shared__ __attribute__((aligned(16))) float sv[LY * LX * LK];
    __shared__ __attribute__((aligned(16))) float sw[27 * ND + ND];
    load_weights<ND>(a, sw);
    const WG g = wg_coords(a);
    const int x0 = g.bx * TX, y0 = g.by * TY;
    const int b = g.bz / a.KG, kg = g.bz - b * a.KG;
    const int nch = a.K / DC, c_lo = kg * nch / a.KG, c_hi = (kg + 1) * nch / a.KG;
    const int t = threadIdx.x, kq = t >> 6, lane = t & 63, py = lane >> 4, px = lane & 15;
    const int gy = y0 + py, gx = x0 + px;
    const T* xv = static_cast<const T*>(a.x);
    // chunk-independent element offsets (int32, host-checked), computed once: a chunk adds c0;
    // invalid slots read offset 0 and are zeroed at the LDS store (selects here would wait)
    int vo[NV], ho;
    uint32_t vok = 0u;
    bool hok;
#pragma unroll
    for (int u = 0; u < NV; ++u) {   // e -> (pixel, i, j, half): c0 + VEC*half .. + VEC - 1
        const int e = t + u * NTH, hf = (8 / VEC == 2) ? (e & 1) : 0, ij = (8 / VEC == 2) ? ((e >> 1) & 3) : (e & 3);
        const int pix = (8 / VEC == 2) ? (e >> 3) : (e >> 2), xx = pix % LX, yy = pix / LX;
        const int gyy = y0 - 1 + yy, gxx = x0 - 1 + xx;
        const bool ok = e < NQ && gyy >= 0 && gyy < a.Hv && gxx >= 0 && gxx < a.Wv;
        vo[u] = ok ? (int)vaddr<PSFM_P3D_PACK>(a, b, 4 * VEC * hf + ij, gyy, gxx) : 0;
        vok |= ok ? 1u << u : 0u;
    }
    const int hi = t & 1;
    {   // kk = 0 <-> V[k0 - 1] = (c0 - 1, i = 1, j = 1); kk = 33 <-> V[k0 + 32] = (c0 + 8, i = 0, j = 0)
        const int pix = t >> 1, xx = pix % LX, yy = pix / LX, gyy = y0 - 1 + yy, gxx = x0 - 1 + xx;
        hok = t < LY * LX * 2 && gyy >= 0 && gyy < a.Hv && gxx >= 0 && gxx < a.Wv;
        ho = hok ? (int)vaddr<PSFM_P3D_PACK>(a, b, hi ? 32 : -1, gyy, gxx) : 0;   // + c0 per chunk
    }
    uint4 vq[NV];
    T hq;   // raw: converted in store() (a conversion here would wait for the loads)
    bool hin = false;
    auto load = [&](int ch) {
        const int c0 = ch * (DC / 4);
#pragma unroll
        for (int u = 0; u < NV; ++u) vq[u] = *reinterpret_cast<const uint4*>(xv + ((vok >> u) & 1u ? vo[u] + c0 : 0));
        hin = hok && (hi ? 4 * c0 + 32 < a.K : c0 > 0);
        hq = xv[hin ? ho + c0 : 0];
    };
    auto store = [&]() {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = t + u * NTH;
            if (e >= NQ) continue;
            const int hf = (8 / VEC == 2) ? (e & 1) : 0, ij = (8 / VEC == 2) ? ((e >> 1) & 3) : (e & 3);
            const int pix = (8 / VEC == 2) ? (e >> 3) : (e >> 2);
            float* row = sv + pix * LK + 1 + 4 * VEC * hf + ij;   // kk = 1 + 4 c' + ij
            const uint4 vv = (vok >> u) & 1u ? vq[u] : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
            if constexpr (sizeof(T) == 2) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    row[8 * q] = __uint_as_float(w[q] << 16);
                    row[8 * q + 4] = __uint_as_float(w[q] & 0xffff0000u);
                }
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) row[4 * q] = __uint_as_float(w[q]);
            }
        }
        if (t < LY * LX * 2) sv[(t >> 1) * LK + ((t & 1) ? DC + 1 : 0)] = hin ? ldi<T>(&hq, 0) : 0.0f;
    };
    T* ydst = static_cast<T*>(a.y) + (gy < a.Hv && gx < a.Wv ? yaddr<PSFM_P3D_PACK>(a, b, 0, 0, gy, gx) : 0);
    if (c_lo < c_hi) load(c_lo);
    for (int ch = c_lo; ch < c_hi; ++ch) {
        __syncthreads();   // the previous chunk's FMAs are done with the tile
        store();
        __syncthreads();
        if (ch + 1 < c_hi) load(ch + 1);
        if (gy >= a.Hv || gx >= a.Wv) continue;
        const int kb = ch * DC + kq * KB;
        float acc[ND][KB];
#pragma unroll
        for (int o = 0; o < ND; ++o)
#pragma unroll
            for (int j = 0; j < KB; ++j) acc[o][j] = sw[27 * ND + o];
#pragma unroll 1   // one shift at a time: the accumulators + 12 V values + 24 weights live (3-4 waves/SIMD)
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll 1
            for (int dx = 0; dx < 3; ++dx) {
                const float4* vr = reinterpret_cast<const float4*>(sv + ((py + dy) * LX + (px + dx)) * LK + kq * KB);
                float v[KB + 4];
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const float4 q = vr[i];
                    v[4 * i] = q.x, v[4 * i + 1] = q.y, v[4 * i + 2] = q.z, v[4 * i + 3] = q.w;
                }
#pragma unroll
                for (int dz = 0; dz < 3; ++dz) {
                    const float4* w4 = reinterpret_cast<const float4*>(sw + ((dz * 3 + dy) * 3 + dx) * ND);
#pragma unroll
                    for (int h = 0; h < ND / 4; ++h) {
                        const float4 wv = w4[h];
                        const float wo[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
                        for (int u = 0; u < 4; ++u)
#pragma unroll
                            for (int j = 0; j < KB; ++j) acc[4 * h + u][j] += wo[u] * v[j + dz];
                    }
                }
            }
#pragma unroll
        for (int o = 0; o < ND; ++o) {
            T* dst = ydst + o * a.K + kb;   // channels_last y: the folded channel o K + k is innermost
            if constexpr (sizeof(T) == 2) {
                uint32_t w[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t lo = __float_as_uint(acc[o][2 * i]), hi = __float_as_uint(acc[o][2 * i + 1]);
                    lo += 0x7fffu + ((lo >> 16) & 1u);
                    hi += 0x7fffu + ((hi >> 16) & 1u);
                    w[i] = (lo >> 16) | (hi & 0xffff0000u);
                }
                *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
            } else {
                reinterpret_cast<float4*>(dst)[0] = make_float4(acc[o][0], acc[o][1], acc[o][2], acc[o][3]);
                reinterpret_cast<float4*>(dst)[1] = make_float4(acc[o][4], acc[o][5], acc[o][6], acc[o][7]);
            }
        }
    }
}

// other layouts (unpack layers, NCHW): thread = (k, pixel), element stores through yaddr
template <typename T, int MODE, int ND>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(P3D_WAVES))) void k_p3d_fwd_generic(P3 a) {
    constexpr int TY = 4, TX = 16, DC = 32, LY = TY + 2, LX = TX + 2, LK = DC + 2;
    __shared__ float sv[LY * LX * LK];
    __shared__ __attribute__((aligned(16))) float sw[27 * ND + ND];
    load_weights<ND>(a, sw);
    const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
    const int b = blockIdx.z / a.KG, kg = blockIdx.z - b * a.KG;
    const int nch = (a.K + DC - 1) / DC, c_lo = kg * nch / a.KG, c_hi = (kg + 1) * nch / a.KG;
    const int dl = threadIdx.x % DC, pg = threadIdx.x / DC;
    for (int ch = c_lo; ch < c_hi; ++ch) {
        const int k0 = ch * DC;
        __syncthreads();
        for (int e = threadIdx.x; e < LY * LX * LK; e += NTH) {
            const int kk = e % LK, rest = e / LK, xx = rest % LX, yy = rest / LX;
            const int gk = k0 - 1 + kk, gy = y0 - 1 + yy, gx = x0 - 1 + xx;
            const bool in = gk >= 0 && gk < a.K && gy >= 0 && gy < a.Hv && gx >= 0 && gx < a.Wv;
            sv[e] = in ? ld<T>(a.x, vaddr<MODE>(a, b, gk, gy, gx)) : 0.0f;
        }
        __syncthreads();
        const int k = k0 + dl;
        if (k >= a.K) continue;
#pragma unroll 1
        for (int pp = 0; pp < (TY * TX) / (NTH / DC); ++pp) {
            const int p = pg + pp * (NTH / DC), py = p / TX, px = p % TX;
            const int gy = y0 + py, gx = x0 + px;
            if (gy >= a.Hv || gx >= a.Wv) continue;
            float acc[ND];
#pragma unroll
            for (int o = 0; o < ND; ++o) acc[o] = sw[27 * ND + o];
#pragma unroll 1  // the 216 weights of d = 8 fully unrolled would not fit 256 VGPRs
            for (int dz = 0; dz < 3; ++dz)
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const float v = sv[((py + dy) * LX + (px + dx)) * LK + dl + dz];
                        const float4* w4 = reinterpret_cast<const float4*>(sw + ((dz * 3 + dy) * 3 + dx) * ND);
#pragma unroll
                        for (int h = 0; h < ND / 4; ++h) {
                            const float4 wv = w4[h];
                            acc[4 * h + 0] += wv.x * v; acc[4 * h + 1] += wv.y * v;
                            acc[4 * h + 2] += wv.z * v; acc[4 * h + 3] += wv.w * v;
                        }
                    }
#pragma unroll
            for (int o = 0; o < ND; ++o) st<T>(a.y, yaddr<MODE>(a, b, o, k, gy, gx), acc[o]);
        }
    }
}



// --------------------------------------------------------------------------------------------
// dV[k, y, x] = sum_o sum_taps w[o, dz, dy, dx] dy[o, k - dz + 1, y - dy + 1, x - dx + 1]
template <typename T, int MODE, int ND>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(P3D_WAVES))) void k_p3d_bwd_x(P3 a) {
    constexpr int TY = 4, TX = 8, DC = 16, LY = TY + 2, LX = TX + 2, LK = DC + 2;
    __shared__ float sg[LY * LX * ND * LK];  // [yy][xx][o][kk]
    __shared__ __attribute__((aligned(16))) float sw[27 * ND + ND];
    load_weights<ND>(a, sw);
    const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
    const int b = blockIdx.z / a.KG, kg = blockIdx.z - b * a.KG;
    const int nch = (a.K + DC - 1) / DC, c_lo = kg * nch / a.KG, c_hi = (kg + 1) * nch / a.KG;
    const int dl = threadIdx.x % DC, pg = threadIdx.x / DC;
    for (int ch = c_lo; ch < c_hi; ++ch) {
        const int k0 = ch * DC;
        __syncthreads();
        for (int e = threadIdx.x; e < LY * LX * ND * LK; e += NTH) {
            const int kk = e % LK, r1 = e / LK, o = r1 % ND, r2 = r1 / ND, xx = r2 % LX, yy = r2 / LX;
            const int gk = k0 - 1 + kk, gy = y0 - 1 + yy, gx = x0 - 1 + xx;
            const bool in = gk >= 0 && gk < a.K && gy >= 0 && gy < a.Hv && gx >= 0 && gx < a.Wv;
            sg[e] = in ? ld<T>(a.dy, yaddr<MODE>(a, b, o, gk, gy, gx)) : 0.0f;
        }
        __syncthreads();
        const int k = k0 + dl;
        if (k >= a.K) continue;
#pragma unroll 1
        for (int pp = 0; pp < (TY * TX) / (NTH / DC); ++pp) {
            const int p = pg + pp * (NTH / DC), py = p / TX, px = p % TX;
            const int gy = y0 + py, gx = x0 + px;
            if (gy >= a.Hv || gx >= a.Wv) continue;
            float acc = 0.0f;
#pragma unroll 1  // d = 8: the fully unrolled weights would spill
            for (int dz = 0; dz < 3; ++dz)
#pragma unroll
                for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const float* g = sg + (((py + 2 - dy) * LX + (px + 2 - dx)) * ND) * LK + dl + 2 - dz;
                        const float4* w4 = reinterpret_cast<const float4*>(sw + ((dz * 3 + dy) * 3 + dx) * ND);
#pragma unroll
                        for (int h = 0; h < ND / 4; ++h) {
                            const float4 wv = w4[h];
                            acc += wv.x * g[(4 * h + 0) * LK] + wv.y * g[(4 * h + 1) * LK] +
                                   wv.z * g[(4 * h + 2) * LK] + wv.w * g[(4 * h + 3) * LK];
                        }
                    }
            st<T>(a.dx, vaddr<MODE>(a, b, k, gy, gx), acc);
        }
    }
}

// dV of a channels_last pack layer, k-pair form: 128 threads, thread = 4 neighbouring pixels x TWO
// consecutive k of a 4 x 16 pixel x 16 k chunk, both k in the halves of packed f32 pairs.  The
// per-(pixel, o) run is stored from k0-1 (index 0) so that the four values (k-1, k, k+1, k+2) a
// thread needs per pixel column are two aligned 8-byte LDS reads: (k-1, k) and (k+1, k+2) are the
// dz = 2 and dz = 0 operand pairs, (k, k+1) the dz = 1 pair — 12 ds_read_b64 feed 36 v_pk_fma_f32
// (72 MACs) per (o, dy) where the one-k form spent 18 ds_read_b32 on 36 MACs.
// One 16-k chunk per workgroup on an XCD-aware 1-D grid: a 128-byte line of a (pixel, o) dy run
// holds 64 k = four chunks, and the four workgroups that read it run back to back on ONE XCD (the
// grid's workgroup w goes to XCD w % 8; logical index = w's rank within its XCD, chunk fastest),
// so the line is fetched into that XCD's L2 once instead of once per chunk.
template <typename T, int ND>
__global__ __launch_bounds__(128, 2) void k_p3d_bwd_x_cl(P3 a, int gxn, int gyn) {
    constexpr int NT2 = 128, TY = 4, TX = 16, DC = 16, LY = TY + 2, LX = TX + 2;
    constexpr int OP = ND < 4 ? ND : 4;   // o per staging pass: 36 KB of LDS, 4 workgroups per CU
    constexpr int OS = 20;                // per-o run: index 0 = k0-1, 1..16 = k0..k0+15, 17 = k0+16
    constexpr int PS = OP * OS + 4;       // per-pixel stride (even: 8-byte aligned pairs)
    constexpr int VEC = 16 / sizeof(T);
    constexpr int UNITS = LY * LX * OP;
    constexpr int ITER = (UNITS + NT2 - 1) / NT2;
    static_assert(ND % OP == 0, "o passes");
    __shared__ __attribute__((aligned(16))) float sg[LY * LX * PS];
    const int nch = a.K / DC;
    int L;
    {
        const int n = gridDim.x, w = blockIdx.x, q = n / 8, rm = n % 8, xcd = w % 8, idx = w / 8;
        L = xcd < rm ? xcd * (q + 1) + idx : rm * (q + 1) + (xcd - rm) * q + idx;
    }
    const int k0 = (L % nch) * DC;
    const int rest = L / nch, tile = rest % (gxn * gyn), b = rest / (gxn * gyn);
    const int x0 = (tile % gxn) * TX, y0 = (tile / gxn) * TY;
    const int t = threadIdx.x, kp = t % 8, r = t / 8, py = r / 4, px0 = (r % 4) * 4;
    const T* dyb = static_cast<const T*>(a.dy) + b * a.ys[0];
    const int ys2 = (int)a.ys[2], ys3 = (int)a.ys[3];
    f2 acc[4] = {f2{0.0f, 0.0f}, f2{0.0f, 0.0f}, f2{0.0f, 0.0f}, f2{0.0f, 0.0f}};
    // the next o pass's dy runs are loaded into registers while this pass computes (raw words:
    // any conversion here would make the loads complete before the compute starts)
    uint4 v[ITER][DC / VEC];
    T e0[ITER], e1[ITER];
    auto load = [&](int o0) {
#pragma unroll
        for (int i = 0; i < ITER; ++i) {
            const int u = t + i * NT2;
            const int yy = u / (LX * OP), rem = u - yy * (LX * OP), xx = rem / OP, o = o0 + rem - xx * OP;
            const int gy = y0 - 1 + yy, gx = x0 - 1 + xx;
            const bool in = u < UNITS && (unsigned)gy < (unsigned)a.Hv && (unsigned)gx < (unsigned)a.Wv;
            const T* src = dyb + (in ? gy * ys2 + gx * ys3 + o * a.K + k0 : 0);
#pragma unroll
            for (int j = 0; j < DC / VEC; ++j)
                v[i][j] = in ? reinterpret_cast<const uint4*>(src)[j] : make_uint4(0, 0, 0, 0);
            e0[i] = in && k0 > 0 ? src[-1] : (T)0;
            e1[i] = in && k0 + DC < a.K ? src[DC] : (T)0;
        }
    };
    load(0);
    for (int o0 = 0; o0 < ND; o0 += OP) {
        __syncthreads();   // the previous pass's reads of sg are done
#pragma unroll
        for (int i = 0; i < ITER; ++i) {
            const int u = t + i * NT2;
            if (u >= UNITS) break;
            const int yy = u / (LX * OP), rem = u - yy * (LX * OP), xx = rem / OP, o = rem - xx * OP;
            float2* d2 = reinterpret_cast<float2*>(sg + (yy * LX + xx) * PS + o * OS);
            float f[DC];
#pragma unroll
            for (int j = 0; j < DC / VEC; ++j) {
                const uint32_t w4[4] = {v[i][j].x, v[i][j].y, v[i][j].z, v[i][j].w};
                if (sizeof(T) == 2) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        f[j * 8 + 2 * q] = __uint_as_float(w4[q] << 16);
                        f[j * 8 + 2 * q + 1] = __uint_as_float(w4[q] & 0xffff0000u);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) f[j * 4 + q] = __uint_as_float(w4[q]);
                }
            }
            d2[0] = make_float2(ldi<T>(&e0[i], 0), f[0]);
#pragma unroll
            for (int j = 1; j < DC / 2; ++j) d2[j] = make_float2(f[2 * j - 1], f[2 * j]);
            d2[DC / 2] = make_float2(f[DC - 1], ldi<T>(&e1[i], 0));
        }
        __syncthreads();
        if (o0 + OP < ND) load(o0 + OP);
#pragma unroll 1
        for (int o = 0; o < OP; ++o)
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const float* g = sg + ((py + 2 - dy) * LX + px0) * PS + o * OS + 2 * kp;
                f2 pa[6], pb[6], pm[6];   // (k-1, k), (k+1, k+2), (k, k+1) per pixel column
#pragma unroll
                for (int j = 0; j < 6; ++j) {
                    const float2 lo = *reinterpret_cast<const float2*>(g + j * PS);
                    const float2 hi = *reinterpret_cast<const float2*>(g + j * PS + 2);
                    pa[j] = f2{lo.x, lo.y};
                    pb[j] = f2{hi.x, hi.y};
                    pm[j] = f2{lo.y, hi.x};
                }
#pragma unroll
                for (int dz = 0; dz < 3; ++dz) {
                    const float* w = a.w + (o0 + o) * 27 + (dz * 3 + dy) * 3;
                    const f2 w0 = f2{w[0], w[0]}, w1 = f2{w[1], w[1]}, w2 = f2{w[2], w[2]};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const f2 c0 = dz == 0 ? pb[q + 2] : dz == 1 ? pm[q + 2] : pa[q + 2];
                        const f2 c1 = dz == 0 ? pb[q + 1] : dz == 1 ? pm[q + 1] : pa[q + 1];
                        const f2 c2 = dz == 0 ? pb[q] : dz == 1 ? pm[q] : pa[q];
                        // one fused multiply-add chain per pair (3 v_pk_fma_f32; the sum-then-add
                        // form took 4 packed ops per 3 MAC pairs)
                        acc[q] = w0 * c0 + acc[q];
                        acc[q] = w1 * c1 + acc[q];
                        acc[q] = w2 * c2 + acc[q];
                    }
                }
            }
    }
    const int k = k0 + 2 * kp, gy = y0 + py;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int gx = x0 + px0 + q;
        if (gy < a.Hv && gx < a.Wv) {
            st<T>(a.dx, vaddr<PSFM_P3D_PACK>(a, b, k, gy, gx), acc[q].x);
            st<T>(a.dx, vaddr<PSFM_P3D_PACK>(a, b, k + 1, gy, gx), acc[q].y);
        }
    }
}

// --------------------------------------------------------------------------------------------
// forward on the matrix cores (bf16, r = 2, channels_last x, K % 32 == 0; pack outputs channels_last,
// unpack outputs pixel-shuffled): y[o, k, p] = bias[o] + sum_{s, dz} w[o, dz, s] V[k + dz - 1, p + s].
// One group = 16 consecutive k of one pixel: A = the im2col rows (row m = k0 + 16 g + m, contraction
// (s, dz') = 4 s + dz' with dz' = 3 a zero slot: 36 of two v_mfma_f32_16x16x32_bf16's 64), B = the
// weights, column n = (o, hi / lo bf16 part): the hi and lo columns of o sit 8 lanes apart and are
// summed after the MFMAs with one DPP row rotate (w = hi + lo to 16 mantissa bits, products of bf16
// values exact in fp32).  A lane's 4 contraction values of one shift are V[k-1 .. k+2] of one
// pixel: the V tile is staged twice in LDS, the second copy one element later, so every lane reads
// its 4 values from a 4-byte aligned pair of dwords (the copy picked by the parity of its row).
// Workgroup = 4 x 16 pixel tile (wave w: tile row w) x 32-k chunks (the dW kernel's XCD-grouped
// grid and V staging); per wave and chunk 32 groups.  C rows = 4 consecutive k of one o: pack
// outputs are one 8-byte store per lane (channel o K + k innermost), unpack outputs four 2-byte
// stores (the 4 k are the 4 sub-pixels of one output channel).
template <int ND, int MODE>
__global__ __launch_bounds__(NTH) void k_p3d_fwd_mfma(P3 a) {
    constexpr bool PK = MODE == PSFM_P3D_PACK;
    constexpr int TY = 4, TX = 16, DC = 32, LY = TY + 2, LX = TX + 2, LKP = 40;
    constexpr int ROWS = LX * LKP + 56;
    typedef short bf8 __attribute__((ext_vector_type(8)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint16_t sv[2][LY * ROWS];
    const WG g = wg_coords(a);
    const int x0 = g.bx * TX, y0 = g.by * TY;
    const int b = g.bz / a.KG, kg = g.bz - b * a.KG;
    const int nch = a.K / DC, c_lo = kg * nch / a.KG, c_hi = (kg + 1) * nch / a.KG;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, m = lane & 15, j = lane >> 4;
    const uint16_t* xv = static_cast<const uint16_t*>(a.x);
    // B fragments: column n = (o, part), contraction block j of MFMA c: shifts s = 8 c + 2 j + h
    // (h = 0, 1), elements 4 h + dz'
    const int o = ND == 8 ? (m & 7) : (m & 3), part = m >> 3;
    const bool ocol = ND == 8 || (m & 7) < 4;
    bf8 Bw[2];
    float bias_o = 0.0f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        uint32_t wd[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t hv[2];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int el = 2 * q + hh, h = el >> 2, dz = el & 3, s = 8 * c + 2 * j + h;
                const bool live = ocol && dz < 3 && s < 9;
                const float wf = live ? a.w[o * 27 + dz * 9 + s] : 0.0f;
                const uint32_t u = __float_as_uint(wf);
                const uint32_t hib = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
                const float lof = wf - __uint_as_float(hib << 16);
                const uint32_t ul = __float_as_uint(lof);
                const uint32_t lob = (ul + 0x7fffu + ((ul >> 16) & 1u)) >> 16;
                hv[hh] = part ? lob : hib;
            }
            wd[q] = hv[0] | (hv[1] << 16);
        }
        Bw[c] = __builtin_bit_cast(bf8, make_uint4(wd[0], wd[1], wd[2], wd[3]));
    }
    if (a.bias && ocol) bias_o = a.bias[o];
    // V staging (as k_p3d_bwd_w_mfma): (pixel, quarter) units of 8 channels, chunk-independent
    // int32 offsets, the chunk halo k0 - 1 / k0 + 32 one element each
    constexpr int NV = (LY * LX * 4 + NTH - 1) / NTH;
    int vo[NV], ho;
    uint32_t vok = 0u;
    bool hok;
#pragma unroll
    for (int u = 0; u < NV; ++u) {
        const int e = t + u * NTH, ij = e & 3, pix = e >> 2, xx = pix % LX, yy = pix / LX;
        const int gyy = y0 - 1 + yy, gxx = x0 - 1 + xx;
        const bool ok = e < LY * LX * 4 && gyy >= 0 && gyy < a.Hv && gxx >= 0 && gxx < a.Wv;
        vo[u] = ok ? (int)vaddr<MODE>(a, b, PK ? ij : 8 * ij, gyy, gxx) : 0;
        vok |= ok ? 1u << u : 0u;
    }
    const int hi = t & 1;
    {
        const int pix = t >> 1, xx = pix % LX, yy = pix / LX, gyy = y0 - 1 + yy, gxx = x0 - 1 + xx;
        hok = t < LY * LX * 2 && gyy >= 0 && gyy < a.Hv && gxx >= 0 && gxx < a.Wv;
        ho = hok ? (int)vaddr<MODE>(a, b, hi ? 32 : -1, gyy, gxx) : 0;
    }
    uint4 vq[NV];
    uint16_t hq;
    bool hin = false;
    auto load = [&](int ch) {
        const int k0 = ch * DC, c0 = PK ? k0 >> 2 : k0;
#pragma unroll
        for (int u = 0; u < NV; ++u) vq[u] = *reinterpret_cast<const uint4*>(xv + ((vok >> u) & 1u ? vo[u] + c0 : 0));
        hin = hok && (hi ? k0 + 32 < a.K : k0 > 0);
        hq = xv[hin ? ho + c0 : 0];
    };
    auto store = [&]() {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = t + u * NTH, ij = e & 3, pix = e >> 2;
            if (e >= LY * LX * 4) continue;
            const uint4 vv = (vok >> u) & 1u ? vq[u] : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
            const int base = (pix / LX) * ROWS + (pix % LX) * LKP + 1 + (PK ? 2 * (ij >> 1) + (ij & 1) : 8 * ij);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e0 = base + (PK ? 8 * q : 2 * q), e1 = base + (PK ? 8 * q + 4 : 2 * q + 1);
                sv[0][e0] = sv[1][e0 + 1] = (uint16_t)(w[q] & 0xffffu);
                sv[0][e1] = sv[1][e1 + 1] = (uint16_t)(w[q] >> 16);
            }
        }
        if (t < LY * LX * 2) {
            const int e = ((t >> 1) / LX) * ROWS + ((t >> 1) % LX) * LKP + ((t & 1) ? 33 : 0);
            sv[0][e] = sv[1][e + 1] = hin ? hq : (uint16_t)0;
        }
    };
    // A geometry: row m -> element kk = 16 gk + m of the pixel's run is V[k - 1]; copy (m & 1)
    // holds it at an even index (4-byte aligned dword pair)
    const int cp = m & 1;
    const uint16_t* va = sv[cp] + cp + m;
    int soff[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int s = min(8 * c + 2 * j + h, 8);
            soff[c][h] = (s / 3) * ROWS + (s % 3) * LKP;
        }
    const bool a1live = j == 0;   // MFMA 1: only block 0 (s = 8, h = 0) carries taps
    if (c_lo < c_hi) load(c_lo);
    for (int ch = c_lo; ch < c_hi; ++ch) {
        __syncthreads();   // the previous chunk's reads of sv are done
        store();
        __syncthreads();
        if (ch + 1 < c_hi) load(ch + 1);
        const int k0 = ch * DC;
        const int gy = y0 + wv;
#pragma unroll 2
        for (int grp = 0; grp < 2 * TX; ++grp) {
            const int px = grp >> 1, gk = grp & 1;
            const uint16_t* vp = va + wv * ROWS + px * LKP + 16 * gk;
            uint32_t aw[2][4];
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t* src = reinterpret_cast<const uint32_t*>(vp + soff[c][h]);
                    aw[c][2 * h] = src[0];
                    aw[c][2 * h + 1] = src[1] & 0xffffu;   // V[k+2] sits in the zero-weight slot: masked
                }
            f4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, make_uint4(aw[0][0], aw[0][1], aw[0][2], aw[0][3])),
                                                         Bw[0], acc, 0, 0, 0);
            const uint4 a1 = a1live ? make_uint4(aw[1][0], aw[1][1], 0u, 0u) : make_uint4(0u, 0u, 0u, 0u);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, a1), Bw[1], acc, 0, 0, 0);
            // column n + 8 (lo part of o) -> lane n: DPP row rotate by 8
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float lo = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(acc[r]), 0x128, 0xf, 0xf, false));
                v[r] = (acc[r] + lo) + bias_o;
            }
            const int gx = x0 + px;
            if (part == 0 && ocol && gy < a.Hv && gx < a.Wv) {
                const int k = k0 + 16 * gk + 4 * j;   // rows 4 j .. 4 j + 3
                uint32_t u[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const uint32_t x = __float_as_uint(v[r]);
                    u[r] = (x + 0x7fffu + ((x >> 16) & 1u)) >> 16;
                }
                uint16_t* y = static_cast<uint16_t*>(a.y);
                if constexpr (PK) {   // channels o K + k .. + 3 of pixel (gy, gx): 8 bytes (host-checked)
                    *reinterpret_cast<uint2*>(y + yaddr<MODE>(a, b, o, k, gy, gx)) = make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
                } else {              // channel (o K + k) / 4 at the 4 sub-pixels
                    const int64_t base = yaddr<MODE>(a, b, o, k, gy, gx);   // sub-pixel (0, 0)
                    y[base] = (uint16_t)u[0];
                    y[base + a.ys[3]] = (uint16_t)u[1];
                    y[base + a.ys[2]] = (uint16_t)u[2];
                    y[base + a.ys[2] + a.ys[3]] = (uint16_t)u[3];
                }
            }
        }
    }
}

// --------------------------------------------------------------------------------------------
// dV of a bf16 channels_last pack layer (r = 2) on the matrix cores.  The transposed stencil splits
// into a channel mix and a spatial shift-sum:
//   G_s[k, p'] = sum_{o, dz} w[o, dz, s] dy[o, k - dz + 1, p']          (s = (ty, tx), 9 shifts)
//   dV[k, y, x] = sum_s G_s[k, y - ty + 1, x - tx + 1]
// The mix is one v_mfma_f32_16x16x32_bf16 product per (halo pixel pair x 8 k): rows = the 9 shifts
// (A = weights), columns = (8 k, 2 pixels), contraction = (dz, o) with every weight split into
// bf16 hi + lo parts (w = hi + lo to 16 mantissa bits; dy is bf16, so each product is exact in
// fp32): d = 4 is 3 dz x 4 o x 2 parts = 24 of one MFMA's 32, d = 8 48 of two MFMAs' 64.  G goes
// to LDS in fp32 and each thread sums its 9 shifted values for two channels of one input
// sub-pixel (one 4-byte bf16 pair store: k and k + 4 are channels c, c + 1 at the same (i, j)).
// Workgroup = 4 x 16 pixels, CPW consecutive 8-k chunks, 256 threads; the dy halo tile is staged
// as sd[pixel][k''][o] (o fastest: a B fragment's 8 contraction values are one 16- (d = 8) or
// 8-byte (d = 4) read), transposed from the (pixel, o) 16-byte runs of channels_last dy.  The next
// chunk's runs are loaded into registers while this chunk's mix and shift-sum run (offsets
// computed once, loads unconditional — out-of-image units read offset 0 — and the validity
// select at the LDS store, so no select makes the prefetch complete early).  XCD-aware 1-D grid
// with the chunk group fastest, as k_p3d_bwd_x_cl: the workgroups sharing a 128-byte dy line run
// back to back on one XCD.
// GRP (pack layers, CPW = 4): the group's four chunks are loaded at once, lane = (pixel, o pair,
// chunk) with the chunk fastest — four lanes read one contiguous 64-byte piece of each (pixel, o)
// dy line instead of four lanes touching four lines (the per-lane line accesses of the chunk-wise
// staging bound it: 0.85-1.0 ms vs the VALU kernel's 0.54 on the first PackNet01 layer); a chunk's
// k0-1 / k0+8 halo elements come from the neighbouring chunks' registers, only the group's two
// ends are extra 2-byte loads.
template <int ND, int CPW, int MODE, bool GRP = false>
__global__ __launch_bounds__(256) void k_p3d_bwd_x_mfma(P3 a, int gxn, int gyn) {
    constexpr int TY = 4, TX = 16, DC = 8, LY = TY + 2, LX = TX + 2, NPIX = LY * LX, LKK = DC + 2;
    constexpr int GS = NPIX * DC + 4;   // per-shift stride of the G tile (floats): 4 GS = 16 mod 64 banks
    constexpr int NPAIR = ND / 2, UNITS = NPIX * NPAIR * (GRP ? CPW : 1), ITER = (UNITS + 255) / 256;
    static_assert(!GRP || (CPW == 4 && MODE == PSFM_P3D_PACK), "grouped staging: pack layers, 4 chunks");
    constexpr int NMF = ND == 8 ? 2 : 1, HW = ND / 2;   // MFMAs per pixel pair; 32-bit words per (pixel, k'')
    constexpr bool PK = MODE == PSFM_P3D_PACK;
    typedef short bf8 __attribute__((ext_vector_type(8)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint32_t sd[NPIX * LKK * HW];
    __shared__ __attribute__((aligned(16))) float sG[9 * GS];
    const int ngr = a.K / (DC * CPW);   // chunk groups (host: K % (8 CPW) == 0)
    int L;
    {
        const int n = gridDim.x, w = blockIdx.x, q = n / 8, rm = n % 8, xcd = w % 8, idx = w / 8;
        L = xcd < rm ? xcd * (q + 1) + idx : rm * (q + 1) + (xcd - rm) * q + idx;
    }
    const int kbase = (L % ngr) * (DC * CPW);
    const int rest = L / ngr, tile = rest % (gxn * gyn), b = rest / (gxn * gyn);
    const int x0 = (tile % gxn) * TX, y0 = (tile / gxn) * TY;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, m = lane & 15, j = lane >> 4;
    const uint16_t* dyb = static_cast<const uint16_t*>(a.dy) + b * a.ys[0];
    const int ys2 = (int)a.ys[2], ys3 = (int)a.ys[3];
    // staging unit = (halo pixel, o pair): k0 .. k0+7 of o and o+1 + the k0-1 / k0+8 halo elements;
    // chunk-independent int32 offsets (host-checked) and validity bits.  Pack: channel o K + k of
    // the pixel, one 16-byte run per o.  Unpack (dy pixel-shuffled): channel c' = (o K + k) / 4 of
    // sub-pixel (2y + i, 2x + j), (i, j) = k & 3 — per o the 8 k are 4 sub-pixels x 2 channels
    // (c', c' + 1), four 4-byte loads.
    int off[ITER], cb[ITER];
    uint32_t ok = 0u;
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
        const int u = t + i * 256, pu = GRP ? u >> 2 : u, pix = pu / NPAIR, o = 2 * (pu % NPAIR);
        const int gy = y0 - 1 + pix / LX, gx = x0 - 1 + pix % LX;
        const bool in = u < UNITS && (unsigned)gy < (unsigned)a.Hv && (unsigned)gx < (unsigned)a.Wv;
        off[i] = in ? (PK ? gy * ys2 + gx * ys3 + o * a.K + (GRP ? 8 * (t & 3) : 0) : 2 * gy * ys2 + 2 * gx * ys3) : 0;
        cb[i] = (o * a.K) >> 2;
        ok |= in ? 1u << i : 0u;
    }
    uint4 v0[ITER], v1[ITER];   // pack: the two runs; unpack: the 4 sub-pixel words of o, o + 1
    uint16_t e[ITER][4];
    auto load = [&](int k0) {
        const bool lo = k0 > 0, hi = k0 + DC < a.K;   // clamped halo reads (zeroed at the store)
#pragma unroll
        for (int i = 0; i < ITER; ++i) {
            if constexpr (GRP) {   // k0 = the group's first k; this lane's chunk t & 3 is in off[]
                const uint16_t* s0 = dyb + off[i] + k0;
                const uint16_t* s1 = s0 + a.K;
                v0[i] = *reinterpret_cast<const uint4*>(s0);
                v1[i] = *reinterpret_cast<const uint4*>(s1);
                const int c = t & 3;
                const bool glo = c == 0 && k0 > 0, ghi = c == 3 && k0 + 4 * DC < a.K;
                e[i][0] = s0[glo ? -1 : (ghi ? DC : 0)];
                e[i][1] = s1[glo ? -1 : (ghi ? DC : 0)];
            } else if constexpr (PK) {
                const uint16_t* s0 = dyb + off[i] + k0;
                const uint16_t* s1 = s0 + a.K;
                v0[i] = *reinterpret_cast<const uint4*>(s0);
                v1[i] = *reinterpret_cast<const uint4*>(s1);
                e[i][0] = s0[lo ? -1 : 0];
                e[i][1] = s1[lo ? -1 : 0];
                e[i][2] = s0[hi ? DC : 0];
                e[i][3] = s1[hi ? DC : 0];
            } else {
                const uint16_t* p = dyb + off[i] + cb[i] + (k0 >> 2);   // (2y, 2x), channel c' of o
                const int ko = a.K >> 2;                                  // o + 1: K / 4 channels on
                uint32_t w[2][4];
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int ij = 0; ij < 4; ++ij)
                        w[r][ij] = *reinterpret_cast<const uint32_t*>(p + r * ko + (ij >> 1) * ys2 + (ij & 1) * ys3);
                v0[i] = make_uint4(w[0][0], w[0][1], w[0][2], w[0][3]);
                v1[i] = make_uint4(w[1][0], w[1][1], w[1][2], w[1][3]);
                // k0 - 1 = channel c' - 1 at (1, 1); k0 + 8 = channel c' + 2 at (0, 0)
                e[i][0] = p[lo ? ys2 + ys3 - 1 : 0];
                e[i][1] = p[lo ? ko + ys2 + ys3 - 1 : 0];
                e[i][2] = p[hi ? 2 : 0];
                e[i][3] = p[hi ? ko + 2 : 0];
            }
        }
    };
    // unpack words -> the pack run order (k0 + kk: kk = 2 i + j of channel c', then of c' + 1)
    auto runs = [](uint4 w) {
        return make_uint4((w.x & 0xffffu) | (w.y << 16), (w.z & 0xffffu) | (w.w << 16),
                          (w.x >> 16) | (w.y & 0xffff0000u), (w.z >> 16) | (w.w & 0xffff0000u));
    };
    // grouped: chunk ci of the group starting at kg; lanes of chunk ci write k'' = 1..8, the lanes of
    // chunk ci - 1 / ci + 1 their last / first element pair as k'' = 0 / 9 (the group ends: the
    // 2-byte halo loads of the chunk 0 / 3 lanes, zero outside 0 .. K-1)
    auto store_g = [&](int kg, int ci) {
        const int c = t & 3;
#pragma unroll
        for (int i = 0; i < ITER; ++i) {
            const int u = t + i * 256;
            if (u >= UNITS) break;
            const bool in = (ok >> i) & 1u;
            const int pu = u >> 2, pix = pu / NPAIR, op = pu % NPAIR;
            uint32_t* d = sd + pix * LKK * HW + op;
            const uint4 p0 = in ? v0[i] : make_uint4(0u, 0u, 0u, 0u), p1 = in ? v1[i] : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t a4[4] = {p0.x, p0.y, p0.z, p0.w}, b4[4] = {p1.x, p1.y, p1.z, p1.w};
            const uint32_t ew = (uint32_t)e[i][0] | ((uint32_t)e[i][1] << 16);
            if (c == ci) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    d[(2 * q + 1) * HW] = (a4[q] & 0xffffu) | (b4[q] << 16);
                    d[(2 * q + 2) * HW] = (a4[q] >> 16) | (b4[q] & 0xffff0000u);
                }
                if (ci == 0) d[0] = in && kg > 0 ? ew : 0u;
                if (ci == 3) d[(LKK - 1) * HW] = in && kg + 4 * DC < a.K ? ew : 0u;
            }
            if (c == ci - 1) d[0] = (a4[3] >> 16) | (b4[3] & 0xffff0000u);            // element 7
            if (c == ci + 1) d[(LKK - 1) * HW] = (a4[0] & 0xffffu) | (b4[0] << 16);  // element 0
        }
    };
    auto store = [&](int k0) {
        const bool lo = k0 > 0, hi = k0 + DC < a.K;
#pragma unroll
        for (int i = 0; i < ITER; ++i) {
            const int u = t + i * 256;
            if (u >= UNITS) break;
            const bool in = (ok >> i) & 1u;
            const int pix = u / NPAIR, op = u % NPAIR;
            uint32_t* d = sd + pix * LKK * HW + op;   // word (o, o + 1) of k'' = 0
            const uint4 r0 = PK ? v0[i] : runs(v0[i]), r1 = PK ? v1[i] : runs(v1[i]);
            const uint4 p0 = in ? r0 : make_uint4(0u, 0u, 0u, 0u), p1 = in ? r1 : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t a4[4] = {p0.x, p0.y, p0.z, p0.w}, b4[4] = {p1.x, p1.y, p1.z, p1.w};
            d[0] = in && lo ? (uint32_t)e[i][0] | ((uint32_t)e[i][1] << 16) : 0u;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                d[(2 * q + 1) * HW] = (a4[q] & 0xffffu) | (b4[q] << 16);
                d[(2 * q + 2) * HW] = (a4[q] >> 16) | (b4[q] & 0xffff0000u);
            }
            d[(LKK - 1) * HW] = in && hi ? (uint32_t)e[i][2] | ((uint32_t)e[i][3] << 16) : 0u;
        }
    };
    load(kbase);
    // A fragments (lane row m = shift s, contraction block j): bf16 hi / lo parts of the weights
    bf8 A[NMF];
#pragma unroll
    for (int c = 0; c < NMF; ++c) {
        uint32_t wd[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t hv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int el = 2 * q + h;
                int dz, o, part;
                bool live;
                if (ND == 8) {   // blocks 4c + j: (dz 0..2, hi), (dz 0..2, lo), zero, zero; element = o
                    const int gb = 4 * c + j;
                    live = gb < 6;
                    dz = gb % 3, part = gb / 3, o = el;
                } else {         // block j: dz = j (j < 3); elements 0..3 hi of o 0..3, 4..7 lo
                    live = j < 3;
                    dz = j, part = el >> 2, o = el & 3;
                }
                live = live && m < 9;
                const float wf = live ? a.w[o * 27 + dz * 9 + m] : 0.0f;
                const uint32_t u = __float_as_uint(wf);
                const uint32_t hib = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;   // RNE
                const float lof = wf - __uint_as_float(hib << 16);               // exact
                const uint32_t ul = __float_as_uint(lof);
                const uint32_t lob = (ul + 0x7fffu + ((ul >> 16) & 1u)) >> 16;
                hv[h] = part ? lob : hib;
            }
            wd[q] = hv[0] | (hv[1] << 16);
        }
        A[c] = __builtin_bit_cast(bf8, make_uint4(wd[0], wd[1], wd[2], wd[3]));
    }
    // B fragment geometry: column m = kk + 8 pp (pixel pp of the pair), contraction block j -> dz
    const int kk = m & 7, pp = m >> 3;
    int dzb[NMF];
    bool zb[NMF];
#pragma unroll
    for (int c = 0; c < NMF; ++c) {
        const int gb = ND == 8 ? 4 * c + j : j;
        zb[c] = ND == 8 ? gb >= 6 : j >= 3;
        dzb[c] = zb[c] ? 0 : (ND == 8 ? gb % 3 : j);
    }
    // G position of k: the two k a shift-sum thread stores adjacent — pack: k, k + 4 (channels c,
    // c + 1 of one input sub-pixel), unpack: k, k + 1 (adjacent channels of x)
    const int prow = PK ? (kk & 3) * 2 + (kk >> 2) : kk;
    // shift-sum thread = (tile pixel, pair): pack k = k0 + 2 i + j and k + 4; unpack k0 + 2 sub, + 1
    const int p = t >> 2, sub = t & 3, py = p / TX, px = p % TX;
    const int oy = y0 + py, ox = x0 + px;
    for (int ci = 0; ci < CPW; ++ci) {
        const int k0 = kbase + ci * DC;
        if (ci) __syncthreads();   // the previous chunk's mix (sd) and shift-sum (sG) are done
        if constexpr (GRP) store_g(kbase, ci);
        else store(k0);
        __syncthreads();
        if (!GRP && ci + 1 < CPW) load(k0 + DC);
        // the channel mix: N tile = halo pixel pair np; C/D map: column = lane & 15, row = 4 j + reg
#pragma unroll 2
        for (int np = wv; np < NPIX / 2; np += 4) {
            const int pix = 2 * np + pp;
            f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int c = 0; c < NMF; ++c) {
                const uint32_t* src = sd + (pix * LKK + kk - dzb[c] + 2) * HW;
                uint4 bw;
                if (ND == 8) {
                    bw = *reinterpret_cast<const uint4*>(src);
                } else {
                    const uint2 h2 = *reinterpret_cast<const uint2*>(src);
                    bw = make_uint4(h2.x, h2.y, h2.x, h2.y);   // the hi and lo blocks share dy
                }
                if (zb[c]) bw = make_uint4(0u, 0u, 0u, 0u);
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[c], __builtin_bit_cast(bf8, bw), acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int s = 4 * j + r;
                if (s < 9) sG[s * GS + pix * DC + prow] = acc[r];
            }
        }
        __syncthreads();
        float2 sum = make_float2(0.0f, 0.0f);
#pragma unroll
        for (int s = 0; s < 9; ++s) {
            const int ty = s / 3, tx = s % 3;
            const float2 g = *reinterpret_cast<const float2*>(sG + s * GS + ((py - ty + 2) * LX + (px - tx + 2)) * DC + 2 * sub);
            sum.x += g.x;
            sum.y += g.y;
        }
        if (oy < a.Hv && ox < a.Wv) {
            const int64_t o = vaddr<MODE>(a, b, PK ? k0 + sub : k0 + 2 * sub, oy, ox);
            uint32_t ux = __float_as_uint(sum.x), uy = __float_as_uint(sum.y);
            ux = (ux + 0x7fffu + ((ux >> 16) & 1u)) >> 16;
            uy = (uy + 0x7fffu + ((uy >> 16) & 1u)) >> 16;
            if (a.xs[1] == 1) {   // the pair's channels adjacent (even offset: host-checked)
                *reinterpret_cast<uint32_t*>(static_cast<uint16_t*>(a.dx) + o) = ux | (uy << 16);
            } else {
                static_cast<uint16_t*>(a.dx)[o] = (uint16_t)ux;
                static_cast<uint16_t*>(a.dx)[o + a.xs[1]] = (uint16_t)uy;
            }
        }
    }
}

// --------------------------------------------------------------------------------------------
// dW[o][tap] = sum_{b,p,k} dy[o, k, p] V[k + dz - 1, p + (dy, dx) - 1], dbias[o] = sum dy[o, ., .]:
// per-workgroup partials over a 4 x 16 pixel tile and its share of the channel chunks.
// Thread t < 252: spatial shift s = t % 9 ((dy, dx) of the tap) and pixel group pg = t / 9
// (pixels pg, pg + 28, pg + 56 of the tile); it keeps the ND x 3 (o, dz) partials of its shift in
// registers: per pixel one 18-channel V run (shared by the three dz) and ND 16-channel dy runs
// feed 48 ND FMAs (~10 FMAs per 16-byte LDS read; one thread per (tap, o) needed 2).  Shift-0
// threads also sum dy for dbias.  The pixel groups are folded in a fixed order through LDS at the
// end (deterministic), one partial row per workgroup as before.
// Staging: dy of a pack layer in channels_last (CL): each (pixel, o) run of 16 channels is one
// pair of 16-byte loads; otherwise element loads through yaddr.
template <typename T, int MODE, int ND, bool CL>
__device__ __forceinline__ void bwd_w_body(const P3& a) {
    constexpr int TY = 4, TX = 16, DC = 16, LY = TY + 2, LX = TX + 2, LK = DC + 2;
    constexpr int NPG = 28, NACT = 9 * NPG, NP = TY * TX;
    constexpr int GS = DC + 4;                  // per-(pixel, o) run stride in sg (16-B aligned, 4 mod 8)
    __shared__ __attribute__((aligned(16))) float sv[LY * LX * LK + 2];  // [yy][xx][kk] with halo
    __shared__ __attribute__((aligned(16))) float sg[NP * ND * GS];      // [p][o][kl]
    const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
    const int b = blockIdx.z / a.KG, kg = blockIdx.z - b * a.KG;
    const int nch = (a.K + DC - 1) / DC, c_lo = kg * nch / a.KG, c_hi = (kg + 1) * nch / a.KG;
    const int t = threadIdx.x;
    const int sft = t % 9, pg = t / 9, sdy = sft / 3, sdx = sft % 3;
    float acc[ND][3], accb[ND];
#pragma unroll
    for (int o = 0; o < ND; ++o) {
        acc[o][0] = acc[o][1] = acc[o][2] = 0.0f;
        accb[o] = 0.0f;
    }
    for (int ch = c_lo; ch < c_hi; ++ch) {
        const int k0 = ch * DC;
        __syncthreads();
        for (int e = t; e < LY * LX * LK; e += NTH) {
            const int kk = e % LK, rest = e / LK, xx = rest % LX, yy = rest / LX;
            const int gk = k0 - 1 + kk, gy = y0 - 1 + yy, gx = x0 - 1 + xx;
            const bool in = gk >= 0 && gk < a.K && gy >= 0 && gy < a.Hv && gx >= 0 && gx < a.Wv;
            sv[e] = in ? ld<T>(a.x, vaddr<MODE>(a, b, gk, gy, gx)) : 0.0f;
        }
        if constexpr (CL) {   // (pixel, o) runs of 16 contiguous channels: 2 x 16-byte loads each
            for (int u = t; u < NP * ND; u += NTH) {
                const int oo = u % ND, p = u / ND, gy = y0 + p / TX, gx = x0 + p % TX;
                float v[16];
                if (gy < a.Hv && gx < a.Wv) {
                    const T* src = static_cast<const T*>(a.dy) + yaddr<MODE>(a, b, oo, k0, gy, gx);
                    if constexpr (sizeof(T) == 2) {
                        const uint4 q0 = reinterpret_cast<const uint4*>(src)[0], q1 = reinterpret_cast<const uint4*>(src)[1];
                        const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            v[2 * i] = __uint_as_float(w[i] << 16);
                            v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
                        }
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const float4 q = reinterpret_cast<const float4*>(src)[i];
                            v[4 * i] = q.x, v[4 * i + 1] = q.y, v[4 * i + 2] = q.z, v[4 * i + 3] = q.w;
                        }
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 16; ++i) v[i] = 0.0f;
                }
                float4* dst = reinterpret_cast<float4*>(sg + (p * ND + oo) * GS);
#pragma unroll
                for (int i = 0; i < 4; ++i) dst[i] = make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
            }
        } else {
            for (int e = t; e < NP * ND * DC; e += NTH) {
                const int kl = e % DC, r1 = e / DC, oo = r1 % ND, p = r1 / ND, py = p / TX, px = p % TX;
                const int gk = k0 + kl, gy = y0 + py, gx = x0 + px;
                const bool in = gk < a.K && gy < a.Hv && gx < a.Wv;
                sg[(p * ND + oo) * GS + kl] = in ? ld<T>(a.dy, yaddr<MODE>(a, b, oo, gk, gy, gx)) : 0.0f;
            }
        }
        __syncthreads();
        if (t < NACT) {
            for (int p = pg; p < NP; p += NPG) {
                const int py = p / TX, px = p % TX;
                const float* vr = sv + ((py + sdy) * LX + (px + sdx)) * LK;   // kk = 0..17 <-> k0-1 .. k0+16
                float v[LK];
#pragma unroll
                for (int i = 0; i < LK; ++i) v[i] = vr[i];
#pragma unroll
                for (int o = 0; o < ND; ++o) {
                    const float4* g4 = reinterpret_cast<const float4*>(sg + (p * ND + o) * GS);
                    float g[DC];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float4 q = g4[i];
                        g[4 * i] = q.x, g[4 * i + 1] = q.y, g[4 * i + 2] = q.z, g[4 * i + 3] = q.w;
                    }
#pragma unroll
                    for (int kl = 0; kl < DC; ++kl) {
                        acc[o][0] += g[kl] * v[kl];
                        acc[o][1] += g[kl] * v[kl + 1];
                        acc[o][2] += g[kl] * v[kl + 2];
                    }
                    if (sft == 0) {
#pragma unroll
                        for (int kl = 0; kl < DC; ++kl) accb[o] += g[kl];
                    }
                }
            }
        }
    }
    // fold the pixel groups in order: red[pg][tap * ND + o], bias rows after the taps
    __syncthreads();
    float* red = sg;   // NPG * (27 ND + ND) <= NP ND GS floats
    if (t < NACT) {
#pragma unroll
        for (int o = 0; o < ND; ++o)
#pragma unroll
            for (int dz = 0; dz < 3; ++dz) red[pg * (28 * ND) + (dz * 9 + sft) * ND + o] = acc[o][dz];
        if (sft == 0) {
#pragma unroll
            for (int o = 0; o < ND; ++o) red[pg * (28 * ND) + 27 * ND + o] = accb[o];
        }
    }
    __syncthreads();
    const int64_t blk = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (t < 28 * ND) {
        float s = 0.0f;
        for (int q = 0; q < NPG; ++q) s += red[q * (28 * ND) + t];
        a.ws[blk * (27 * ND + ND) + t] = s;
    }
}

// --------------------------------------------------------------------------------------------
// dW on the matrix cores — bf16 channels_last PACK layers (every PackNet encoder pack layer; the
// first one is 10 G MACs per pass).  For one pixel p and a 32-channel chunk, the contribution to
// dW is a small GEMM: A = dy[o][k] (d rows x 32 k) times B = the pixel's packed neighbourhood
// B[k][n] = V[k + dz - 1, p + (sdy, sdx) - 1] for the 27 taps n = dz*9 + sdy*3 + sdx, plus a column
// of ones (n = 27: the bias gradient sum_k dy) — one v_mfma_f32_16x16x32_bf16 per 16 columns
// (M = 16 rows, d real; N = 32 columns, 28 real), accumulated over the tile's pixels and the
// workgroup's chunks in fp32.  Workgroup = 4 x 16 pixel tile, 4 waves (wave w: tile row w).
// LDS: V halo tile sv[yy][xx][kk] = V[k0 - 1 + kk] (kk < 34, rows padded to 40: 16-B aligned), the
// (pixel, o) dy runs sg[p][o][32].  A lane's B fragment (8 consecutive k of its column) starts
// dz elements into an aligned 16-B run: one ds_read_b128 + one ds_read_b32, and a 0 / 1 / 2
// element shift (the dword funnel of dz = 1 is v_alignbyte).  Staging: x is channels_last and
// V[k = 4c + 2i + j, y, x] = x[b, 2y + i, 2x + j, c], so each (pixel, i, j) gives 8 channels of
// the chunk as one 16-byte load (k = k0 + 4e + 2i + j); the chunk halo k0 - 1 / k0 + 32 is one
// element each.  Fixed instruction order, no atomics: deterministic; products of bf16 values are
// exact in fp32 (the VALU kernel's arithmetic up to the accumulation order).
// UNPACK layers (round 4): V = x itself, channels_last, so a (pixel, quarter) staging unit is 8
// consecutive k (one 16-byte load, stored as a contiguous run); dy is pixel-shuffled: channel c' =
// (o K + k) / 4 of sub-pixel (2y + i, 2x + j), (i, j) = k & 3, so a (pixel, o, sub-pixel) unit is 8
// channels c' (16 bytes) = every 4th k of the 32-k run, stored interleaved.
template <int ND, int MODE = PSFM_P3D_PACK>
__global__ __launch_bounds__(NTH) void k_p3d_bwd_w_mfma(P3 a) {
    constexpr bool PK = MODE == PSFM_P3D_PACK;
    constexpr int TY = 4, TX = 16, DC = 32, LY = TY + 2, LX = TX + 2, LKP = 40, NP = TY * TX;
    // LDS strides in 16-byte units: a pixel's V run 5, a tile row 97 (= 18 x 5 + 7), a (pixel, o)
    // dy run 5.  The 9 spatial shifts a 16-lane MFMA fragment read touches sit at 5 sx + 97 sy
    // = 5 sx + sy (mod 16): 9 distinct 4-bank groups; the A rows m = 0..7 at 5 m (mod 16): distinct
    // (rows of 40 / 32 elements had 2-way conflicts: 13.6 % of the kernel's CU cycles, PMC)
    constexpr int ROWS = LX * LKP + 56, DCP = 40;
    typedef short bf8 __attribute__((ext_vector_type(8)));
    typedef float f4 __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) uint16_t sv[LY * ROWS];
    __shared__ __attribute__((aligned(16))) uint16_t sg[NP * ND * DCP];
    // the 4 waves' accumulators at the end reuse the dy tile's LDS (3 workgroups per CU stay)
    typedef float RedT[2][64][4];
    static_assert(sizeof(float) * 4 * 2 * 64 * 4 <= sizeof(uint16_t) * NP * ND * DCP, "red fits in sg");
    const WG g = wg_coords(a);
    const int x0 = g.bx * TX, y0 = g.by * TY;
    const int b = g.bz / a.KG, kg = g.bz - b * a.KG;
    const int nch = a.K / DC, c_lo = kg * nch / a.KG, c_hi = (kg + 1) * nch / a.KG;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int m = lane & 15, kq = (lane >> 4) * 8;
    // this lane's B columns in the two halves: kind 0 = tap (dz, sdy, sdx), 1 = ones, 2 = zero
    int kind[2], dz[2], off[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int n = 16 * h + m;
        kind[h] = n < 27 ? 0 : (n == 27 ? 1 : 2);
        const int tap = n < 27 ? n : 0, s = tap % 9;
        dz[h] = tap / 9;
        off[h] = (s / 3) * ROWS + (s % 3) * LKP + kq;   // + (tile row, column) of the pixel
    }
    const uint16_t* xv = static_cast<const uint16_t*>(a.x);
    const uint16_t* gy = static_cast<const uint16_t*>(a.dy);
    f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    // software pipeline: the next chunk's global loads are issued into registers right after this
    // chunk's tiles are in LDS, so their latency runs under this chunk's MFMA loop
    constexpr int NV = (LY * LX * 4 + NTH - 1) / NTH;   // 16-byte V runs per thread
    static_assert(LY * LX * 2 <= NTH && (NP * ND * 4) % NTH == 0, "staging slots");
    // chunk-independent element offsets (int32: host-checked), computed once: a chunk adds c0 = k0 / 4
    // (x) or k0 (dy); out-of-image / out-of-range slots read offset 0 and are zeroed by a select
    // (no exec-mask branches around the loads)
    int vo[NV], go[ND], ho;
    uint32_t vok = 0u, gok = 0u;
    bool hok;
#pragma unroll
    for (int u = 0; u < NV; ++u) {   // (yy, xx, i, j) -> 8 channels c0 .. c0+7 = k0 + 4e + 2i + j
        const int e = t + u * NTH, ij = e & 3, pix = e >> 2, xx = pix % LX, yy = pix / LX;
        const int gyy = y0 - 1 + yy, gxx = x0 - 1 + xx;
        const bool ok = e < LY * LX * 4 && gyy >= 0 && gyy < a.Hv && gxx >= 0 && gxx < a.Wv;
        vo[u] = ok ? (int)vaddr<MODE>(a, b, PK ? ij : 8 * ij, gyy, gxx) : 0;
        vok |= ok ? 1u << u : 0u;
    }
    const int hi = t & 1;
    {   // chunk halo: kk = 0 <-> V[k0 - 1] = (c0 - 1, i = 1, j = 1); kk = 33 <-> V[k0 + 32] = (c0 + 8, 0, 0)
        const int pix = t >> 1, xx = pix % LX, yy = pix / LX, gyy = y0 - 1 + yy, gxx = x0 - 1 + xx;
        hok = t < LY * LX * 2 && gyy >= 0 && gyy < a.Hv && gxx >= 0 && gxx < a.Wv;
        ho = hok ? (int)vaddr<MODE>(a, b, hi ? 32 : -1, gyy, gxx) : 0;   // + the chunk's channel below
    }
#pragma unroll
    for (int u = 0; u < ND; ++u) {   // dy runs: (pixel, o) -> 32 channels o K + k0 .., 4 x 16 B
        const int e = t + u * NTH, qd = e & 3, po = e >> 2, o = po % ND, p = po / ND;
        const int gyy = y0 + p / TX, gxx = x0 + p % TX;
        const bool ok = gyy < a.Hv && gxx < a.Wv;
        go[u] = ok ? (int)yaddr<MODE>(a, b, o, 0, gyy, gxx) + (PK ? 8 * qd : (qd >> 1) * (int)a.ys[2] + (qd & 1) * (int)a.ys[3]) : 0;
        gok |= ok ? 1u << u : 0u;
    }
    uint4 vq[NV], gq[ND];   // NP * ND * 4 / NTH = ND dy slots per thread
    uint16_t hq;
    // load(): loads only (the validity selects sit in store(): a select here would make the
    // loads of the NEXT chunk complete before this chunk's MFMA loop starts)
    bool hin = false;
    auto load = [&](int ch) {
        const int k0 = ch * DC, c0 = PK ? k0 >> 2 : k0, g0 = PK ? k0 : k0 >> 2;   // x / dy channel of the chunk
#pragma unroll
        for (int u = 0; u < NV; ++u) vq[u] = *reinterpret_cast<const uint4*>(xv + ((vok >> u) & 1u ? vo[u] + c0 : 0));
        // k = k0 - 1 -> channel c0 - 1 (i = j = 1); k = k0 + 32 -> channel c0 + 8 (i = j = 0): the
        // offset ho holds the pixel part with channel -1 (i = j = 1) or 8 (i = j = 0)
        hin = hok && (hi ? k0 + 32 < a.K : k0 > 0);
        hq = xv[hin ? ho + c0 : 0];
#pragma unroll
        for (int u = 0; u < ND; ++u) gq[u] = *reinterpret_cast<const uint4*>(gy + ((gok >> u) & 1u ? go[u] + g0 : 0));
    };
    auto store = [&]() {
#pragma unroll
        for (int u = 0; u < NV; ++u) {
            const int e = t + u * NTH, ij = e & 3, pix = e >> 2;
            if (e >= LY * LX * 4) continue;
            const uint4 vv = (vok >> u) & 1u ? vq[u] : make_uint4(0u, 0u, 0u, 0u);
            const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
            uint16_t* row = sv + (pix / LX) * ROWS + (pix % LX) * LKP + 1 + (PK ? 2 * (ij >> 1) + (ij & 1) : 8 * ij);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                row[PK ? 8 * q : 2 * q] = (uint16_t)(w[q] & 0xffffu);
                row[PK ? 8 * q + 4 : 2 * q + 1] = (uint16_t)(w[q] >> 16);
            }
        }
        if (t < LY * LX * 2) sv[((t >> 1) / LX) * ROWS + ((t >> 1) % LX) * LKP + ((t & 1) ? 33 : 0)] = hin ? hq : (uint16_t)0;
#pragma unroll
        for (int u = 0; u < ND; ++u) {
            const int e = t + u * NTH, qd = e & 3, po = e >> 2;
            const uint4 gv = (gok >> u) & 1u ? gq[u] : make_uint4(0u, 0u, 0u, 0u);   // po = p * ND + o
            if constexpr (PK) {
                reinterpret_cast<uint4*>(sg + po * DCP)[qd] = gv;
            } else {   // sub-pixel qd: channels c' + cc -> k = 4 cc + qd
                const uint32_t w[4] = {gv.x, gv.y, gv.z, gv.w};
                uint16_t* dst = sg + po * DCP + qd;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    dst[8 * q] = (uint16_t)(w[q] & 0xffffu);
                    dst[8 * q + 4] = (uint16_t)(w[q] >> 16);
                }
            }
        }
    };
    if (c_lo < c_hi) load(c_lo);
    for (int ch = c_lo; ch < c_hi; ++ch) {
        __syncthreads();   // the previous chunk's MFMA loop is done with the tiles
        store();
        __syncthreads();
        if (ch + 1 < c_hi) load(ch + 1);
#pragma unroll 4
        for (int px = 0; px < TX; ++px) {
            // branch-free fragments: every lane loads (rows m >= ND and the ones / zero columns
            // read a valid run and are replaced by selects), so the loop carries no exec-mask
            // branches around its LDS reads
            const int p = wv * TX + px;
            const uint4 ar = *reinterpret_cast<const uint4*>(sg + (p * ND + (m < ND ? m : 0)) * DCP + kq);
            const bf8 A = __builtin_bit_cast(bf8, m < ND ? ar : make_uint4(0u, 0u, 0u, 0u));
            bf8 Bf[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint16_t* src = sv + wv * ROWS + px * LKP + off[h];
                const uint4 d = *reinterpret_cast<const uint4*>(src);
                const uint32_t d4 = *reinterpret_cast<const uint32_t*>(src + 8);
                const uint32_t dd[5] = {d.x, d.y, d.z, d.w, d4};
                const uint32_t fill = kind[h] == 1 ? 0x3f803f80u : 0u;   // bf16 1.0 pairs | zero column
                uint32_t o4[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t v = dz[h] == 0 ? dd[q]
                                     : dz[h] == 2 ? dd[q + 1]
                                                  : __builtin_amdgcn_alignbyte(dd[q + 1], dd[q], 2);
                    o4[q] = kind[h] == 0 ? v : fill;
                }
                Bf[h] = __builtin_bit_cast(bf8, make_uint4(o4[0], o4[1], o4[2], o4[3]));
            }
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf[0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bf[1], acc1, 0, 0, 0);
        }
    }
    // the 4 waves' accumulators in wave order -> partial row [tap][o] (taps 0..26), [27 ND + o] bias
    __syncthreads();   // every wave is done with the dy tile that red reuses
    RedT* red = reinterpret_cast<RedT*>(sg);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        red[wv][0][lane][r] = acc0[r];
        red[wv][1][lane][r] = acc1[r];
    }
    __syncthreads();
    const int64_t blk = ((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;   // any 1-1 map
    // C/D map of 16x16x32: column = lane & 15, row = (lane >> 4) * 4 + register
    for (int e = t; e < 28 * ND; e += NTH) {
        const int o = e % ND, n = e / ND, h = n >> 4, col = n & 15;
        const int ln = (o >> 2) * 16 + col, r = o & 3;
        const float v = ((red[0][h][ln][r] + red[1][h][ln][r]) + red[2][h][ln][r]) + red[3][h][ln][r];
        a.ws[blk * (27 * ND + ND) + e] = v;   // e = n * ND + o: taps then the bias row
    }
}

template <typename T, int MODE, int ND, bool CL>
__global__ __launch_bounds__(NTH) void k_p3d_bwd_w(P3 a) { bwd_w_body<T, MODE, ND, CL>(a); }

template <typename T, int MODE, int ND>
__global__ __launch_bounds__(NTH) void k_p3d_bwd_w_generic(P3 a) { bwd_w_body<T, MODE, ND, false>(a); }

// fixed-order fp64 reduction of the partials -> dw [o][tap], dbias [o]: one workgroup per output
// (strided fp64 partial sums per thread, then the wave butterflies and the 4 waves in order)
template <int ND>
__global__ __launch_bounds__(NTH) void k_p3d_reduce_w(const float* ws, int64_t nblk, float* dw, float* db) {
    __shared__ double red[NTH / 64];
    const int t = blockIdx.x, tid = threadIdx.x;
    double s = 0.0;
    for (int64_t i = tid; i < nblk; i += NTH) s += (double)ws[i * (27 * ND + ND) + t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = s;
    __syncthreads();
    if (tid != 0) return;
    const double v = ((red[0] + red[1]) + red[2]) + red[3];
    if (t < 27 * ND) {
        if (dw) dw[(t % ND) * 27 + t / ND] = (float)v;
    } else if (db) {
        db[t - 27 * ND] = (float)v;
    }
}

// workgroups along the channel axis: enough to fill the chip when the image is small
int k_groups(int K, int DC, int tiles) {
    const int nch = (K + DC - 1) / DC;
    return std::max(1, std::min(nch, (2048 + tiles - 1) / std::max(tiles, 1)));
}

int check_desc(const psfm_p3d_desc* t) {
    if (!t) return fail(-1, "null descriptor");
    if (t->mode != PSFM_P3D_PACK && t->mode != PSFM_P3D_UNPACK) return fail(-2, "bad mode");
    if (t->dtype != PSFM_P3D_F32 && t->dtype != PSFM_P3D_BF16) return fail(-2, "bad dtype");
    if (t->B < 1 || t->C < 1 || t->Hv < 1 || t->Wv < 1 || t->r < 1) return fail(-3, "bad shape");
    if (t->d != 4 && t->d != 8) return fail(-4, "d (3-D features) must be 4 or 8");
    if (t->mode == PSFM_P3D_UNPACK && (t->d * t->C) % (t->r * t->r)) return fail(-3, "d*C not divisible by r^2");
    return 0;
}

P3 make(const psfm_p3d_desc* t) {
    P3 a{};
    a.B = t->B;
    a.C = t->C;
    a.Hv = t->Hv;
    a.Wv = t->Wv;
    a.r = t->r;
    a.K = t->mode == PSFM_P3D_PACK ? t->C * t->r * t->r : t->C;
    for (int i = 0; i < 4; ++i) {
        a.xs[i] = t->xs[i];
        a.ys[i] = t->ys[i];
    }
    return a;
}

#define P3D_LAUNCH_D(KERNEL, ND, grid, st, a, t)                                                        \
    do {                                                                                                \
        if ((t)->dtype == PSFM_P3D_BF16) {                                                              \
            if ((t)->mode == PSFM_P3D_PACK)                                                             \
                hipLaunchKernelGGL((KERNEL<uint16_t, PSFM_P3D_PACK, ND>), grid, dim3(NTH), 0, st, a);   \
            else                                                                                        \
                hipLaunchKernelGGL((KERNEL<uint16_t, PSFM_P3D_UNPACK, ND>), grid, dim3(NTH), 0, st, a); \
        } else {                                                                                        \
            if ((t)->mode == PSFM_P3D_PACK)                                                             \
                hipLaunchKernelGGL((KERNEL<float, PSFM_P3D_PACK, ND>), grid, dim3(NTH), 0, st, a);      \
            else                                                                                        \
                hipLaunchKernelGGL((KERNEL<float, PSFM_P3D_UNPACK, ND>), grid, dim3(NTH), 0, st, a);    \
        }                                                                                               \
    } while (0)
#define P3D_LAUNCH(KERNEL, grid, st, a, t)                                                              \
    do {                                                                                                \
        if ((t)->d == 4)                                                                                \
            P3D_LAUNCH_D(KERNEL, 4, grid, st, a, t);                                                    \
        else                                                                                            \
            P3D_LAUNCH_D(KERNEL, 8, grid, st, a, t);                                                    \
    } while (0)

dim3 grid_of(P3& a, int TY, int TX, int DC) {
    const int gx = (a.Wv + TX - 1) / TX, gy = (a.Hv + TY - 1) / TY;
    a.KG = k_groups(a.K, DC, gx * gy * a.B);
    a.lin = 0;
    return dim3(gx, gy, a.B * a.KG);
}
// the XCD-grouped 1-D grid (wg_coords): kg_chunks channel chunks of DC per workgroup
dim3 grid_lin(P3& a, int TY, int TX, int DC, int kg_chunks) {
    a.gxn = (a.Wv + TX - 1) / TX;
    a.gyn = (a.Hv + TY - 1) / TY;
    a.KG = std::max(1, ((a.K + DC - 1) / DC) / kg_chunks);
    a.lin = 1;
    return dim3((unsigned)((int64_t)a.gxn * a.gyn * a.B * a.KG));
}
constexpr int P3D_FWD_CPW = 2;   // channel chunks per workgroup, channels_last pack forward
constexpr int P3D_DW_CPW = 2;    // and MFMA weight gradient (the next chunk's loads overlap the MFMAs)

}  // namespace

extern "C" {

int psfm_p3d_fwd(const psfm_p3d_desc* t, const void* x, const float* w, const float* bias, void* y, void* stream) {
    if (int e = check_desc(t)) return e;
    if (!x || !w || !y) return fail(-1, "null pointer");
    P3 a = make(t);
    a.x = x;
    a.y = y;
    a.w = w;
    a.bias = bias;
    dim3 grid = grid_of(a, 4, 16, 32);
    hipStream_t st = (hipStream_t)stream;
    // channels_last pack output: each thread's 8 folded channels are one aligned 16-byte run
    const int vec = t->dtype == PSFM_P3D_BF16 ? 8 : 4;
    const bool vst = t->mode == PSFM_P3D_PACK && a.ys[1] == 1 && a.K % 8 == 0 && a.ys[0] % vec == 0 &&
                     a.ys[2] % vec == 0 && a.ys[3] % vec == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0;
    // channels_last x with r = 2 as well: 16-byte staging loads (k_p3d_fwd_cl)
    const int64_t xmax = (int64_t)(t->B - 1) * a.xs[0] + (int64_t)(t->C - 1) * a.xs[1] +
                         (int64_t)(2 * a.Hv - 1) * a.xs[2] + (int64_t)(2 * a.Wv - 1) * a.xs[3];   // int32 staging offsets
    const bool xcl = vst && t->r == 2 && a.K % 32 == 0 && a.xs[1] == 1 && a.xs[0] % vec == 0 &&
                     a.xs[2] % vec == 0 && a.xs[3] % vec == 0 && a.xs[0] >= 0 && a.xs[2] >= 0 && a.xs[3] >= 0 &&
                     xmax < INT32_MAX - 64 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    // the matrix-core form (k_p3d_fwd_mfma): bf16, r = 2, channels_last x with 16-byte 8-channel runs,
    // 32-k chunks, channels_last y (pack: 8-byte 4-channel stores); PSFM_P3D_FWD=mfma / valu (A/B)
    const int fknob = knob(KNOB_P3D_FWD);
    // default: d = 8 (PackNet01) every layer, d = 4 (PackNetSAN01) unpack layers only — with 4 of the
    // 16 MFMA columns useful per part the d = 4 pack layers run faster on the VALU kernel
    // (profiles/r04/p3d/ab_fwd_*: first PackNet01 layer 449 -> 400-421 us, unpack 96x320 133 -> 62;
    // first PackNetSAN01 layer 90 vs 124-136)
    const bool fwant = fknob ? fknob == 1 : (P3D_FWD_MFMA_DEFAULT || t->d == 8 || t->mode == PSFM_P3D_UNPACK);
    const int64_t xmaxm = t->mode == PSFM_P3D_PACK ? xmax
                                                   : (int64_t)(t->B - 1) * a.xs[0] + (int64_t)(a.K - 1) * a.xs[1] +
                                                         (int64_t)(a.Hv - 1) * a.xs[2] + (int64_t)(a.Wv - 1) * a.xs[3];
    const bool fmfma = fwant && t->dtype == PSFM_P3D_BF16 && t->r == 2 && a.K % 32 == 0 && a.xs[1] == 1 &&
                       a.xs[0] % 8 == 0 && a.xs[2] % 8 == 0 && a.xs[3] % 8 == 0 && a.xs[0] >= 0 && a.xs[2] >= 0 &&
                       a.xs[3] >= 0 && xmaxm < INT32_MAX - 64 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                       a.ys[1] == 1 &&
                       (t->mode == PSFM_P3D_UNPACK || (a.ys[0] % 4 == 0 && a.ys[2] % 4 == 0 && a.ys[3] % 4 == 0 &&
                                                      (reinterpret_cast<uintptr_t>(y) & 7) == 0));
    if (fmfma) {
        grid = grid_lin(a, 4, 16, 32, P3D_FWD_CPW);
        if (t->mode == PSFM_P3D_PACK) {
            if (t->d == 4) hipLaunchKernelGGL((k_p3d_fwd_mfma<4, PSFM_P3D_PACK>), grid, dim3(NTH), 0, st, a);
            else hipLaunchKernelGGL((k_p3d_fwd_mfma<8, PSFM_P3D_PACK>), grid, dim3(NTH), 0, st, a);
        } else {
            if (t->d == 4) hipLaunchKernelGGL((k_p3d_fwd_mfma<4, PSFM_P3D_UNPACK>), grid, dim3(NTH), 0, st, a);
            else hipLaunchKernelGGL((k_p3d_fwd_mfma<8, PSFM_P3D_UNPACK>), grid, dim3(NTH), 0, st, a);
        }
    } else if (xcl) {
        grid = grid_lin(a, 4, 16, 32, P3D_FWD_CPW);
        if (t->dtype == PSFM_P3D_BF16) {
            if (t->d == 4) hipLaunchKernelGGL((k_p3d_fwd_cl<uint16_t, 4>), grid, dim3(NTH), 0, st, a);
            else hipLaunchKernelGGL((k_p3d_fwd_cl<uint16_t, 8>), grid, dim3(NTH), 0, st, a);
        } else {
            if (t->d == 4) hipLaunchKernelGGL((k_p3d_fwd_cl<float, 4>), grid, dim3(NTH), 0, st, a);
            else hipLaunchKernelGGL((k_p3d_fwd_cl<float, 8>), grid, dim3(NTH), 0, st, a);
        }
    } else if (vst) {
        grid = grid_lin(a, 4, 16, 32, P3D_FWD_CPW);
        if (t->dtype == PSFM_P3D_BF16) {
            if (t->d == 4) hipLaunchKernelGGL((k_p3d_fwd<uint16_t, PSFM_P3D_PACK, 4>), grid, dim3(NTH), 0, st, a);
            else hipLaunchKernelGGL((k_p3d_fwd<uint16_t, PSFM_P3D_PACK, 8>), grid, dim3(NTH), 0, st, a);
        } else {
            if (t->d == 4) hipLaunchKernelGGL((k_p3d_fwd<float, PSFM_P3D_PACK, 4>), grid, dim3(NTH), 0, st, a);
            else hipLaunchKernelGGL((k_p3d_fwd<float, PSFM_P3D_PACK, 8>), grid, dim3(NTH), 0, st, a);
        }
    } else {
        P3D_LAUNCH(k_p3d_fwd_generic, grid, st, a, t);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail((int)e, std::string("launch: ") + hipGetErrorString(e));
}

int64_t psfm_p3d_ws_floats(const psfm_p3d_desc* t) {
    if (check_desc(t)) return -1;
    P3 a = make(t);
    const dim3 g = grid_of(a, 4, 16, 16);
    const dim3 gl = grid_lin(a, 4, 16, 32, P3D_DW_CPW);
    return std::max((int64_t)g.x * g.y * g.z, (int64_t)gl.x) * 28 * t->d;
}

int psfm_p3d_bwd(const psfm_p3d_desc* t, const void* x, const float* w, const void* dy, void* dx, float* dw,
                 float* dbias, float* ws, void* stream) {
    if (int e = check_desc(t)) return e;
    if (!x || !w || !dy) return fail(-1, "null pointer");
    if ((dw || dbias) && !ws) return fail(-1, "weight gradient needs the workspace");
    hipStream_t st = (hipStream_t)stream;
    P3 a = make(t);
    a.x = x;
    a.dy = dy;
    a.dx = dx;
    a.w = w;
    {
        // the fast staging path indexes dy with int32 offsets from each image's base
        const int64_t mx = (int64_t)(t->d * a.K - 1) * a.ys[1] + (int64_t)(a.Hv - 1) * a.ys[2] + (int64_t)(a.Wv - 1) * a.ys[3];
        a.dy32 = a.ys[1] >= 0 && a.ys[2] >= 0 && a.ys[3] >= 0 && mx < (int64_t)INT32_MAX;
    }
    if (dx) {
        // channel-contiguous dy of a pack layer (channels_last), every 16-k run 16-byte aligned
        const int vec = t->dtype == PSFM_P3D_BF16 ? 8 : 4;
        const bool cl8 = t->mode == PSFM_P3D_PACK && a.dy32 && a.ys[1] == 1 && a.K % 8 == 0 &&
                         a.ys[0] % vec == 0 && a.ys[2] % vec == 0 && a.ys[3] % vec == 0 &&
                         (reinterpret_cast<uintptr_t>(dy) & 15) == 0;
        const bool cl = cl8 && a.K % 16 == 0;
        // the matrix-core form: bf16, r = 2; 4-byte stores of (c, c + 1) pairs when x is channels_last
        // with even strides (else two 2-byte stores)
        const bool xpair = a.xs[1] != 1 || (a.xs[0] % 2 == 0 && a.xs[2] % 2 == 0 && a.xs[3] % 2 == 0 &&
                                            (reinterpret_cast<uintptr_t>(dx) & 3) == 0);
        // the P3D_DX knob (A/B): 1 the matrix-core form, 2 the VALU k-pair kernel (3 grouped staging, A/B builds)
        const int dknob = knob(KNOB_P3D_DX);
        // default: the matrix-core form for unpack layers (2x the generic kernel at every PackNet
        // shape), the VALU k-pair kernel for pack layers (the matrix-core form's staging issues 1.5x
        // its per-lane line accesses: 0.85-1.0 vs 0.54 ms on the first PackNet01 layer,
        // profiles/r04/p3d/)
        const bool want = dknob ? dknob != 2 : t->mode == PSFM_P3D_UNPACK || P3D_DX_MFMA_DEFAULT;
        // unpack layers: channels_last dy (2 Hv x 2 Wv, d K / 4 channels), 4-byte sub-pixel words
        const int64_t umax = (int64_t)(t->d * a.K / 4 - 1) * a.ys[1] + (int64_t)(2 * a.Hv - 1) * a.ys[2] +
                             (int64_t)(2 * a.Wv - 1) * a.ys[3];
        const bool ucl = t->mode == PSFM_P3D_UNPACK && a.ys[1] == 1 && a.K % 8 == 0 && a.ys[0] % 2 == 0 &&
                         a.ys[2] % 2 == 0 && a.ys[3] % 2 == 0 && a.ys[2] >= 0 && a.ys[3] >= 0 &&
                         umax < (int64_t)INT32_MAX && (reinterpret_cast<uintptr_t>(dy) & 3) == 0;
        const bool mfma = (cl8 || ucl) && t->dtype == PSFM_P3D_BF16 && t->r == 2 && xpair && want;
        if (mfma) {
            const int gxn = (a.Wv + 15) / 16, gyn = (a.Hv + 3) / 4;
            // 8-k chunks per workgroup: 2 when that still leaves >= 1024 workgroups (unpack 96x320 / 48x160
            // layers: 128 vs 138 us), else 1 (the small layers want the workgroups)
            int cpw = a.K % 16 == 0 && (int64_t)gxn * gyn * a.B * (a.K / 16) >= 1024 ? 2 : 1;
            const dim3 g1((unsigned)(gxn * gyn * a.B * (a.K / (8 * cpw))));
#define P3D_DXM(ND, CPW)                                                                                              \
    do {                                                                                                              \
        if (t->mode == PSFM_P3D_PACK)                                                                                 \
            hipLaunchKernelGGL((k_p3d_bwd_x_mfma<ND, CPW, PSFM_P3D_PACK>), g1, dim3(256), 0, st, a, gxn, gyn);        \
        else                                                                                                          \
            hipLaunchKernelGGL((k_p3d_bwd_x_mfma<ND, CPW, PSFM_P3D_UNPACK>), g1, dim3(256), 0, st, a, gxn, gyn);      \
    } while (0)
            if (t->d == 4) {
                if (cpw == 2) P3D_DXM(4, 2);
                else P3D_DXM(4, 1);
            } else {
                if (cpw == 2) P3D_DXM(8, 2);
                else P3D_DXM(8, 1);
            }
#undef P3D_DXM
        } else if (cl) {
            const int gxn = (a.Wv + 15) / 16, gyn = (a.Hv + 3) / 4;
            const dim3 g1((unsigned)(gxn * gyn * a.B * (a.K / 16)));   // one 16-k chunk per workgroup
            if (t->dtype == PSFM_P3D_BF16) {
                if (t->d == 4) hipLaunchKernelGGL((k_p3d_bwd_x_cl<uint16_t, 4>), g1, dim3(128), 0, st, a, gxn, gyn);
                else hipLaunchKernelGGL((k_p3d_bwd_x_cl<uint16_t, 8>), g1, dim3(128), 0, st, a, gxn, gyn);
            } else {
                if (t->d == 4) hipLaunchKernelGGL((k_p3d_bwd_x_cl<float, 4>), g1, dim3(128), 0, st, a, gxn, gyn);
                else hipLaunchKernelGGL((k_p3d_bwd_x_cl<float, 8>), g1, dim3(128), 0, st, a, gxn, gyn);
            }
        } else {
            const dim3 grid = grid_of(a, 4, 8, 16);
            P3D_LAUNCH(k_p3d_bwd_x, grid, st, a, t);
        }
    }
    if (dw || dbias) {
        P3 aw = make(t);
        aw.x = x;
        aw.dy = dy;
        aw.ws = ws;
        dim3 grid = grid_of(aw, 4, 16, 16);
        // channels_last dy of a pack layer: 16-channel runs are contiguous and 16-byte aligned
        const int vec = t->dtype == PSFM_P3D_BF16 ? 8 : 4;
        const bool cl = t->mode == PSFM_P3D_PACK && a.ys[1] == 1 && a.K % 16 == 0 && a.ys[0] % vec == 0 &&
                        a.ys[2] % vec == 0 && a.ys[3] % vec == 0 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0;
        // the matrix-core form: bf16, r = 2, channels_last x (8-channel 16-byte runs) and 32-k chunks
        // (and every element offset of x and dy below 2^31: the kernel's staging offsets are int32)
        const int64_t xmax = (int64_t)(t->B - 1) * a.xs[0] + (int64_t)(t->C - 1) * a.xs[1] +
                             (int64_t)(2 * a.Hv - 1) * a.xs[2] + (int64_t)(2 * a.Wv - 1) * a.xs[3];
        const int64_t ymax = (int64_t)(t->B - 1) * a.ys[0] + (int64_t)(t->d * a.K - 1) * a.ys[1] +
                             (int64_t)(a.Hv - 1) * a.ys[2] + (int64_t)(a.Wv - 1) * a.ys[3];
        const bool mfma = cl && t->dtype == PSFM_P3D_BF16 && t->r == 2 && a.K % 32 == 0 && a.xs[1] == 1 &&
                          t->C % 8 == 0 && a.xs[0] % 8 == 0 && a.xs[2] % 8 == 0 && a.xs[3] % 8 == 0 &&
                          a.xs[0] >= 0 && a.xs[2] >= 0 && a.xs[3] >= 0 && a.ys[0] >= 0 && xmax < INT32_MAX - 64 &&
                          ymax < INT32_MAX - 64 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && MFMA_DW;
        // unpack layers (round 4): x channels_last (V = x: 8-k 16-byte runs), dy channels_last
        // pixel-shuffled (8-channel 16-byte runs per sub-pixel); PSFM_P3D_DW=generic: the VALU kernel (A/B)
        const int64_t uxmax = (int64_t)(t->B - 1) * a.xs[0] + (int64_t)(a.K - 1) * a.xs[1] +
                              (int64_t)(a.Hv - 1) * a.xs[2] + (int64_t)(a.Wv - 1) * a.xs[3];
        const int64_t uymax = (int64_t)(t->B - 1) * a.ys[0] + (int64_t)(t->d * a.K / 4 - 1) * a.ys[1] +
                              (int64_t)(2 * a.Hv - 1) * a.ys[2] + (int64_t)(2 * a.Wv - 1) * a.ys[3];
        const bool dw_generic = knob(KNOB_P3D_DW) == 1;
        const bool umfma = t->mode == PSFM_P3D_UNPACK && t->dtype == PSFM_P3D_BF16 && t->r == 2 && a.K % 32 == 0 &&
                           a.xs[1] == 1 && a.xs[0] % 8 == 0 && a.xs[2] % 8 == 0 && a.xs[3] % 8 == 0 && a.xs[0] >= 0 &&
                           a.xs[2] >= 0 && a.xs[3] >= 0 && a.ys[1] == 1 && a.ys[0] % 8 == 0 && a.ys[2] % 8 == 0 &&
                           a.ys[3] % 8 == 0 && a.ys[0] >= 0 && a.ys[2] >= 0 && a.ys[3] >= 0 && uxmax < INT32_MAX - 64 &&
                           uymax < INT32_MAX - 64 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                           (reinterpret_cast<uintptr_t>(dy) & 15) == 0 && MFMA_DW && !dw_generic;
        if (mfma) {
            grid = grid_lin(aw, 4, 16, 32, P3D_DW_CPW);
            if (t->d == 4) hipLaunchKernelGGL(k_p3d_bwd_w_mfma<4>, grid, dim3(NTH), 0, st, aw);
            else hipLaunchKernelGGL(k_p3d_bwd_w_mfma<8>, grid, dim3(NTH), 0, st, aw);
        } else if (umfma) {
            grid = grid_lin(aw, 4, 16, 32, P3D_DW_CPW);
            if (t->d == 4) hipLaunchKernelGGL((k_p3d_bwd_w_mfma<4, PSFM_P3D_UNPACK>), grid, dim3(NTH), 0, st, aw);
            else hipLaunchKernelGGL((k_p3d_bwd_w_mfma<8, PSFM_P3D_UNPACK>), grid, dim3(NTH), 0, st, aw);
        } else if (cl) {
            if (t->dtype == PSFM_P3D_BF16) {
                if (t->d == 4) hipLaunchKernelGGL((k_p3d_bwd_w<uint16_t, PSFM_P3D_PACK, 4, true>), grid, dim3(NTH), 0, st, aw);
                else hipLaunchKernelGGL((k_p3d_bwd_w<uint16_t, PSFM_P3D_PACK, 8, true>), grid, dim3(NTH), 0, st, aw);
            } else {
                if (t->d == 4) hipLaunchKernelGGL((k_p3d_bwd_w<float, PSFM_P3D_PACK, 4, true>), grid, dim3(NTH), 0, st, aw);
                else hipLaunchKernelGGL((k_p3d_bwd_w<float, PSFM_P3D_PACK, 8, true>), grid, dim3(NTH), 0, st, aw);
            }
        } else {
            P3D_LAUNCH(k_p3d_bwd_w_generic, grid, st, aw, t);
        }
        const int64_t nblk = (int64_t)grid.x * grid.y * grid.z;
        if (t->d == 4)
            hipLaunchKernelGGL(k_p3d_reduce_w<4>, dim3(28 * 4), dim3(NTH), 0, st, (const float*)ws, nblk, dw, dbias);
        else
            hipLaunchKernelGGL(k_p3d_reduce_w<8>, dim3(28 * 8), dim3(NTH), 0, st, (const float*)ws, nblk, dw, dbias);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail((int)e, std::string("launch: ") + hipGetErrorString(e));
}

const char* psfm_p3d_last_error(void) { return g_err.c_str(); }

}  // extern "C"
