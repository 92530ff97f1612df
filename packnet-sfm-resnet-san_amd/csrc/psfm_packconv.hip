// psfm_packconv.hip — the composed PackNet packing layer for MI355X (gfx950), behind
// include/psfm_packconv.h.
//
// Reference: packnet_sfm/networks/layers/packnet/layers01.py:213-247 (PackLayerConv3d: packing ->
// Conv3d(1 -> d, 3x3x3, pad 1) -> view -> Conv2D) and :10-37 (Conv2D: ConstantPad2d(k//2) ->
// Conv2d).  The reference materialises the packed volume V [B, d 4C, H/2, W/2] (755 MB at the
// first PackNet01 layer, B = 6) and convolves it with a d 4C k^2-deep kernel.  Here Conv3d and
// Conv2d are composed into one (k+2) x (k+2) convolution over the packed channels P (read from x
// in place: the packing is addressing), and the reference's zero padding of V is restored by
// the edge terms described in the header.  Kernels:
//   k_pc_conv<KH, KW>  implicit-GEMM convolution on v_mfma_f32_16x16x32_bf16.  A workgroup owns a
//                      4-row x 64-column output tile and 64 output channels; the K loop walks
//                      32-channel chunks of the input (per sub-pixel for P) and, per chunk, the KH
//                      tap rows.  The chunk's halo tile (4 + KH - 1 rows x 64 + KW - 1 columns) and
//                      each tap row's weights are staged in LDS (double-buffered, the next step's
//                      global loads in flight during the current step's MFMAs; the
//                      operand fragments of tap column b + 1 read from LDS during column b's
//                      MFMAs).  Wave w computes output row w, 64 pixels x 64 channels = 4 x 4
//                      accumulator tiles (two rows per wave measured slower: DESIGN.md).  The
//                      epilogue goes through LDS so every store is a 16-byte run.  One kernel
//                      serves the main forward (epilogue: bias table - edge terms -> bf16 y), the
//                      main backward (dy in, written through the packing permutation into dx, +
//                      edge terms) and the 1-D edge convolutions (KH = 1, fp32 out).
//   k_pc_wgrad<KW>     weight gradient sum_p G[p][m] IN[p + tap][kin] on the matrix cores: both
//                      operands are pixel-major in memory, the MFMA contracts pixels, so both are
//                      read transposed from XOR-swizzled LDS images by ds_read_b64_tr_b16
//                      (conflict-free).  Per-split partials, reduced in a fixed order.
//   corner / bias-table kernels: fp32, tiny.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>

#include "../../include/psfm_packconv.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

typedef short bf8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
// staging registers as a native vector (uint4's struct copies became global -> private -> LDS memcpys
// that SROA left in scratch)
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

enum { OUT_F32 = 0, OUT_Y = 1, OUT_DX = 2 };
constexpr int MAXPROB = 8;

__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
__device__ __forceinline__ uint32_t f2bf(float v) {
    uint32_t u = __float_as_uint(v);
    if ((u & 0x7f800000u) == 0x7f800000u) return (u >> 16) | ((u & 0xffffu) ? 0x40u : 0u);  // inf / NaN stay
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;                                          // RNE
}

// An input image read in 32-channel chunks: chunk q = sub * (cin / 32) + cc covers channels
// cc*32 .. cc*32+31 at element offset sub_off[sub] (the sub-pixel of x for the packed P, the
// frame line of dy for the edge backward).
struct Geo {
    const uint16_t* p;
    int64_t s_outer, s_row, s_col;
    int64_t sub_off[4];
    int nsub, cin;
    int rin, cols_in;   // valid input rows / columns (zero outside)
};

struct ConvProb {
    Geo in;
    int outer, rows, cols;   // output extents
    int ph, pw;              // output (r, c) reads input (r + a - ph, c + b - pw)
    int cop, co;             // padded (multiple of 64) / real output channels
    const uint16_t* w;       // [cop/64][nq][KH][KW][4][64][8]
    int mode;
    void* out;
    int64_t o_outer, o_row, o_col;
    int ecs;                 // channel stride of the edge buffers
    const float* e[4];       // edge buffers T, B, L, R: [b][pos][ecs]
    const float* bt;         // OUT_Y: [2pk+1][2pk+1][C]
    int C, pk, Ho, Wo;
};

struct ConvArgs {
    ConvProb p[4];
    int nprob, outer_max, ntc;
    int nbw;   // 64-channel output tiles per workgroup (launch_conv: > 1 only when every problem's input
               // chunks fit the two P buffers, so the staged tile serves all of them)
};

__device__ __forceinline__ int row_class(int y, int n, int pk) {
    return y < pk ? y : (y >= n - pk ? 2 * pk - (n - 1 - y) : pk);
}

// --------------------------------------------------------------------------------------------
template <int KH, int KW>
__global__ __launch_bounds__(256, 1) void k_pc_conv(const ConvArgs A) {
    constexpr int TY = 4, TX = 64, HR = TY + KH - 1, HC = TX + KW - 1;
    constexpr int NP = (HR * HC + 15) & ~15;          // pixels per kq plane (multiple of 16: conflict-free)
    constexpr int PB = 4 * NP * 16;                   // one P buffer [kq][pix][8 bf16]
    constexpr int WB = KW * 4 * 64 * 16;              // one weight buffer [b][kq][n][8 bf16]
    constexpr int NPE = (4 * HR * HC + 255) / 256;    // P staging entries per thread
    constexpr int EPB = 4 * 64 * 68 * 4;              // epilogue tile [wave][px][68 floats], after the P buffers
    constexpr int SMEM = 2 * PB + (2 * WB > EPB ? 2 * WB : EPB);
    static_assert(SMEM <= 160 * 1024, "k_pc_conv LDS");
    __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];

    const int prob = blockIdx.z / A.outer_max, o = blockIdx.z - prob * A.outer_max;
    const ConvProb& P = A.p[prob];
    const int tr = blockIdx.x / A.ntc, tc = blockIdx.x - tr * A.ntc;
    const int r0 = tr * TY, c0 = tc * TX, nb0 = blockIdx.y * A.nbw;
    if (o >= P.outer || r0 >= P.rows || c0 >= P.cols || nb0 * 64 >= P.cop) return;   // whole workgroup

    const int t = threadIdx.x, lane = t & 63, wv = t >> 6, l15 = lane & 15, kq = lane >> 4;
    const int ncc = P.in.cin >> 5, nq = P.in.nsub * ncc, nsteps = nq * KH;
    const uint16_t* inb = P.in.p + o * P.in.s_outer;

    // chunk-independent staging offsets of this thread's P entries (pix, k4): int32 (host-checked)
    int poff[NPE];
    uint32_t pok = 0u;
#pragma unroll
    for (int u = 0; u < NPE; ++u) {
        const int e = t + u * 256, pix = e >> 2, k4 = e & 3, hr = pix / HC, hc = pix - hr * HC;
        const int ir = r0 + hr - P.ph, ic = c0 + hc - P.pw;
        const bool ok = e < 4 * HR * HC && ir >= 0 && ir < P.in.rin && ic >= 0 && ic < P.in.cols_in;
        poff[u] = ok ? (int)(ir * P.in.s_row + ic * P.in.s_col) + k4 * 8 : 0;
        pok |= ok ? 1u << u : 0u;
    }
    const uint16_t* wbase = P.w;   // the current 64-channel output tile's weights
    const uint16_t* pbase = inb;   // the current chunk's source (sub-pixel offset + 32-channel block)
#define PC_LOADP(q_)                                                                                        \
    {                                                                                                       \
        const int sub_ = (q_) / ncc, cc_ = (q_) - sub_ * ncc;                                               \
        pbase = inb + P.in.sub_off[sub_] + cc_ * 32;                                                        \
        _Pragma("unroll") for (int u = 0; u < NPE; ++u) preg[u] =                                           \
            (pok >> u) & 1u ? *reinterpret_cast<const u4v*>(pbase + poff[u]) : u4v{0u, 0u, 0u, 0u};         \
    }
#define PC_STOREP(buf_)                                                                                     \
    _Pragma("unroll") for (int u = 0; u < NPE; ++u) {                                                       \
        const int e_ = t + u * 256;                                                                         \
        if (e_ < 4 * HR * HC)                                                                               \
            *reinterpret_cast<u4v*>(smem + (buf_) * PB + ((e_ & 3) * NP + (e_ >> 2)) * 16) = preg[u];      \
    }
    // a step's weights straight into LDS buffer buf_ (LDS-DMA, no VGPRs: each wave-instruction writes
    // 1 KB, its 64 lanes' 16 bytes in lane order, and the image is the source's byte order)
#define PC_DMAW(s_, buf_)                                                                                   \
    {                                                                                                       \
        const u4v* src_ = reinterpret_cast<const u4v*>(wbase + (size_t)(s_) * KW * 2048) + t;               \
        _Pragma("unroll") for (int u = 0; u < KW; ++u) __builtin_amdgcn_global_load_lds(                    \
            src_ + u * 256, (__attribute__((address_space(3))) void*)(smem + 2 * PB + (buf_) * WB + u * 4096 + wv * 1024), \
            16, 0, 0);                                                                                      \
    }

    // output tiles nb0 .. nb0 + nbw - 1 in turn; with nbw > 1 every input chunk (nq <= 2) is staged once,
    // by the first tile, into P buffer q, and the later tiles stage only their weights
#pragma unroll 1
    for (int nbi = 0; nbi < A.nbw; ++nbi) {
    const int nb = nb0 + nbi;
    if (nb * 64 >= P.cop) break;   // whole workgroup
    const bool first = nbi == 0;
    wbase = P.w + (size_t)nb * nq * KH * KW * 2048;
    f4 acc[4][4];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[f][g] = f4{0.f, 0.f, 0.f, 0.f};

    {
        u4v preg[NPE];
        PC_DMAW(0, 0);
        if (first) {
            PC_LOADP(0);
            PC_STOREP(0);
        }
    }
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
        const int q = s / KH, a = s - q * KH;
        // the chunk's last step: stage the next chunk (resident chunks only once)
        const bool nxq = first && s + 1 < nsteps && a == KH - 1;
        // staging registers local to the step (loaded at its top, stored at its end): arrays carried
        // across iterations were demoted to scratch
        u4v preg[NPE];
        // the next step's weights into the other buffer (read by step s - 1, which every wave has left)
        if (s + 1 < nsteps) PC_DMAW(s + 1, (s + 1) & 1);
        if (nxq) PC_LOADP(q + 1);
        // the loads above go out before the MFMAs (the scheduler otherwise sinks them to their
        // LDS stores at the end of the step and the step waits out their whole latency)
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t* Wl = smem + 2 * PB + (s & 1) * WB + (kq * 64 + l15) * 16;
        const uint8_t* Pl0 = smem + (q & 1) * PB + (kq * NP + (wv + a) * HC + l15) * 16;
        // operand fragments double-buffered in registers: tap column b + 1's reads are in flight while
        // b's MFMAs run (one wave per SIMD: nothing else hides the LDS latency)
        bf8 Bf[2][4], Af[2][4];
#pragma unroll
        for (int g = 0; g < 4; ++g) Bf[0][g] = *reinterpret_cast<const bf8*>(Wl + (16 * g) * 16);
#pragma unroll
        for (int f = 0; f < 4; ++f) Af[0][f] = *reinterpret_cast<const bf8*>(Pl0 + (16 * f) * 16);
#pragma unroll
        for (int b = 0; b < KW; ++b) {
            const int u = b & 1;
            if (b + 1 < KW) {
#pragma unroll
                for (int g = 0; g < 4; ++g) Bf[u ^ 1][g] = *reinterpret_cast<const bf8*>(Wl + ((b + 1) * 256 + 16 * g) * 16);
#pragma unroll
                for (int f = 0; f < 4; ++f) Af[u ^ 1][f] = *reinterpret_cast<const bf8*>(Pl0 + (16 * f + b + 1) * 16);
            }
            __builtin_amdgcn_sched_barrier(0);   // keep b + 1's reads ahead of b's MFMAs
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[u][f], Bf[u][g], acc[f][g], 0, 0, 0);
        }
        if (nxq) PC_STOREP((q + 1) & 1);
        __syncthreads();   // with the DMA in flight: vmcnt(0) first
    }
    // epilogue: accumulators -> LDS [wave][px][n] (row stride 68 floats, after the P buffers, over the
    // weight buffers) -> 8-channel runs
    {
        float* ep = reinterpret_cast<float*>(smem + 2 * PB) + wv * 64 * 68;
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int r = 0; r < 4; ++r) ep[(16 * f + 4 * kq + r) * 68 + 16 * g + l15] = acc[f][g][r];
    }
    __syncthreads();
    const int Y = r0 + wv;
    const float* ep = reinterpret_cast<const float*>(smem + 2 * PB) + wv * 64 * 68;
#pragma unroll 1
    for (int i = 0; i < (Y < P.rows ? 8 : 0); ++i) {
        const int item = lane + 64 * i, px = item >> 3, n0 = (item & 7) * 8, X = c0 + px;
        if (X >= P.cols) continue;
        const float4 va = *reinterpret_cast<const float4*>(ep + px * 68 + n0);
        const float4 vb = *reinterpret_cast<const float4*>(ep + px * 68 + n0 + 4);
        float v[8] = {va.x, va.y, va.z, va.w, vb.x, vb.y, vb.z, vb.w};
        const int n = nb * 64 + n0;
        if (P.mode == OUT_F32) {
            float* dst = static_cast<float*>(P.out) + o * P.o_outer + Y * P.o_row + X * P.o_col + n;
            *reinterpret_cast<float4*>(dst) = va;
            *reinterpret_cast<float4*>(dst + 4) = vb;
            continue;
        }
        if (n >= P.co) continue;
        const int pk = P.pk;
        if (P.mode == OUT_Y) {
            const int rc = row_class(Y, P.Ho, pk), cc = row_class(X, P.Wo, pk);
            const float* bt = P.bt + (rc * (2 * pk + 1) + cc) * P.C + n;
            const int C = P.C;
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] += bt[j];
            if (Y < pk) {
                const float* e = P.e[0] + (o * P.Wo + X) * P.ecs + (pk - 1 - Y) * C + n;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] -= e[j];
            }
            if (Y >= P.Ho - pk) {
                const float* e = P.e[1] + (o * P.Wo + X) * P.ecs + (P.Ho - 1 - Y) * C + n;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] -= e[j];
            }
            if (X < pk) {
                const float* e = P.e[2] + (o * P.Ho + Y) * P.ecs + (pk - 1 - X) * C + n;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] -= e[j];
            }
            if (X >= P.Wo - pk) {
                const float* e = P.e[3] + (o * P.Ho + Y) * P.ecs + (P.Wo - 1 - X) * C + n;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] -= e[j];
            }
            uint16_t* dst = static_cast<uint16_t*>(P.out) + o * P.o_outer + Y * P.o_row + X * P.o_col + n;
            *reinterpret_cast<uint4*>(dst) = make_uint4(f2bf(v[0]) | f2bf(v[1]) << 16, f2bf(v[2]) | f2bf(v[3]) << 16,
                                                       f2bf(v[4]) | f2bf(v[5]) << 16, f2bf(v[6]) | f2bf(v[7]) << 16);
        } else {   // OUT_DX: packed channel kin = s C + c of P pixel (Y, X) -> x pixel (2Y + i, 2X + j), s = 2 i + j
            const float* e[4] = {Y == 0 ? P.e[0] + (o * P.Wo + X) * P.ecs + n : nullptr,
                                 Y == P.Ho - 1 ? P.e[1] + (o * P.Wo + X) * P.ecs + n : nullptr,
                                 X == 0 ? P.e[2] + (o * P.Ho + Y) * P.ecs + n : nullptr,
                                 X == P.Wo - 1 ? P.e[3] + (o * P.Ho + Y) * P.ecs + n : nullptr};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (e[k]) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] -= e[k][j];
                }
            const int sub = n / P.C, c = n - sub * P.C;
            uint16_t* dst = static_cast<uint16_t*>(P.out) + o * P.o_outer + (2 * Y + (sub >> 1)) * P.o_row +
                            (2 * X + (sub & 1)) * P.o_col + c;
            *reinterpret_cast<uint4*>(dst) = make_uint4(f2bf(v[0]) | f2bf(v[1]) << 16, f2bf(v[2]) | f2bf(v[3]) << 16,
                                                       f2bf(v[4]) | f2bf(v[5]) << 16, f2bf(v[6]) | f2bf(v[7]) << 16);
        }
    }
    __syncthreads();   // the epilogue tile overlays the weight buffers the next output tile stages into
    }
#undef PC_LOADP
#undef PC_STOREP
#undef PC_DMAW
}

// --------------------------------------------------------------------------------------------
// weight gradient: part[split][a][mb][kb][m 64][b KW][kin 64] = sum over the split's pixels p of
// G[p][mb*64 + m] * IN[p + (a - ph, b - pw)][kb*64 + kin].  Pixel blocks are 64 columns of one
// output row; per block the G tile [64 px][64 ch] and the IN tile [64 + KW - 1 px][64 ch] are
// staged into LDS images with 128-byte rows whose 16-byte chunks are XOR-swizzled by the row, so
// that the ds_read_b64_tr_b16 operand reads (4 pixel rows x 16 channels per 16-lane group, 8
// rows per 32-lane half) hit 8 distinct bank octets.  Wave w owns kin columns 16w..16w+15: KW x 4
// accumulator tiles (b, m tile).
struct WProb {
    Geo in;
    const uint16_t* g;
    int64_t g_outer, g_row, g_col;
    int gc;                  // G channels
    int outer, rows, cols;   // the pixels summed over
    int ph, pw;
    int nsplit;
    float* part;
};

struct WArgs {
    WProb p[MAXPROB];
    int nprob, KH, nmb, nkb;
};

__device__ __forceinline__ int wswz(int px) { return (((px >> 1) & 1) | (((px >> 3) & 1) << 1)) << 1; }

template <int KW>
__global__ __launch_bounds__(256, 2) void k_pc_wgrad(const WArgs A) {
    constexpr int TX = 64, HC = TX + KW - 1;
    constexpr int GB = 64 * 128, IB = HC * 128;
    constexpr int NGE = 2, NIE = (HC * 8 + 255) / 256;
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * (GB + IB)];
    const WProb& P = A.p[blockIdx.z];
    const int split = blockIdx.x;
    if (split >= P.nsplit) return;
    const int nmk = A.nmb * A.nkb, a = blockIdx.y / nmk, mk = blockIdx.y - a * nmk, mb = mk / A.nkb,
              kb = mk - mb * A.nkb;
    const int ncb = (P.cols + TX - 1) / TX, nblk = P.outer * P.rows * ncb;
    const int bi0 = (int)((int64_t)split * nblk / P.nsplit), bi1 = (int)((int64_t)(split + 1) * nblk / P.nsplit);
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int ncc = P.in.cin >> 5, nq = P.in.nsub * ncc;

    // staging loads: unconditional, from the tile's own address or (out of range) from the image
    // base, the zero selected at the LDS store — a load under a lane-divergent branch made the
    // wait-count pass drain every earlier load before the next one (vmcnt(0) between the loads)
    uint4 greg[NGE], ireg[NIE];
    uint32_t gok = 0u, iok = 0u;
    // block-independent parts of this thread's staging entries, once: the channel offset of each IN
    // entry (sub-pixel plane + 32-channel chunk: a per-lane index into sub_off, selected here rather
    // than per load) and which entries exist
    int64_t ich[NIE];
    uint32_t iq_ok = 0u, g_ok = 0u;
#pragma unroll
    for (int u = 0; u < NIE; ++u) {
        const int e = t + u * 256, ch = e & 7, q = kb * 2 + (ch >> 2);
        const int sub = q / ncc, cc = q - sub * ncc;
        const int64_t so = sub == 0 ? P.in.sub_off[0] : sub == 1 ? P.in.sub_off[1] : sub == 2 ? P.in.sub_off[2]
                                                                                                 : P.in.sub_off[3];
        ich[u] = so + cc * 32 + (ch & 3) * 8;
        iq_ok |= (e < HC * 8 && q < nq) ? 1u << u : 0u;
    }
#pragma unroll
    for (int u = 0; u < NGE; ++u) g_ok |= (mb * 64 + ((t + u * 256) & 7) * 8 < P.gc) ? 1u << u : 0u;
    auto load = [&](int bi) {
        const int cb = bi % ncb, rr = bi / ncb, r = rr % P.rows, o = rr / P.rows, c0 = cb * TX;
        const uint16_t* gb = P.g + o * P.g_outer;
        gok = 0u;
#pragma unroll
        for (int u = 0; u < NGE; ++u) {
            const int e = t + u * 256, px = e >> 3, ch = e & 7;
            const bool ok = ((g_ok >> u) & 1u) && c0 + px < P.cols;
            const int64_t off = ok ? r * P.g_row + (c0 + px) * P.g_col + mb * 64 + ch * 8 : 0;
            greg[u] = *reinterpret_cast<const uint4*>(gb + off);
            gok |= ok ? 1u << u : 0u;
        }
        const int ir = r + a - P.ph;
        const bool row_ok = ir >= 0 && ir < P.in.rin;   // wave-uniform
        const uint16_t* ib = P.in.p + o * P.in.s_outer + (row_ok ? ir : 0) * P.in.s_row;
        iok = 0u;
#pragma unroll
        for (int u = 0; u < NIE; ++u) {
            const int e = t + u * 256, px = e >> 3, ic = c0 + px - P.pw;
            const bool ok = row_ok && ((iq_ok >> u) & 1u) && ic >= 0 && ic < P.in.cols_in;
            const int64_t off = ok ? ic * P.in.s_col + ich[u] : 0;
            ireg[u] = *reinterpret_cast<const uint4*>(ib + off);
            iok |= ok ? 1u << u : 0u;
        }
    };
    auto store = [&](int buf) {
        uint8_t* gs = smem + buf * (GB + IB);
        uint8_t* is = gs + GB;
#pragma unroll
        for (int u = 0; u < NGE; ++u) {
            const int e = t + u * 256, px = e >> 3, ch = e & 7;
            const uint32_t m = (gok >> u) & 1u ? 0xffffffffu : 0u;   // a value mask, not a select of two arrays
            *reinterpret_cast<uint4*>(gs + px * 128 + ((ch ^ wswz(px)) << 4)) =
                make_uint4(greg[u].x & m, greg[u].y & m, greg[u].z & m, greg[u].w & m);
        }
#pragma unroll
        for (int u = 0; u < NIE; ++u) {
            const int e = t + u * 256, px = e >> 3, ch = e & 7;
            const uint32_t m = (iok >> u) & 1u ? 0xffffffffu : 0u;
            if (e < HC * 8)
                *reinterpret_cast<uint4*>(is + px * 128 + ((ch ^ wswz(px)) << 4)) =
                    make_uint4(ireg[u].x & m, ireg[u].y & m, ireg[u].z & m, ireg[u].w & m);
        }
    };

    f4 acc[KW][4];
#pragma unroll
    for (int b = 0; b < KW; ++b)
#pragma unroll
        for (int f = 0; f < 4; ++f) acc[b][f] = f4{0.f, 0.f, 0.f, 0.f};

    // tr-read lane roles: group gq = lane >> 4 takes pixel rows 8 gq .. 8 gq + 7; lane 4 q + p of the
    // group supplies row q (+ 4 for the second read), columns 4 p .. 4 p + 3 of the 16-column block
    const int gq = lane >> 4, qr = (lane & 15) >> 2, pc = lane & 3;
    if (bi0 < bi1) {
        load(bi0);
        store(0);
    }
    __syncthreads();
    for (int bi = bi0; bi < bi1; ++bi) {
        const int buf = (bi - bi0) & 1;
        const bool nx = bi + 1 < bi1;
        if (nx) load(bi + 1);
        __builtin_amdgcn_sched_barrier(0);   // the next block's loads go out before this block's MFMAs
        uint8_t* gs = smem + buf * (GB + IB);
        uint8_t* is = gs + GB;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf8 Af[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const int ch = 2 * f + (pc >> 1);
                const int px0 = ks * 32 + 8 * gq + qr, px1 = px0 + 4;
                typedef __attribute__((address_space(3))) s4 lds_s4;
                const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s4*)(gs + px0 * 128 + ((ch ^ wswz(px0)) << 4) + 8 * (pc & 1)));
                const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s4*)(gs + px1 * 128 + ((ch ^ wswz(px1)) << 4) + 8 * (pc & 1)));
                Af[f] = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
#pragma unroll
            for (int b = 0; b < KW; ++b) {
                const int ch = 2 * wv + (pc >> 1);
                const int px0 = ks * 32 + 8 * gq + qr + b, px1 = px0 + 4;
                typedef __attribute__((address_space(3))) s4 lds_s4;
                const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s4*)(is + px0 * 128 + ((ch ^ wswz(px0)) << 4) + 8 * (pc & 1)));
                const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                    (lds_s4*)(is + px1 * 128 + ((ch ^ wswz(px1)) << 4) + 8 * (pc & 1)));
                const bf8 Bf = bf8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
                for (int f = 0; f < 4; ++f) acc[b][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Af[f], Bf, acc[b][f], 0, 0, 0);
            }
        }
        if (nx) store(buf ^ 1);
        __syncthreads();
    }
    // partials: [m][b][kin] of this (split, a, mb, kb) block; D row = m (4 per lane), column = kin
    float* dst = P.part + ((((int64_t)split * A.KH + a) * A.nmb + mb) * A.nkb + kb) * (64 * KW * 64);
#pragma unroll
    for (int b = 0; b < KW; ++b)
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[((16 * f + 4 * gq + r) * KW + b) * 64 + 16 * wv + (lane & 15)] = acc[b][f][r];
}

// out[(m * KH + a) * KW + b][kin] (m < gc, kin < Kin) = scale * sum over splits, fixed order
struct RProb {
    const float* part;
    float* out;
    int nsplit;
    float scale;
};
struct RArgs {
    RProb p[MAXPROB];
    int KH, KW, nmb, nkb, gc, Kin;
};
__global__ __launch_bounds__(256) void k_pc_wreduce(const RArgs A) {
    const RProb& P = A.p[blockIdx.y];
    const int64_t n = (int64_t)A.gc * A.KH * A.KW * A.Kin;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int kin = (int)(i % A.Kin);
    int64_t r = i / A.Kin;
    const int b = (int)(r % A.KW);
    r /= A.KW;
    const int a = (int)(r % A.KH);
    const int m = (int)(r / A.KH);
    const int mb = m >> 6, kb = kin >> 6;
    const int64_t blk = 64 * A.KW * 64, stride = (int64_t)A.KH * A.nmb * A.nkb * blk;
    const float* src = P.part + ((int64_t)(a * A.nmb + mb) * A.nkb + kb) * blk + ((m & 63) * A.KW + b) * 64 + (kin & 63);
    float s = 0.f;
    for (int sp = 0; sp < P.nsplit; ++sp) s += src[sp * stride];
    P.out[i] = P.scale * s;
}

// --------------------------------------------------------------------------------------------
// corner terms.  Corner cn = TL, BL, TR, BR: P corner pixel (Yp, Xp); its frame pixels
// (Y(i), X(j)) = (top ? pk-1-i : Ho-1-i, left ? pk-1-j : Wo-1-j), i, j < pk.
struct CornerArgs {
    const uint16_t* x;
    int64_t xs0, xs2, xs3;
    const uint16_t* dy;
    int64_t ys0, ys2, ys3;
    const float* w;   // [4][pk][pk][C][4C]
    float* eL;        // edge buffers L / R [b][pos][ecs]
    float* eR;
    int ecs;
    float* dw;        // [4][pk][pk][C][4C]
    int B, C, pk, Ho, Wo;
};

__device__ __forceinline__ float p_corner(const CornerArgs& A, int cn, int b, int kin) {
    const bool top = (cn & 1) == 0, left = cn < 2;
    const int Yp = top ? 0 : A.Ho - 1, Xp = left ? 0 : A.Wo - 1, s = kin / A.C, c = kin - s * A.C;
    return bf2f(A.x[b * A.xs0 + (2 * Yp + (s >> 1)) * A.xs2 + (2 * Xp + (s & 1)) * A.xs3 + c]);
}
__device__ __forceinline__ float dy_at(const CornerArgs& A, int cn, int b, int i, int j, int m) {
    const bool top = (cn & 1) == 0, left = cn < 2;
    const int Y = top ? A.pk - 1 - i : A.Ho - 1 - i, X = left ? A.pk - 1 - j : A.Wo - 1 - j;
    return bf2f(A.dy[b * A.ys0 + Y * A.ys2 + X * A.ys3 + m]);
}

// forward: e{L,R}[b][Y(i)][j C + m] -= sum_kin w[cn][i][j][m][kin] P_cn[b][kin].  A workgroup per
// (cn, i, j, 4 channels m): the corner pixel's packed channels of the batch are staged in LDS; wave
// w owns m = 4 mb + w, its lanes split kin (coalesced weight reads) and every image is reduced
// across the wave at the end.
constexpr int CORNER_MAXB = 16;
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__global__ __launch_bounds__(256) void k_pc_corner_fwd(const CornerArgs A) {
    extern __shared__ float sp[];   // [B][K]
    const int pk = A.pk, K = 4 * A.C, nmb = (A.C + 3) / 4;
    const int mb = blockIdx.x % nmb, r = blockIdx.x / nmb, ij = r % (pk * pk), cn = r / (pk * pk), i = ij / pk, j = ij % pk;
    for (int e = threadIdx.x; e < A.B * K; e += 256) sp[e] = p_corner(A, cn, e / K, e % K);
    __syncthreads();
    const int lane = threadIdx.x & 63, m = mb * 4 + (threadIdx.x >> 6);
    if (m >= A.C) return;
    const float* w = A.w + (((int64_t)(cn * pk + i) * pk + j) * A.C + m) * K;
    float acc[CORNER_MAXB];
#pragma unroll
    for (int b = 0; b < CORNER_MAXB; ++b) acc[b] = 0.f;
    for (int kin = lane; kin < K; kin += 64) {
        const float wv = w[kin];
#pragma unroll
        for (int b = 0; b < CORNER_MAXB; ++b)
            if (b < A.B) acc[b] += wv * sp[b * K + kin];
    }
    const bool top = (cn & 1) == 0, left = cn < 2;
    const int Y = top ? pk - 1 - i : A.Ho - 1 - i;
    float* eo = left ? A.eL : A.eR;
#pragma unroll
    for (int b = 0; b < CORNER_MAXB; ++b)
        if (b < A.B) {
            const float v = wave_sum(acc[b]);
            if (lane == 0) eo[((int64_t)b * A.Ho + Y) * A.ecs + j * A.C + m] -= v;
        }
}

// backward: d{L,R}[b][Yp][kin] -= sum_{i, j, m} w[cn][i][j][m][kin] dy[b][Y(i)][X(j)][m].  A workgroup
// per (cn, 64 kin): the corner frame's dy values of the batch are staged in LDS; lane = kin
// (coalesced weight reads), the 4 waves split the (i, j, m) rows, fixed-order combine in LDS.
__global__ __launch_bounds__(256) void k_pc_corner_bwd(const CornerArgs A) {
    extern __shared__ float sd[];   // [B][pk pk C] then the 4-wave combine [4][B][64]
    const int pk = A.pk, K = 4 * A.C, nkb = (K + 63) / 64, cn = blockIdx.x / nkb, kb = blockIdx.x % nkb;
    const int nv = pk * pk * A.C;
    for (int e = threadIdx.x; e < A.B * nv; e += 256) {
        const int b = e / nv, r = e % nv, m = r % A.C, ij = r / A.C;
        sd[e] = dy_at(A, cn, b, ij / pk, ij % pk, m);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, kin = kb * 64 + lane;
    float acc[CORNER_MAXB];
#pragma unroll
    for (int b = 0; b < CORNER_MAXB; ++b) acc[b] = 0.f;
    if (kin < K) {
        const float* w = A.w + (int64_t)cn * nv * K + kin;
        const int r0 = wv * nv / 4, r1 = (wv + 1) * nv / 4;
        for (int r = r0; r < r1; ++r) {
            const float wvv = w[(int64_t)r * K];
#pragma unroll
            for (int b = 0; b < CORNER_MAXB; ++b)
                if (b < A.B) acc[b] += wvv * sd[b * nv + r];
        }
    }
    float* cmb = sd + A.B * nv;
    __syncthreads();
#pragma unroll
    for (int b = 0; b < CORNER_MAXB; ++b)
        if (b < A.B) cmb[(wv * A.B + b) * 64 + lane] = acc[b];
    __syncthreads();
    if (wv == 0 && kin < K) {
        const bool top = (cn & 1) == 0, left = cn < 2;
        const int Yp = top ? 0 : A.Ho - 1;
        float* eo = left ? A.eL : A.eR;
        for (int b = 0; b < A.B; ++b) {
            const float v = (cmb[(0 * A.B + b) * 64 + lane] + cmb[(1 * A.B + b) * 64 + lane]) +
                            (cmb[(2 * A.B + b) * 64 + lane] + cmb[(3 * A.B + b) * 64 + lane]);
            eo[((int64_t)b * A.Ho + Yp) * A.ecs + kin] -= v;
        }
    }
}

// weight gradient: dw[cn][i][j][m][kin] = sum_b dy[b][Y(i)][X(j)][m] P_cn[b][kin]
__global__ __launch_bounds__(256) void k_pc_corner_wgrad(const CornerArgs A) {
    const int pk = A.pk, K = 4 * A.C;
    const int64_t n = (int64_t)4 * pk * pk * A.C * K;
    const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= n) return;
    const int kin = (int)(id % K);
    int64_t r = id / K;
    const int m = (int)(r % A.C);
    r /= A.C;
    const int j = (int)(r % pk);
    r /= pk;
    const int i = (int)(r % pk), cn = (int)(r / pk);
    float s = 0.f;
    for (int b = 0; b < A.B; ++b) s += dy_at(A, cn, b, i, j, m) * p_corner(A, cn, b, kin);
    A.dw[id] = s;
}

// bias-table gradient, stage 1: part[b][Y][cc][m] = sum over X of class cc of dy[b][Y][X][m]
// (one workgroup per (b, Y); 8-channel groups x X lanes, fixed-order LDS reduction)
__global__ __launch_bounds__(256) void k_pc_bt_rows(const uint16_t* dy, int64_t ys0, int64_t ys2, int64_t ys3, int C,
                                                    int Ho, int Wo, int pk, float* part) {
    __shared__ float red[256 * 8];
    const int b = blockIdx.x / Ho, Y = blockIdx.x - b * Ho, ncls = 2 * pk + 1;
    const int ncg = C >> 3, t = threadIdx.x;
    const int nxl = 256 / ncg, cg = t % ncg, xl = t / ncg;
    for (int cls = 0; cls < ncls; ++cls) {
        const int x0 = cls < pk ? cls : (cls > pk ? Wo - 1 - (2 * pk - cls) : pk);
        const int x1 = cls == pk ? Wo - pk : x0 + 1;
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (xl < nxl)
            for (int X = x0 + xl; X < x1; X += nxl) {
                const uint4 u = *reinterpret_cast<const uint4*>(dy + b * ys0 + Y * ys2 + X * ys3 + cg * 8);
                const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    s[2 * k] += __uint_as_float(w[k] << 16);
                    s[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
                }
            }
#pragma unroll
        for (int k = 0; k < 8; ++k) red[t * 8 + k] = s[k];
        __syncthreads();
        for (int m = t; m < C; m += 256) {
            const int g = m >> 3, k = m & 7;
            float v = 0.f;
            for (int l = 0; l < nxl; ++l) v += red[(l * ncg + g) * 8 + k];
            part[(((int64_t)b * Ho + Y) * ncls + cls) * C + m] = v;
        }
        __syncthreads();
    }
}

// stage 2: dbt[rc][cc][m] = sum over b and the rows Y of class rc: one workgroup per (rc, cc,
// 64-channel block), 4 row groups x 64 channels, fixed-order combine
__global__ __launch_bounds__(256) void k_pc_bt_cols(const float* part, int B, int C, int Ho, int pk, float* dbt) {
    __shared__ float red[4][64];
    const int ncls = 2 * pk + 1, ncb = (C + 63) / 64;
    const int cb = blockIdx.x % ncb, cc = (blockIdx.x / ncb) % ncls, rc = blockIdx.x / (ncb * ncls);
    const int m = cb * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;
    const int y0 = rc < pk ? rc : (rc > pk ? Ho - 1 - (2 * pk - rc) : pk);
    const int y1 = rc == pk ? Ho - pk : y0 + 1, nrow = B * (y1 - y0);
    float s = 0.f;
    if (m < C)
        for (int r = grp; r < nrow; r += 4) {
            const int b = r / (y1 - y0), Y = y0 + r % (y1 - y0);
            s += part[(((int64_t)b * Ho + Y) * ncls + cc) * C + m];
        }
    red[grp][threadIdx.x & 63] = s;
    __syncthreads();
    if (grp == 0 && m < C) {
        const int l = threadIdx.x;
        dbt[(rc * ncls + cc) * C + m] = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    }
}

// --------------------------------------------------------------------------------------------
// weight composition (forward) and its chain rule (backward).  The operands are the module's fp32
// parameters rounded to bf16 (autocast's casts); sums in fp32.
__device__ __forceinline__ float rbf(float v) { return bf2f((uint16_t)f2bf(v)); }

struct CompArgs {
    const float* W2;   // [C][d Kp][k][k]
    const float* w3;   // [d][27]
    const float* b3;   // [d] or null
    int C, d, k, Kp, pk, ke, copC, copE;
    uint16_t* wf;
    uint16_t* wb;
    uint16_t* ef[4];
    uint16_t* eb[4];
    float* corner;
    float* bt;
    float* bs;         // scratch [C][k][k]
};

// Weff[m][kin][a][b] = sum_{o, dz, dy, dx} W2[m][o Kp + kp + 1 - dz][a - dy][b - dx] w3[o][dz][dy][dx]
// (kp = 4 c + s for kin = s C + c), written into wf and (taps flipped) wb.  A thread owns one output
// row (m, kin, a): every W2 row it needs (o, dz, dy) is loaded once and spread over the KE columns.
template <int K>
__global__ __launch_bounds__(256) void k_pc_comp_main(const CompArgs A) {
    constexpr int KE = K + 2;
    __shared__ float sw[8 * 27];
    for (int i = threadIdx.x; i < A.d * 27; i += 256) sw[i] = rbf(A.w3[i]);
    __syncthreads();
    const int K4 = 4 * A.C;
    // thread order (m, a, s, c) with c fastest: consecutive threads read consecutive W2 channel rows
    const int64_t n = (int64_t)A.copC * KE * K4, id = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= n) return;
    const int c = (int)(id % A.C);
    int64_t r = id / A.C;
    const int s = (int)(r % 4);
    r /= 4;
    const int a = (int)(r % KE), m = (int)(r / KE), kin = s * A.C + c, kp = 4 * c + s;
    float acc[KE];
#pragma unroll
    for (int b = 0; b < KE; ++b) acc[b] = 0.f;
    if (m < A.C) {
        for (int o = 0; o < A.d; ++o)
#pragma unroll
            for (int dz = 0; dz < 3; ++dz) {
                const int kk = kp + 1 - dz;
                if (kk < 0 || kk >= A.Kp) continue;
                const float* w2 = A.W2 + ((int64_t)m * A.d * A.Kp + o * A.Kp + kk) * K * K;
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    const int i = a - dy;
                    if (i < 0 || i >= K) continue;
                    float row[K];
#pragma unroll
                    for (int j = 0; j < K; ++j) row[j] = rbf(w2[i * K + j]);
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx) {
                        const float wv = sw[o * 27 + dz * 9 + dy * 3 + dx];
#pragma unroll
                        for (int j = 0; j < K; ++j) acc[j + dx] += wv * row[j];
                    }
                }
            }
    }
    const int64_t fbase = (((int64_t)(m >> 6) * (K4 >> 5) + (kin >> 5)) * KE + a) * KE * 2048 +
                          (((kin >> 3) & 3) * 64 + (m & 63)) * 8 + (kin & 7);
#pragma unroll
    for (int b = 0; b < KE; ++b) A.wf[fbase + b * 2048] = (uint16_t)f2bf(acc[b]);
    if (m < A.C) {
        const int64_t bbase = (((int64_t)(kin >> 6) * (A.C >> 5) + (m >> 5)) * KE + (KE - 1 - a)) * KE * 2048 +
                              (((m >> 3) & 3) * 64 + (kin & 63)) * 8 + (m & 7);
#pragma unroll
        for (int b = 0; b < KE; ++b) A.wb[bbase + (KE - 1 - b) * 2048] = (uint16_t)f2bf(acc[b]);
    }
}

// edge lines: U_T[e] = tap row i = e of W2 with w3's dy = 2 plane, U_B[e] row pk+1+e with dy = 0,
// U_L / U_R the same for columns; column n = e C + m of ef, input channel n of eb (taps flipped).
// A thread owns the KE taps of one (edge, n, kin).
template <int K>
__global__ __launch_bounds__(256) void k_pc_comp_edges(const CompArgs A) {
    constexpr int KE = K + 2;
    __shared__ float sw[8 * 27];
    for (int i = threadIdx.x; i < A.d * 27; i += 256) sw[i] = rbf(A.w3[i]);
    __syncthreads();
    const int K4 = 4 * A.C, pk = A.pk, nE = pk * A.C;
    const int64_t n = (int64_t)4 * A.copE * K4, id = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= n) return;
    const int c = (int)(id % A.C);
    int64_t r = id / A.C;
    const int s = (int)(r % 4);
    r /= 4;
    const int nn = (int)(r % A.copE), edge = (int)(r / A.copE), kin = s * A.C + c, kp = 4 * c + s;
    float acc[KE];
#pragma unroll
    for (int q = 0; q < KE; ++q) acc[q] = 0.f;
    if (nn < nE) {
        const int e = nn / A.C, m = nn - e * A.C;
        const bool rowl = edge < 2;
        const int fixed = (edge & 1) ? pk + 1 + e : e, plane = (edge & 1) ? 0 : 2;
        for (int o = 0; o < A.d; ++o)
#pragma unroll
            for (int dz = 0; dz < 3; ++dz) {
                const int kk = kp + 1 - dz;
                if (kk < 0 || kk >= A.Kp) continue;
                const float* w2 = A.W2 + ((int64_t)m * A.d * A.Kp + o * A.Kp + kk) * K * K;
                float line[K];
#pragma unroll
                for (int v = 0; v < K; ++v) line[v] = rbf(rowl ? w2[fixed * K + v] : w2[v * K + fixed]);
#pragma unroll
                for (int t = 0; t < 3; ++t) {
                    const float wv = sw[o * 27 + dz * 9 + (rowl ? plane * 3 + t : t * 3 + plane)];
#pragma unroll
                    for (int v = 0; v < K; ++v) acc[v + t] += wv * line[v];
                }
            }
    }
    const int64_t fbase = ((int64_t)(nn >> 6) * (K4 >> 5) + (kin >> 5)) * KE * 2048 + (((kin >> 3) & 3) * 64 + (nn & 63)) * 8 +
                          (kin & 7);
#pragma unroll
    for (int sp = 0; sp < KE; ++sp) A.ef[edge][fbase + sp * 2048] = (uint16_t)f2bf(acc[sp]);
    if (nn < nE) {
        const int64_t bbase = ((int64_t)(kin >> 6) * (nE >> 5) + (nn >> 5)) * KE * 2048 + (((nn >> 3) & 3) * 64 + (kin & 63)) * 8 +
                              (nn & 7);
#pragma unroll
        for (int sp = 0; sp < KE; ++sp) A.eb[edge][bbase + (KE - 1 - sp) * 2048] = (uint16_t)f2bf(acc[sp]);
    }
}

// corners [cn][i][j][m][kin] (fp32) = sum_{o, dz} W2[m][o Kp + kp + 1 - dz][i'][j'] w3[o][dz][dyc][dxc]
__global__ __launch_bounds__(256) void k_pc_comp_corner(const CompArgs A) {
    const int k = A.k, K4 = 4 * A.C, pk = A.pk;
    const int64_t n = (int64_t)4 * pk * pk * A.C * K4, id = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (id >= n) return;
    const int kin = (int)(id % K4);
    int64_t r = id / K4;
    const int m = (int)(r % A.C);
    r /= A.C;
    const int j = (int)(r % pk);
    r /= pk;
    const int i = (int)(r % pk), cn = (int)(r / pk);
    const bool top = (cn & 1) == 0, left = cn < 2;
    const int ii = top ? i : pk + 1 + i, jj = left ? j : pk + 1 + j, tap = (top ? 2 : 0) * 3 + (left ? 2 : 0);
    const int s = kin / A.C, c = kin - s * A.C, kp = 4 * c + s;
    float v = 0.f;
    for (int o = 0; o < A.d; ++o)
        for (int dz = 0; dz < 3; ++dz) {
            const int kk = kp + 1 - dz;
            if (kk < 0 || kk >= A.Kp) continue;
            v += rbf(A.W2[((int64_t)m * A.d * A.Kp + o * A.Kp + kk) * k * k + ii * k + jj]) * rbf(A.w3[o * 27 + dz * 9 + tap]);
        }
    A.corner[id] = v;
}

// Bs[m][i][j] = sum_{o, kp} b3[o] W2[m][o Kp + kp][i][j]: one workgroup per (m, i, j), fixed-order tree
__global__ __launch_bounds__(256) void k_pc_comp_bias(const CompArgs A) {
    __shared__ float red[256];
    const int kk2 = A.k * A.k, m = blockIdx.x / kk2, ij = blockIdx.x - m * kk2, nch = A.d * A.Kp;
    float s = 0.f;
    for (int ch = threadIdx.x; ch < nch; ch += 256)
        s += rbf(A.b3[ch / A.Kp]) * rbf(A.W2[((int64_t)m * nch + ch) * kk2 + ij]);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) A.bs[blockIdx.x] = red[0];
}

__device__ __forceinline__ bool in_class(int i, int cls, int pk, int k) {
    const int lo = pk - cls > 0 ? pk - cls : 0, hi = 3 * pk - cls < k - 1 ? 3 * pk - cls : k - 1;
    return i >= lo && i <= hi;
}

// bt[rc][cc][m] = sum over the in-image taps (i in I(rc), j in J(cc)) of Bs[m][i][j]
__global__ __launch_bounds__(256) void k_pc_comp_bt(const CompArgs A) {
    const int pk = A.pk, k = A.k, ncls = 2 * pk + 1, n = ncls * ncls * A.C, id = blockIdx.x * 256 + threadIdx.x;
    if (id >= n) return;
    const int m = id % A.C, cc = (id / A.C) % ncls, rc = id / (A.C * ncls);
    float v = 0.f;
    if (A.b3)
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < k; ++j)
                if (in_class(i, rc, pk, k) && in_class(j, cc, pk, k)) v += A.bs[(m * k + i) * k + j];
    A.bt[id] = v;
}

struct CompBwdArgs {
    const float* W2;
    const float* w3;
    const float* b3;
    const float* dwm;   // [C][ke][ke][4C]
    const float* de;    // [4][pk][C][ke][4C]
    const float* dc;    // [4][pk][pk][C][4C]
    const float* dbt;   // [2pk+1][2pk+1][C]
    float* dW2;
    float* part;        // [d][nchunk][28]
    int C, d, k, Kp, pk, ke, nchunk;
};

// chain rule for one Conv3d feature o (blockIdx.y) over a chunk of W2 rows (m, kp, i): for each of
// the 27 taps the upstream row G[b] = dWeff[m][kp+dz-1][i+dy][b] (b < KE; + the edge-line and corner
// gradients whose composition used this (i, j, tap)); dW2[j] = sum_tap w3[o][tap] G[j+dx] +
// b3[o] dBs[m][i][j]; dw3[o][tap] and db3[o] accumulate W2 G / W2 dBs per thread, then a
// fixed-order workgroup tree.  Thread order (m, i, s, c), c fastest: consecutive threads read
// consecutive packed channels kin of the gradients.
template <int K>
__global__ __launch_bounds__(256) void k_pc_comp_bwd(const CompBwdArgs A) {
    constexpr int KE = K + 2;
    __shared__ float red[28][256];
    __shared__ float sw[27];
    const int o = blockIdx.y, t = threadIdx.x, pk = A.pk, K4 = 4 * A.C, ncls = 2 * pk + 1;
    if (t < 27) sw[t] = rbf(A.w3[o * 27 + t]);
    __syncthreads();
    const float b3o = A.b3 ? rbf(A.b3[o]) : 0.f;
    float acc[28];
#pragma unroll
    for (int q = 0; q < 28; ++q) acc[q] = 0.f;
    const int64_t nrow = (int64_t)A.C * K * A.Kp;
    const int64_t e0 = nrow * blockIdx.x / A.nchunk, e1 = nrow * (blockIdx.x + 1) / A.nchunk;
    for (int64_t e = e0 + t; e < e1; e += 256) {
        const int c = (int)(e % A.C);
        int64_t r = e / A.C;
        const int s = (int)(r % 4);
        r /= 4;
        const int i = (int)(r % K), m = (int)(r / K), kp = 4 * c + s;
        const int64_t w2i = ((int64_t)m * A.d * A.Kp + o * A.Kp + kp) * K * K + i * K;
        float w[K], g[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            w[j] = rbf(A.W2[w2i + j]);
            float dbs = 0.f;
            for (int rc = 0; rc < ncls; ++rc)
                if (in_class(i, rc, pk, K))
                    for (int cc = 0; cc < ncls; ++cc)
                        if (in_class(j, cc, pk, K)) dbs += A.dbt[(rc * ncls + cc) * A.C + m];
            g[j] = b3o * dbs;
            acc[27] += w[j] * dbs;
        }
#pragma unroll
        for (int dz = 0; dz < 3; ++dz) {
            const int kk = kp + dz - 1;
            if (kk < 0 || kk >= A.Kp) continue;
            const int kin = (kk & 3) * A.C + (kk >> 2);
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                float G[KE];
                const float* src = A.dwm + ((int64_t)m * KE + i + dy) * KE * K4 + kin;
#pragma unroll
                for (int bb = 0; bb < KE; ++bb) G[bb] = src[bb * K4];
                if (dy == 2 && i < pk) {           // edge T line e = i (its taps run over b = j + dx)
                    const float* u = A.de + (((int64_t)0 * pk + i) * A.C + m) * KE * K4 + kin;
#pragma unroll
                    for (int bb = 0; bb < KE; ++bb) G[bb] += u[bb * K4];
                }
                if (dy == 0 && i > pk) {           // edge B line e = i - pk - 1
                    const float* u = A.de + (((int64_t)1 * pk + i - pk - 1) * A.C + m) * KE * K4 + kin;
#pragma unroll
                    for (int bb = 0; bb < KE; ++bb) G[bb] += u[bb * K4];
                }
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const int tap = dz * 9 + dy * 3 + dx;
                    float at = 0.f;
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        float Gj = G[j + dx];
                        // edge L / R lines (their taps run over i + dy) and corners, for this (i, j, tap)
                        if (dx == 2 && j < pk) Gj += A.de[((((int64_t)2 * pk + j) * A.C + m) * KE + i + dy) * K4 + kin];
                        if (dx == 0 && j > pk) Gj += A.de[((((int64_t)3 * pk + j - pk - 1) * A.C + m) * KE + i + dy) * K4 + kin];
                        if (dy == 2 && dx == 2 && i < pk && j < pk)
                            Gj += A.dc[((((int64_t)0 * pk + i) * pk + j) * A.C + m) * K4 + kin];
                        if (dy == 0 && dx == 2 && i > pk && j < pk)
                            Gj += A.dc[((((int64_t)1 * pk + i - pk - 1) * pk + j) * A.C + m) * K4 + kin];
                        if (dy == 2 && dx == 0 && i < pk && j > pk)
                            Gj += A.dc[((((int64_t)2 * pk + i) * pk + j - pk - 1) * A.C + m) * K4 + kin];
                        if (dy == 0 && dx == 0 && i > pk && j > pk)
                            Gj += A.dc[((((int64_t)3 * pk + i - pk - 1) * pk + j - pk - 1) * A.C + m) * K4 + kin];
                        g[j] += sw[tap] * Gj;
                        at += w[j] * Gj;
                    }
                    acc[tap] += at;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < K; ++j) A.dW2[w2i + j] = g[j];
    }
#pragma unroll
    for (int q = 0; q < 28; ++q) red[q][t] = acc[q];
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w)
#pragma unroll
            for (int q = 0; q < 28; ++q) red[q][t] += red[q][t + w];
        __syncthreads();
    }
    if (t < 28) A.part[((int64_t)o * A.nchunk + blockIdx.x) * 28 + t] = red[t][0];
}

__global__ __launch_bounds__(256) void k_pc_comp_bwd_red(const float* part, int d, int nchunk, float* dw3, float* db3) {
    const int id = blockIdx.x * 256 + threadIdx.x;
    if (id >= d * 28) return;
    const int o = id / 28, q = id - o * 28;
    float s = 0.f;
    for (int c = 0; c < nchunk; ++c) s += part[((int64_t)o * nchunk + c) * 28 + q];
    if (q < 27) dw3[o * 27 + q] = s;
    else if (db3) db3[o] = s;
}

// --------------------------------------------------------------------------------------------
struct Shape {
    int B, C, H, W, k, pk, ke, pe, Ho, Wo, Kin, copC, copE;
};

Shape shape_of(const psfm_pc_desc* t) {
    Shape s;
    s.B = t->B, s.C = t->C, s.H = t->H, s.W = t->W, s.k = t->k;
    s.pk = t->k / 2, s.ke = t->k + 2, s.pe = s.pk + 1, s.Ho = t->H / 2, s.Wo = t->W / 2, s.Kin = 4 * t->C;
    s.copC = (s.C + 63) & ~63;
    s.copE = (s.pk * s.C + 63) & ~63;
    return s;
}

int check_desc(const psfm_pc_desc* t) {
    if (!t) return fail(-1, "null descriptor");
    const Shape s = shape_of(t);
    if (s.B < 1 || s.C < 32 || s.C % 32 || s.C > 1024) return fail(-1, "C must be a multiple of 32 (32..1024)");
    if (s.H % 2 || s.W % 2) return fail(-1, "H and W must be even");
    if (t->k != 3 && t->k != 5) return fail(-1, "k must be 3 or 5");
    if (t->d != 4 && t->d != 8) return fail(-1, "d must be 4 or 8");
    if (s.Ho < 2 * s.pk + 1 || s.Wo < 2 * s.pk + 1) return fail(-1, "image smaller than the kernel frame");
    // the corner kernels stage one corner of the batch in (dynamic) LDS: <= 64 KB
    if (s.B > CORNER_MAXB || (int64_t)s.B * s.Kin * 4 > 65536 ||
        ((int64_t)s.B * s.pk * s.pk * s.C + 4 * s.B * 64) * 4 > 65536)
        return fail(-1, "B <= 16 and B * 4C * 4 bytes <= 64 KB (corner kernels stage the batch's corner pixels in LDS)");
    if (t->xs[1] != 1 || t->ys[1] != 1) return fail(-1, "x and y must be channels_last (channel stride 1)");
    for (int i : {0, 2, 3})
        if (t->xs[i] % 8 || t->ys[i] % 8 || t->xs[i] < 0 || t->ys[i] < 0)
            return fail(-1, "strides must be non-negative multiples of 8 elements");
    // every staging offset is int32 (relative to an image base, or across the batch for edge lines)
    const int64_t xmax = (int64_t)s.B * t->xs[0] + (int64_t)s.H * t->xs[2] + (int64_t)s.W * t->xs[3];
    const int64_t ymax = (int64_t)s.B * t->ys[0] + (int64_t)s.Ho * t->ys[2] + (int64_t)s.Wo * t->ys[3];
    if (xmax >= INT32_MAX || ymax >= INT32_MAX) return fail(-1, "tensor too large for int32 staging offsets");
    return 0;
}

struct WsLayout {
    int64_t eT, eB, eL, eR;            // forward edge buffers (copE channels)
    int64_t dT, dB, dL, dR;            // backward edge buffers (Kin channels)
    int64_t part_main, part_edge, bt_part, comp_part, total;
    int S_main, S_edge, nchunk;
};

WsLayout ws_layout(const Shape& s) {
    WsLayout L;
    int64_t o = 0;
    auto take = [&](int64_t n) {
        const int64_t r = o;
        o += (n + 63) & ~(int64_t)63;
        return r;
    };
    L.eT = take((int64_t)s.B * s.Wo * s.copE);
    L.eB = take((int64_t)s.B * s.Wo * s.copE);
    L.eL = take((int64_t)s.B * s.Ho * s.copE);
    L.eR = take((int64_t)s.B * s.Ho * s.copE);
    L.dT = take((int64_t)s.B * s.Wo * s.Kin);
    L.dB = take((int64_t)s.B * s.Wo * s.Kin);
    L.dL = take((int64_t)s.B * s.Ho * s.Kin);
    L.dR = take((int64_t)s.B * s.Ho * s.Kin);
    const int nmb = s.copC / 64, nkb = s.Kin / 64;
    const int64_t blk = (int64_t)64 * s.ke * 64;
    // main weight gradient: at most one round of workgroups (two per CU: 256 CUs x 2 slots), each with
    // >= 4 pixel blocks.  Rounding the split count up put 532 workgroups on 512 slots for the PackNet01
    // pack layers (grid y = 28): the 20 left over ran as a second round as long as the first
    const int grid_y = s.ke * nmb * nkb;
    const int nblk = s.B * s.Ho * ((s.Wo + 63) / 64);
    L.S_main = std::max(1, std::min(512 / grid_y, std::max(1, nblk / 4)));
    const int nblk_e = s.B * ((std::max(s.Ho, s.Wo) + 63) / 64);
    L.S_edge = std::max(1, std::min(8, nblk_e / 2));
    L.part_main = take((int64_t)L.S_main * s.ke * nmb * nkb * blk);
    L.part_edge = take((int64_t)4 * s.pk * L.S_edge * nmb * nkb * blk);
    L.bt_part = take((int64_t)s.B * s.Ho * (2 * s.pk + 1) * s.C);
    const int64_t nel = (int64_t)s.C * s.k * s.Kin;   // chain-rule W2 rows per Conv3d feature
    L.nchunk = (int)std::max<int64_t>(16, std::min<int64_t>(1024, nel / 1024));
    L.comp_part = take((int64_t)8 * L.nchunk * 28);
    L.total = o;
    return L;
}

struct WbufLayout {
    int64_t wf, wb, ef[4], eb[4], corner, bt, bs, total;   // byte offsets
};

WbufLayout wbuf_layout(const Shape& s) {
    WbufLayout L;
    int64_t o = 0;
    auto take = [&](int64_t n) {
        const int64_t r = o;
        o += (n + 255) & ~(int64_t)255;
        return r;
    };
    L.wf = take((int64_t)s.copC / 64 * (s.Kin / 32) * s.ke * s.ke * 4096);
    L.wb = take((int64_t)s.Kin / 64 * (s.C / 32) * s.ke * s.ke * 4096);
    for (int e = 0; e < 4; ++e) L.ef[e] = take((int64_t)s.copE / 64 * (s.Kin / 32) * s.ke * 4096);
    for (int e = 0; e < 4; ++e) L.eb[e] = take((int64_t)s.Kin / 64 * (s.pk * s.C / 32) * s.ke * 4096);
    L.corner = take((int64_t)4 * s.pk * s.pk * s.C * s.Kin * 4);
    L.bt = take((int64_t)(2 * s.pk + 1) * (2 * s.pk + 1) * s.C * 4);
    L.bs = take((int64_t)s.C * s.k * s.k * 4);
    L.total = o;
    return L;
}

Geo geo_P(const psfm_pc_desc* t, const uint16_t* x) {   // the packed P of the whole batch
    Geo g;
    g.p = x;
    g.s_outer = t->xs[0];
    g.s_row = 2 * t->xs[2];
    g.s_col = 2 * t->xs[3];
    g.sub_off[0] = 0, g.sub_off[1] = t->xs[3], g.sub_off[2] = t->xs[2], g.sub_off[3] = t->xs[2] + t->xs[3];
    g.nsub = 4;
    g.cin = t->C;
    g.rin = t->H / 2;
    g.cols_in = t->W / 2;
    return g;
}

// P's first / last row / column as a [B rows][L columns] image: edge 0 T, 1 B, 2 L, 3 R
Geo geo_P_edge(const psfm_pc_desc* t, const uint16_t* x, int edge) {
    Geo g = geo_P(t, x);
    const int Ho = t->H / 2, Wo = t->W / 2;
    g.s_outer = 0;
    g.s_row = t->xs[0];
    g.rin = t->B;
    if (edge < 2) {
        g.p = x + (edge == 1 ? 2 * (int64_t)(Ho - 1) * t->xs[2] : 0);
        g.s_col = 2 * t->xs[3];
        g.cols_in = Wo;
    } else {
        g.p = x + (edge == 3 ? 2 * (int64_t)(Wo - 1) * t->xs[3] : 0);
        g.s_col = 2 * t->xs[2];
        g.cols_in = Ho;
    }
    return g;
}

// dy's frame lines of edge `edge` as a [B rows][L columns] image with pk "sub-images" (line e)
Geo geo_dy_edge(const psfm_pc_desc* t, const uint16_t* dy, int edge) {
    const Shape s = shape_of(t);
    Geo g;
    g.p = dy;
    g.s_outer = 0;
    g.s_row = t->ys[0];
    g.nsub = s.pk;
    g.cin = s.C;
    g.rin = s.B;
    for (int e = 0; e < 4; ++e) g.sub_off[e] = 0;
    for (int e = 0; e < s.pk; ++e) {
        if (edge == 0) g.sub_off[e] = (int64_t)(s.pk - 1 - e) * t->ys[2];
        if (edge == 1) g.sub_off[e] = (int64_t)(s.Ho - 1 - e) * t->ys[2];
        if (edge == 2) g.sub_off[e] = (int64_t)(s.pk - 1 - e) * t->ys[3];
        if (edge == 3) g.sub_off[e] = (int64_t)(s.Wo - 1 - e) * t->ys[3];
    }
    g.s_col = edge < 2 ? t->ys[3] : t->ys[2];
    g.cols_in = edge < 2 ? s.Wo : s.Ho;
    return g;
}

template <int KH, int KW>
void launch_conv(const ConvArgs& A, int rows_max, int cols_max, int cop_max, hipStream_t st) {
    ConvArgs a = A;
    a.ntc = (cols_max + 63) / 64;
    // every problem's input chunks (nsub x cin / 32) fit the two P buffers: one workgroup runs all the
    // 64-channel output tiles of its pixel tile, staging the input once (the dx backward: 4 tiles)
    bool resident = true;
    for (int i = 0; i < a.nprob; ++i) resident = resident && a.p[i].in.nsub * (a.p[i].in.cin >> 5) <= 2;
    a.nbw = resident ? cop_max / 64 : 1;
    const dim3 grid((unsigned)(((rows_max + 3) / 4) * a.ntc), (unsigned)(cop_max / 64 / a.nbw),
                    (unsigned)(a.nprob * a.outer_max));
    hipLaunchKernelGGL((k_pc_conv<KH, KW>), grid, dim3(256), 0, st, a);
}

void conv_dispatch(const ConvArgs& A, int KH, int KW, int rows_max, int cols_max, int cop_max, hipStream_t st) {
    if (KH == 7) launch_conv<7, 7>(A, rows_max, cols_max, cop_max, st);
    else if (KH == 5) launch_conv<5, 5>(A, rows_max, cols_max, cop_max, st);
    else if (KW == 7) launch_conv<1, 7>(A, rows_max, cols_max, cop_max, st);
    else launch_conv<1, 5>(A, rows_max, cols_max, cop_max, st);
}

CornerArgs corner_args(const psfm_pc_desc* t, const Shape& s, const void* x, const void* dy, const float* w) {
    CornerArgs c;
    c.x = static_cast<const uint16_t*>(x);
    c.xs0 = t->xs[0], c.xs2 = t->xs[2], c.xs3 = t->xs[3];
    c.dy = static_cast<const uint16_t*>(dy);
    c.ys0 = t->ys[0], c.ys2 = t->ys[2], c.ys3 = t->ys[3];
    c.w = w;
    c.eL = c.eR = nullptr;
    c.ecs = 0;
    c.dw = nullptr;
    c.B = s.B, c.C = s.C, c.pk = s.pk, c.Ho = s.Ho, c.Wo = s.Wo;
    return c;
}

}  // namespace

extern "C" {

int64_t psfm_pc_ws_floats(const psfm_pc_desc* t) {
    if (check_desc(t)) return -1;
    return ws_layout(shape_of(t)).total;
}

int64_t psfm_pc_wbuf_bytes(const psfm_pc_desc* t) {
    if (check_desc(t)) return -1;
    return wbuf_layout(shape_of(t)).total;
}

int psfm_pc_weights_of(const psfm_pc_desc* t, const void* wbuf, psfm_pc_weights* out) {
    if (int e = check_desc(t)) return e;
    if (!wbuf || !out) return fail(-1, "null pointer");
    const WbufLayout L = wbuf_layout(shape_of(t));
    const uint8_t* b = static_cast<const uint8_t*>(wbuf);
    out->wf = b + L.wf;
    out->wb = b + L.wb;
    for (int e = 0; e < 4; ++e) {
        out->ef[e] = b + L.ef[e];
        out->eb[e] = b + L.eb[e];
    }
    out->corner = reinterpret_cast<const float*>(b + L.corner);
    out->bt = reinterpret_cast<const float*>(b + L.bt);
    return 0;
}

int psfm_pc_compose(const psfm_pc_desc* t, const float* W2, const float* w3, const float* b3, void* wbuf, void* stream) {
    if (int e = check_desc(t)) return e;
    if (!W2 || !w3 || !wbuf) return fail(-1, "null pointer");
    const Shape s = shape_of(t);
    const WbufLayout L = wbuf_layout(s);
    hipStream_t st = (hipStream_t)stream;
    uint8_t* b = static_cast<uint8_t*>(wbuf);
    CompArgs A{};
    A.W2 = W2, A.w3 = w3, A.b3 = b3;
    A.C = s.C, A.d = t->d, A.k = s.k, A.Kp = s.Kin, A.pk = s.pk, A.ke = s.ke, A.copC = s.copC, A.copE = s.copE;
    A.wf = reinterpret_cast<uint16_t*>(b + L.wf);
    A.wb = reinterpret_cast<uint16_t*>(b + L.wb);
    for (int e = 0; e < 4; ++e) {
        A.ef[e] = reinterpret_cast<uint16_t*>(b + L.ef[e]);
        A.eb[e] = reinterpret_cast<uint16_t*>(b + L.eb[e]);
    }
    A.corner = reinterpret_cast<float*>(b + L.corner);
    A.bt = reinterpret_cast<float*>(b + L.bt);
    A.bs = reinterpret_cast<float*>(b + L.bs);
    const int64_t nm = (int64_t)s.copC * s.ke * s.Kin, ne = (int64_t)4 * s.copE * s.Kin,
                  nc = (int64_t)4 * s.pk * s.pk * s.C * s.Kin;
    if (s.k == 5) {
        hipLaunchKernelGGL(k_pc_comp_main<5>, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, st, A);
        hipLaunchKernelGGL(k_pc_comp_edges<5>, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st, A);
    } else {
        hipLaunchKernelGGL(k_pc_comp_main<3>, dim3((unsigned)((nm + 255) / 256)), dim3(256), 0, st, A);
        hipLaunchKernelGGL(k_pc_comp_edges<3>, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st, A);
    }
    hipLaunchKernelGGL(k_pc_comp_corner, dim3((unsigned)((nc + 255) / 256)), dim3(256), 0, st, A);
    if (b3) hipLaunchKernelGGL(k_pc_comp_bias, dim3((unsigned)(s.C * s.k * s.k)), dim3(256), 0, st, A);
    const int nb = (2 * s.pk + 1) * (2 * s.pk + 1) * s.C;
    hipLaunchKernelGGL(k_pc_comp_bt, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, st, A);
    const hipError_t er = hipGetLastError();
    return er == hipSuccess ? 0 : fail((int)er, std::string("launch: ") + hipGetErrorString(er));
}

int psfm_pc_compose_bwd(const psfm_pc_desc* t, const float* W2, const float* w3, const float* b3, const float* dwmain,
                        const float* dedge, const float* dcorner, const float* dbt, float* dW2, float* dw3, float* db3,
                        float* ws, void* stream) {
    if (int e = check_desc(t)) return e;
    if (!W2 || !w3 || !dwmain || !dedge || !dcorner || !dbt || !dW2 || !dw3 || !ws) return fail(-1, "null pointer");
    const Shape s = shape_of(t);
    const WsLayout L = ws_layout(s);
    hipStream_t st = (hipStream_t)stream;
    CompBwdArgs A{};
    A.W2 = W2, A.w3 = w3, A.b3 = b3, A.dwm = dwmain, A.de = dedge, A.dc = dcorner, A.dbt = dbt;
    A.dW2 = dW2;
    A.part = ws + L.comp_part;
    A.C = s.C, A.d = t->d, A.k = s.k, A.Kp = s.Kin, A.pk = s.pk, A.ke = s.ke, A.nchunk = L.nchunk;
    if (s.k == 5) hipLaunchKernelGGL(k_pc_comp_bwd<5>, dim3((unsigned)L.nchunk, (unsigned)t->d), dim3(256), 0, st, A);
    else hipLaunchKernelGGL(k_pc_comp_bwd<3>, dim3((unsigned)L.nchunk, (unsigned)t->d), dim3(256), 0, st, A);
    hipLaunchKernelGGL(k_pc_comp_bwd_red, dim3((t->d * 28 + 255) / 256), dim3(256), 0, st, (const float*)A.part, t->d,
                       L.nchunk, dw3, db3);
    const hipError_t er = hipGetLastError();
    return er == hipSuccess ? 0 : fail((int)er, std::string("launch: ") + hipGetErrorString(er));
}

int psfm_pc_fwd(const psfm_pc_desc* t, const psfm_pc_weights* w, const void* x, void* y, float* ws, void* stream) {
    if (int e = check_desc(t)) return e;
    if (!w || !x || !y || !ws || !w->wf || !w->corner || !w->bt) return fail(-1, "null pointer");
    for (int e = 0; e < 4; ++e)
        if (!w->ef[e]) return fail(-1, "null edge weights");
    const Shape s = shape_of(t);
    const WsLayout L = ws_layout(s);
    hipStream_t st = (hipStream_t)stream;
    const uint16_t* xb = static_cast<const uint16_t*>(x);
    float* eb[4] = {ws + L.eT, ws + L.eB, ws + L.eL, ws + L.eR};

    // 1. edge convolutions: E[b][pos][e C + m] = sum_s,kin U[e][m][kin][s] P_line[b][pos + s - pe][kin]
    ConvArgs E{};
    E.nprob = 4;
    E.outer_max = 1;
    for (int e = 0; e < 4; ++e) {
        ConvProb& p = E.p[e];
        p.in = geo_P_edge(t, xb, e);
        p.outer = 1;
        p.rows = s.B;
        p.cols = e < 2 ? s.Wo : s.Ho;
        p.ph = 0;
        p.pw = s.pe;
        p.cop = s.copE;
        p.co = s.pk * s.C;
        p.w = static_cast<const uint16_t*>(w->ef[e]);
        p.mode = OUT_F32;
        p.out = eb[e];
        p.o_outer = 0;
        p.o_row = (int64_t)p.cols * s.copE;
        p.o_col = s.copE;
    }
    conv_dispatch(E, 1, s.ke, s.B, std::max(s.Ho, s.Wo), s.copE, st);
    // 2. corner terms into E_L / E_R
    {
        CornerArgs c = corner_args(t, s, x, nullptr, w->corner);
        c.eL = eb[2];
        c.eR = eb[3];
        c.ecs = s.copE;
        const size_t lds = (size_t)s.B * s.Kin * sizeof(float);
        hipLaunchKernelGGL(k_pc_corner_fwd, dim3(4 * s.pk * s.pk * ((s.C + 3) / 4)), dim3(256), lds, st, c);
    }
    // 3. main convolution + epilogue
    ConvArgs M{};
    M.nprob = 1;
    M.outer_max = s.B;
    ConvProb& p = M.p[0];
    p.in = geo_P(t, xb);
    p.outer = s.B;
    p.rows = s.Ho;
    p.cols = s.Wo;
    p.ph = p.pw = s.pe;
    p.cop = s.copC;
    p.co = s.C;
    p.w = static_cast<const uint16_t*>(w->wf);
    p.mode = OUT_Y;
    p.out = y;
    p.o_outer = t->ys[0];
    p.o_row = t->ys[2];
    p.o_col = t->ys[3];
    p.ecs = s.copE;
    for (int e = 0; e < 4; ++e) p.e[e] = eb[e];
    p.bt = w->bt;
    p.C = s.C, p.pk = s.pk, p.Ho = s.Ho, p.Wo = s.Wo;
    conv_dispatch(M, s.ke, s.ke, s.Ho, s.Wo, s.copC, st);
    const hipError_t er = hipGetLastError();
    return er == hipSuccess ? 0 : fail((int)er, std::string("launch: ") + hipGetErrorString(er));
}

int psfm_pc_bwd(const psfm_pc_desc* t, const psfm_pc_weights* w, const void* x, const void* dy, void* dx,
                float* dwmain, float* dedge, float* dcorner, float* dbt, float* ws, void* stream) {
    if (int e = check_desc(t)) return e;
    if (!w || !x || !dy || !ws) return fail(-1, "null pointer");
    const Shape s = shape_of(t);
    const WsLayout L = ws_layout(s);
    hipStream_t st = (hipStream_t)stream;
    const uint16_t* xb = static_cast<const uint16_t*>(x);
    const uint16_t* gb = static_cast<const uint16_t*>(dy);
    if (dx) {
        if (!w->wb || !w->corner) return fail(-1, "null backward weights");
        for (int e = 0; e < 4; ++e)
            if (!w->eb[e]) return fail(-1, "null edge weights");
        float* db[4] = {ws + L.dT, ws + L.dB, ws + L.dL, ws + L.dR};
        // 1. edge transposed convolutions: D[b][pos][kin] = sum U^T dy over the frame lines
        ConvArgs E{};
        E.nprob = 4;
        E.outer_max = 1;
        for (int e = 0; e < 4; ++e) {
            ConvProb& p = E.p[e];
            p.in = geo_dy_edge(t, gb, e);
            p.outer = 1;
            p.rows = s.B;
            p.cols = e < 2 ? s.Wo : s.Ho;
            p.ph = 0;
            p.pw = s.pe;
            p.cop = p.co = s.Kin;
            p.w = static_cast<const uint16_t*>(w->eb[e]);
            p.mode = OUT_F32;
            p.out = db[e];
            p.o_outer = 0;
            p.o_row = (int64_t)p.cols * s.Kin;
            p.o_col = s.Kin;
        }
        conv_dispatch(E, 1, s.ke, s.B, std::max(s.Ho, s.Wo), s.Kin, st);
        // 2. corner adjoints into D_L / D_R
        {
            CornerArgs c = corner_args(t, s, x, dy, w->corner);
            c.eL = db[2];
            c.eR = db[3];
            c.ecs = s.Kin;
            const size_t lds = ((size_t)s.B * s.pk * s.pk * s.C + 4 * s.B * 64) * sizeof(float);
            hipLaunchKernelGGL(k_pc_corner_bwd, dim3(4 * ((s.Kin + 63) / 64)), dim3(256), lds, st, c);
        }
        // 3. main transposed convolution into dx through the packing permutation
        ConvArgs M{};
        M.nprob = 1;
        M.outer_max = s.B;
        ConvProb& p = M.p[0];
        p.in.p = gb;
        p.in.s_outer = t->ys[0];
        p.in.s_row = t->ys[2];
        p.in.s_col = t->ys[3];
        for (int e = 0; e < 4; ++e) p.in.sub_off[e] = 0;
        p.in.nsub = 1;
        p.in.cin = s.C;
        p.in.rin = s.Ho;
        p.in.cols_in = s.Wo;
        p.outer = s.B;
        p.rows = s.Ho;
        p.cols = s.Wo;
        p.ph = p.pw = s.pe;
        p.cop = p.co = s.Kin;
        p.w = static_cast<const uint16_t*>(w->wb);
        p.mode = OUT_DX;
        p.out = dx;
        p.o_outer = t->xs[0];
        p.o_row = t->xs[2];
        p.o_col = t->xs[3];
        p.ecs = s.Kin;
        for (int e = 0; e < 4; ++e) p.e[e] = db[e];
        p.C = s.C, p.pk = s.pk, p.Ho = s.Ho, p.Wo = s.Wo;
        conv_dispatch(M, s.ke, s.ke, s.Ho, s.Wo, s.Kin, st);
    }
    const int nmb = s.copC / 64, nkb = s.Kin / 64;
    auto wgrad = [&](WArgs& A, int KH, int smax, const RArgs& R) {
        A.KH = KH;
        A.nmb = nmb;
        A.nkb = nkb;
        const dim3 grid((unsigned)smax, (unsigned)(KH * nmb * nkb), (unsigned)A.nprob);
        if (s.ke == 7) hipLaunchKernelGGL(k_pc_wgrad<7>, grid, dim3(256), 0, st, A);
        else hipLaunchKernelGGL(k_pc_wgrad<5>, grid, dim3(256), 0, st, A);
        const int64_t n = (int64_t)s.C * KH * s.ke * s.Kin;
        hipLaunchKernelGGL(k_pc_wreduce, dim3((unsigned)((n + 255) / 256), (unsigned)A.nprob), dim3(256), 0, st, R);
    };
    if (dwmain) {
        WArgs A{};
        A.nprob = 1;
        WProb& p = A.p[0];
        p.in = geo_P(t, xb);
        p.g = gb;
        p.g_outer = t->ys[0];
        p.g_row = t->ys[2];
        p.g_col = t->ys[3];
        p.gc = s.C;
        p.outer = s.B;
        p.rows = s.Ho;
        p.cols = s.Wo;
        p.ph = p.pw = s.pe;
        p.nsplit = L.S_main;
        p.part = ws + L.part_main;
        RArgs R{};
        R.p[0] = RProb{p.part, dwmain, L.S_main, 1.0f};
        R.KH = s.ke, R.KW = s.ke, R.nmb = nmb, R.nkb = nkb, R.gc = s.C, R.Kin = s.Kin;
        wgrad(A, s.ke, L.S_main, R);
    }
    if (dedge) {
        WArgs A{};
        RArgs R{};
        A.nprob = 4 * s.pk;
        const int64_t pstride = (int64_t)L.S_edge * nmb * nkb * 64 * s.ke * 64;
        for (int e = 0; e < 4; ++e)
            for (int l = 0; l < s.pk; ++l) {
                WProb& p = A.p[e * s.pk + l];
                p.in = geo_P_edge(t, xb, e);
                const Geo gl = geo_dy_edge(t, gb, e);
                p.g = gb + gl.sub_off[l];
                p.g_outer = 0;
                p.g_row = gl.s_row;
                p.g_col = gl.s_col;
                p.gc = s.C;
                p.outer = 1;
                p.rows = s.B;
                p.cols = gl.cols_in;
                p.ph = 0;
                p.pw = s.pe;
                p.nsplit = L.S_edge;
                p.part = ws + L.part_edge + (e * s.pk + l) * pstride;
                R.p[e * s.pk + l] = RProb{p.part, dedge + (int64_t)(e * s.pk + l) * s.C * s.ke * s.Kin, L.S_edge, -1.0f};
            }
        R.KH = 1, R.KW = s.ke, R.nmb = nmb, R.nkb = nkb, R.gc = s.C, R.Kin = s.Kin;
        wgrad(A, 1, L.S_edge, R);
    }
    if (dcorner) {
        if (!w->corner) return fail(-1, "null corner weights");
        CornerArgs c = corner_args(t, s, x, dy, w->corner);
        c.dw = dcorner;
        const int64_t n = (int64_t)4 * s.pk * s.pk * s.C * s.Kin;
        hipLaunchKernelGGL(k_pc_corner_wgrad, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, c);
    }
    if (dbt) {
        float* part = ws + L.bt_part;
        hipLaunchKernelGGL(k_pc_bt_rows, dim3(s.B * s.Ho), dim3(256), 0, st, gb, t->ys[0], t->ys[2], t->ys[3], s.C,
                           s.Ho, s.Wo, s.pk, part);
        const int n = (2 * s.pk + 1) * (2 * s.pk + 1) * ((s.C + 63) / 64);
        hipLaunchKernelGGL(k_pc_bt_cols, dim3(n), dim3(256), 0, st, (const float*)part, s.B, s.C, s.Ho, s.pk, dbt);
    }
    const hipError_t er = hipGetLastError();
    return er == hipSuccess ? 0 : fail((int)er, std::string("launch: ") + hipGetErrorString(er));
}

const char* psfm_pc_last_error(void) { return g_err.c_str(); }

}  // extern "C"
