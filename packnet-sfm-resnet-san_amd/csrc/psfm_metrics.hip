// psfm_metrics.hip — depth evaluation metrics (the Abs Rel gate) for MI355X (gfx950), behind the
// C-ABI of include/psfm_metrics.h.
//
// Reference: packnet_sfm/utils/depth.py:258-447 compute_depth_metrics.  One 1024-thread
// workgroup per image: valid mask (depth bounds on gt + Garg crop) -> exact lower medians of the
// valid gt and pred values by a 4-pass 8-bit radix select (integer LDS histograms of order-
// preserving float keys: exact and order independent) -> median scaling -> the seven metrics
// with fp64 fixed-order block sums.  A one-wave kernel then averages over the batch.  The image
// reads are L2-resident after the first pass (gt + pred = 1 MB per 192x640 image).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/psfm_metrics.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

constexpr int MT = 1024;
constexpr int MW = MT / 64;

struct MArgs {
    psfm_metrics_params p;
    const float* gt;
    const float* pred;
    float* per;  // [B][8]
    int y1, y2, x1, x2;
};

// order-preserving map of IEEE fp32 onto uint32 (negative values reversed), and back
__device__ __forceinline__ uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float funkey(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__device__ __forceinline__ bool is_valid(const MArgs& a, float g, int i) {
    bool v = g > a.p.min_depth && g < a.p.max_depth;  // :328-329 (fp32 compares)
    if (a.p.crop_garg) {
        const int y = i / a.p.W, x = i - y * a.p.W;
        v = v && y >= a.y1 && y < a.y2 && x >= a.x1 && x < a.x2;  // :330-334
    }
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(MT) void k_metrics(MArgs a) {
    __shared__ uint32_t hist[2][256];
    __shared__ uint32_t s_prefix[2], s_k[2], s_count;
    __shared__ double red[MW][7];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int plane = a.p.H * a.p.W;
    const float* g = a.gt + (size_t)b * plane;
    const float* pr = a.pred + (size_t)b * plane;

    // valid-pixel count
    if (tid == 0) s_count = 0;
    __syncthreads();
    uint32_t n = 0;
    for (int i = tid; i < plane; i += MT) n += is_valid(a, g[i], i) ? 1u : 0u;
    atomicAdd(&s_count, n);
    __syncthreads();
    const uint32_t N = s_count;
    float* out = a.per + (size_t)b * 8;
    if (N == 0) {  // no valid pixel: skipped by the batch average (:362-365)
        if (tid < 8) out[tid] = 0.0f;
        return;
    }

    float scale = 1.0f;
    if (a.p.use_gt_scale) {
        // lower median (torch.median) of the valid gt and pred values: rank (N-1)/2
        if (tid < 2) {
            s_prefix[tid] = 0u;
            s_k[tid] = (N - 1u) / 2u;
        }
        uint32_t hmask = 0u;
        for (int shift = 24; shift >= 0; shift -= 8) {
            for (int t = tid; t < 512; t += MT) hist[t >> 8][t & 255] = 0u;
            __syncthreads();
            const uint32_t pg = s_prefix[0], pp = s_prefix[1];
            for (int i = tid; i < plane; i += MT) {
                const float gv = g[i];
                if (!is_valid(a, gv, i)) continue;
                const uint32_t kg = fkey(gv), kp = fkey(pr[i]);
                if ((kg & hmask) == pg) atomicAdd(&hist[0][(kg >> shift) & 255u], 1u);
                if ((kp & hmask) == pp) atomicAdd(&hist[1][(kp >> shift) & 255u], 1u);
            }
            __syncthreads();
            if (tid < 2) {  // find the digit holding rank k
                uint32_t k = s_k[tid], cum = 0u;
                int d = 0;
                for (; d < 255; ++d) {
                    const uint32_t h = hist[tid][d];
                    if (cum + h > k) break;
                    cum += h;
                }
                s_k[tid] = k - cum;
                s_prefix[tid] |= (uint32_t)d << shift;
            }
            hmask |= 255u << shift;
            __syncthreads();
        }
        const float gmed = funkey(s_prefix[0]), pmed = funkey(s_prefix[1]);
        scale = gmed / pmed;  // :382 (fp32)
    }

    double acc[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int i = tid; i < plane; i += MT) {
        const float gv = g[i];
        if (!is_valid(a, gv, i)) continue;
        const float p = a.p.use_gt_scale ? pr[i] * scale : pr[i];
        const float th = fmaxf(gv / p, p / gv);  // :414
        const float d = gv - p;                   // :419
        const float lg = logf(gv) - logf(p);
        acc[0] += (double)(fabsf(d) / gv);
        acc[1] += (double)(d * d / gv);
        acc[2] += (double)(d * d);
        acc[3] += (double)(lg * lg);
        acc[4] += th < 1.25f ? 1.0 : 0.0;
        acc[5] += th < 1.5625f ? 1.0 : 0.0;    // 1.25 ** 2 (exact in fp32)
        acc[6] += th < 1.953125f ? 1.0 : 0.0;  // 1.25 ** 3
    }
#pragma unroll
    for (int m = 0; m < 7; ++m) {
        const double v = wave_sum_d(acc[m]);
        if (lane == 0) red[wave][m] = v;
    }
    __syncthreads();
    if (tid < 7) {
        double s = 0.0;
        for (int w = 0; w < MW; ++w) s += red[w][tid];
        const double mean = s / (double)N;
        out[tid] = (float)((tid == 2 || tid == 3) ? sqrt(mean) : mean);  // rmse, rmse_log (:422-424)
    }
    if (tid == 7) out[7] = (float)N;
}

// batch average: sum over images in order, / B (skipped images add 0, :446-447)
__global__ __launch_bounds__(64) void k_metrics_final(const float* per, int B, float* out) {
    const int m = threadIdx.x;
    if (m >= 7) return;
    double s = 0.0;
    for (int b = 0; b < B; ++b)
        if (per[b * 8 + 7] > 0.0f) s += (double)per[b * 8 + m];
    out[m] = (float)(s / (double)B);
}

}  // namespace

extern "C" {

int psfm_depth_metrics(const psfm_metrics_params* p, const float* gt, const float* pred, float* per_image,
                       float* out, void* stream) {
    if (!p || !gt || !pred || !per_image || !out) return fail(-1, "null metrics argument");
    if (p->B < 1 || p->H < 1 || p->W < 1) return fail(-2, "bad B/H/W");
    if ((long long)p->H * p->W > (1LL << 30)) return fail(-2, "image too large");
    MArgs a{};
    a.p = *p;
    a.gt = gt;
    a.pred = pred;
    a.per = per_image;
    // crop bounds as the reference computes them: int(fraction * size) in double precision
    a.y1 = (int)(0.40810811 * p->H);
    a.y2 = (int)(0.99189189 * p->H);
    a.x1 = (int)(0.03594771 * p->W);
    a.x2 = (int)(0.96405229 * p->W);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_metrics, dim3(p->B), dim3(MT), 0, st, a);
    hipLaunchKernelGGL(k_metrics_final, dim3(1), dim3(64), 0, st, (const float*)per_image, p->B, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail((int)e, std::string("launch: ") + hipGetErrorString(e));
    return 0;
}

const char* psfm_metrics_last_error(void) { return g_err.c_str(); }

}  // extern "C"
