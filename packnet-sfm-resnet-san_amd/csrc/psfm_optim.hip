// psfm_optim.hip — fused mixed-precision Adam step and gradient pack (include/psfm_optim.h).
//
// Replaces torch.optim.Adam.step over the 'Depth'/'Pose' param groups
// (reference: packnet_sfm/models/model_wrapper.py:172-216) plus the per-tensor dtype casts of a
// bf16-weight / fp32-master training step: ONE launch reads each gradient in its own dtype,
// updates the fp32 master weight and both moments (flat, contiguous buffers) and writes the
// rounded model weight back.  HBM-bound: 2 (bf16 grad) + 3x4 read + 3x4 write + 2 (bf16 weight)
// = 28 B per parameter.
//
// Work decomposition: one 256-thread workgroup per PSFM_OPT_CHUNK (=1024) elements of ONE
// tensor, 4 consecutive elements per lane (16-B master/moment accesses; tensor offsets are
// multiples of 4 and chunk starts multiples of 1024, so vector accesses are aligned), scalar
// tail at the end of a tensor.  The step counter lives on the device (graph replays advance it).
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "psfm_optim.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

constexpr int kThreads = 256;
static_assert(PSFM_OPT_CHUNK == 4 * kThreads, "one 4-element group per lane");

__device__ __forceinline__ float bf16_to_f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// round-to-nearest-even, NaN kept quiet (c10::BFloat16 semantics)
__device__ __forceinline__ uint16_t f_to_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

__device__ __forceinline__ void load_grad(const psfm_optim_tensor& t, int64_t i, int n, float g[4]) {
    if (t.flags & PSFM_OPT_GRAD_BF16) {
        const uint16_t* gp = static_cast<const uint16_t*>(t.grad) + i;
        if (n == 4) {
            const uint2 v = *reinterpret_cast<const uint2*>(gp);
            g[0] = bf16_to_f(v.x & 0xffff), g[1] = bf16_to_f(v.x >> 16);
            g[2] = bf16_to_f(v.y & 0xffff), g[3] = bf16_to_f(v.y >> 16);
        } else {
            for (int k = 0; k < n; ++k) g[k] = bf16_to_f(gp[k]);
        }
    } else {
        const float* gp = static_cast<const float*>(t.grad) + i;
        if (n == 4) {
            const float4 v = *reinterpret_cast<const float4*>(gp);
            g[0] = v.x, g[1] = v.y, g[2] = v.z, g[3] = v.w;
        } else {
            for (int k = 0; k < n; ++k) g[k] = gp[k];
        }
    }
}

__device__ __forceinline__ void load4(const float* p, int n, float v[4]) {
    if (n == 4) {
        const float4 q = *reinterpret_cast<const float4*>(p);
        v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
    } else {
        for (int k = 0; k < n; ++k) v[k] = p[k];
    }
}

__device__ __forceinline__ void store4(float* p, int n, const float v[4]) {
    if (n == 4) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
        for (int k = 0; k < n; ++k) p[k] = v[k];
    }
}

__global__ __launch_bounds__(kThreads) void k_grad_pack(const psfm_optim_tensor* __restrict__ tensors,
                                                        const int32_t* __restrict__ chunks, float* flat_grad) {
    const int ti = chunks[2 * blockIdx.x];
    const psfm_optim_tensor t = tensors[ti];
    const int64_t i = (int64_t)chunks[2 * blockIdx.x + 1] + 4 * threadIdx.x;
    if (i >= t.numel) return;
    const int n = (int)min<int64_t>(4, t.numel - i);
    float g[4];
    load_grad(t, i, n, g);
    store4(flat_grad + t.offset + i, n, g);
}

__global__ void k_step_inc(int32_t* step) { *step += 1; }

__global__ __launch_bounds__(kThreads) void k_adam(const psfm_optim_tensor* __restrict__ tensors,
                                                   const int32_t* __restrict__ chunks,
                                                   const psfm_adam_hparams* __restrict__ hparams,
                                                   const int32_t* __restrict__ step,
                                                   const float* __restrict__ flat_grad, float grad_scale,
                                                   float* __restrict__ master, float* __restrict__ exp_avg,
                                                   float* __restrict__ exp_avg_sq) {
    const int ti = chunks[2 * blockIdx.x];
    const psfm_optim_tensor t = tensors[ti];
    const int64_t i = (int64_t)chunks[2 * blockIdx.x + 1] + 4 * threadIdx.x;
    if (i >= t.numel) return;
    const int n = (int)min<int64_t>(4, t.numel - i);
    const psfm_adam_hparams h = hparams[t.group];
    // bias corrections as ATen's fused Adam: in the op math type from the float step count
    const float st = (float)*step;
    const float bc1 = 1.0f - powf(h.beta1, st);
    const float bc2 = 1.0f - powf(h.beta2, st);
    const float step_size = h.lr / bc1;
    const float bc2_sqrt = sqrtf(bc2);
    const int64_t f = t.offset + i;
    float g[4], p[4], m[4], v[4];
    if (flat_grad) {
        load4(flat_grad + f, n, g);
        for (int k = 0; k < 4; ++k) g[k] *= grad_scale;
    } else {
        load_grad(t, i, n, g);
    }
    load4(master + f, n, p);
    load4(exp_avg + f, n, m);
    load4(exp_avg_sq + f, n, v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float gk = g[k];
        if (h.weight_decay != 0.0f) gk += p[k] * h.weight_decay;
        m[k] = h.beta1 * m[k] + (1.0f - h.beta1) * gk;
        v[k] = h.beta2 * v[k] + (1.0f - h.beta2) * gk * gk;
        const float denom = (sqrtf(v[k]) / bc2_sqrt) + h.eps;
        p[k] -= step_size * m[k] / denom;
    }
    store4(master + f, n, p);
    store4(exp_avg + f, n, m);
    store4(exp_avg_sq + f, n, v);
    if (t.flags & PSFM_OPT_PARAM_BF16) {
        uint16_t* pp = static_cast<uint16_t*>(t.param) + i;
        if (n == 4) {
            *reinterpret_cast<uint2*>(pp) = make_uint2((uint32_t)f_to_bf16(p[0]) | ((uint32_t)f_to_bf16(p[1]) << 16),
                                                       (uint32_t)f_to_bf16(p[2]) | ((uint32_t)f_to_bf16(p[3]) << 16));
        } else {
            for (int k = 0; k < n; ++k) pp[k] = f_to_bf16(p[k]);
        }
    } else {
        store4(static_cast<float*>(t.param) + i, n, p);
    }
}

}  // namespace

extern "C" {

int psfm_optim_plan_chunks(int n, const int64_t* numel, int32_t* chunks, int cap) {
    if (n < 0 || (n > 0 && !numel)) return fail(-1, "psfm_optim_plan_chunks: bad tensor list");
    int64_t k = 0;
    for (int t = 0; t < n; ++t) {
        if (numel[t] < 0 || numel[t] > (int64_t)INT32_MAX) return fail(-2, "psfm_optim_plan_chunks: bad numel");
        for (int64_t s = 0; s < numel[t]; s += PSFM_OPT_CHUNK, ++k) {
            if (chunks) {
                if (k >= cap) return fail(-3, "psfm_optim_plan_chunks: chunk buffer too small");
                chunks[2 * k] = t;
                chunks[2 * k + 1] = (int32_t)s;
            }
        }
    }
    if (k > INT32_MAX) return fail(-4, "psfm_optim_plan_chunks: too many chunks");
    return (int)k;
}

int psfm_grad_pack(const psfm_optim_tensor* tensors, const int32_t* chunks, int nchunks, float* flat_grad,
                   void* stream) {
    if (!tensors || !chunks || !flat_grad || nchunks < 0) return fail(-1, "psfm_grad_pack: null argument");
    if (nchunks == 0) return 0;
    hipLaunchKernelGGL(k_grad_pack, dim3(nchunks), dim3(kThreads), 0, (hipStream_t)stream, tensors, chunks,
                       flat_grad);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail((int)e, std::string("psfm_grad_pack: ") + hipGetErrorString(e));
}

int psfm_adam_step(const psfm_optim_tensor* tensors, const int32_t* chunks, int nchunks,
                   const psfm_adam_hparams* hparams, int32_t* step, const float* flat_grad, float grad_scale,
                   float* master, float* exp_avg, float* exp_avg_sq, void* stream) {
    if (!tensors || !chunks || !hparams || !step || !master || !exp_avg || !exp_avg_sq || nchunks < 0)
        return fail(-1, "psfm_adam_step: null argument");
    const hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_step_inc, dim3(1), dim3(1), 0, st, step);
    if (nchunks > 0)
        hipLaunchKernelGGL(k_adam, dim3(nchunks), dim3(kThreads), 0, st, tensors, chunks, hparams, step,
                           flat_grad, grad_scale, master, exp_avg, exp_avg_sq);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail((int)e, std::string("psfm_adam_step: ") + hipGetErrorString(e));
}

const char* psfm_optim_last_error(void) { return g_err.c_str(); }

}  // extern "C"
