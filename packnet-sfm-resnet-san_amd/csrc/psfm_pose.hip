// psfm_pose.hip — pose algebra and pinhole camera records for the photometric loss
// (include/psfm_pose.h).  A few hundred floats per step: one thread per pose / record, one
// launch each.  The point is the launch count on the step's critical path (the ATen chain is
// ~100 dependent kernels of a few floats each), not bandwidth.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "../../include/psfm.h"
#include "../../include/psfm_pose.h"

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int launch_status() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail((int)e, std::string("launch: ") + hipGetErrorString(e));
}

struct MatPtrs {
    float* m[PSFM_POSE_MAX_CTX];
};
struct ConstMatPtrs {
    const float* m[PSFM_POSE_MAX_CTX];
};

// A = Rx(x) Ry(y), R = A Rz(z) (euler2mat, pose_utils.py:8-37: xmat.bmm(ymat).bmm(zmat)).  The
// products with the zero / one entries of the elementary matrices are exact, so each entry of
// A is one rounded product and each entry of R one two-term sum, as in the reference's bmm.
struct Euler {
    float cx, sx, cy, sy, cz, sz;
    float a[3][3];
    __device__ explicit Euler(const float* v) {
#pragma clang fp contract(off)
        cx = cosf(v[3]); sx = sinf(v[3]);
        cy = cosf(v[4]); sy = sinf(v[4]);
        cz = cosf(v[5]); sz = sinf(v[5]);
        a[0][0] = cy;       a[0][1] = 0.0f; a[0][2] = sy;
        a[1][0] = sx * sy;  a[1][1] = cx;   a[1][2] = -(sx * cy);
        a[2][0] = -(cx * sy); a[2][1] = sx; a[2][2] = cx * cy;
    }
};

__global__ __launch_bounds__(64) void k_pose_fwd(const float* __restrict__ vec, int B, int N, MatPtrs out) {
#pragma clang fp contract(off)
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * N) return;
    const int b = t / N, j = t - b * N;
    const float* v = vec + (size_t)t * 6;
    const Euler e(v);
    float* m = out.m[j] + (size_t)b * 16;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        m[4 * i + 0] = e.a[i][0] * e.cz + e.a[i][1] * e.sz;
        m[4 * i + 1] = e.a[i][0] * -e.sz + e.a[i][1] * e.cz;
        m[4 * i + 2] = e.a[i][2];
        m[4 * i + 3] = v[i];
    }
    m[12] = 0.0f; m[13] = 0.0f; m[14] = 0.0f; m[15] = 1.0f;
}

// dL/dvec from dL/dR, dL/dt (the chain rule through R = A Rz, A = Rx Ry and the sin / cos of
// each angle); the reference's autograd graph of the same expressions (bmm, stack, sin, cos)
__global__ __launch_bounds__(64) void k_pose_bwd(const float* __restrict__ vec, int B, int N, ConstMatPtrs gm,
                                                 float* __restrict__ gvec) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * N) return;
    const int b = t / N, j = t - b * N;
    float* o = gvec + (size_t)t * 6;
    const float* g = gm.m[j];
    if (!g) {
#pragma unroll
        for (int k = 0; k < 6; ++k) o[k] = 0.0f;
        return;
    }
    g += (size_t)b * 16;
    const Euler e(vec + (size_t)t * 6);
    float ga[3][3];
    float gcz = 0.0f, gsz = 0.0f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float g0 = g[4 * i], g1 = g[4 * i + 1];
        ga[i][0] = g0 * e.cz - g1 * e.sz;
        ga[i][1] = g0 * e.sz + g1 * e.cz;
        ga[i][2] = g[4 * i + 2];
        gcz += g0 * e.a[i][0] + g1 * e.a[i][1];
        gsz += g0 * e.a[i][1] - g1 * e.a[i][0];
        o[i] = g[4 * i + 3];
    }
    const float gcy = ga[0][0] - ga[1][2] * e.sx + ga[2][2] * e.cx;
    const float gsy = ga[0][2] + ga[1][0] * e.sx - ga[2][0] * e.cx;
    const float gcx = ga[1][1] - ga[2][0] * e.sy + ga[2][2] * e.cy;
    const float gsx = ga[1][0] * e.sy - ga[1][2] * e.cy + ga[2][1];
    o[3] = gsx * e.cx - gcx * e.sx;
    o[4] = gsy * e.cy - gcy * e.sy;
    o[5] = gsz * e.cz - gcz * e.sz;
}

// Camera.scaled -> scale_intrinsics (camera_utils.py:16-22, in place on a clone, fp32 ops one by
// one) and Kinv (camera.py:72-81: the clone of K with 1/fx, 1/fy, -cx/fx, -cy/fy; `1.0 / t` is
// reciprocal, IEEE in both)
__device__ __forceinline__ void scaled_k(const float* k, float s, bool scale, float* o) {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < 9; ++i) o[i] = k[i];
    if (scale) {
        o[0] = o[0] * s;
        o[4] = o[4] * s;
        o[2] = (o[2] + 0.5f) * s - 0.5f;
        o[5] = (o[5] + 0.5f) * s - 0.5f;
    }
}

__global__ __launch_bounds__(64) void k_cam_records(const float* __restrict__ K, const float* __restrict__ refK,
                                                    const float* __restrict__ T, int t_stride, int B, int N, int S,
                                                    float s, int scale, float* __restrict__ cam) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= S * N * B) return;
    const int b = t % B, j = (t / B) % N;
    float k[9], r[9];
    scaled_k(K + (size_t)b * 9, s, scale != 0, k);
    scaled_k(refK + (size_t)b * 9, s, scale != 0, r);
    float* o = cam + (size_t)t * PSFM_CAMREC;
#pragma unroll
    for (int i = 0; i < 9; ++i) o[i] = k[i];
    o[0] = 1.0f / k[0];
    o[4] = 1.0f / k[4];
    o[2] = -k[2] / k[0];
    o[5] = -k[5] / k[4];
#pragma unroll
    for (int i = 0; i < 9; ++i) o[9 + i] = r[i];
    const float* tt = T + ((size_t)j * B + b) * t_stride;
#pragma unroll
    for (int i = 0; i < 12; ++i) o[18 + i] = tt[i];
#pragma unroll
    for (int i = 30; i < PSFM_CAMREC; ++i) o[i] = 0.0f;
}

}  // namespace

extern "C" {

int psfm_pose_from_vec_fwd(const float* vec, int B, int N, float* const* mats, void* stream) {
    if (!vec || !mats || B < 1 || N < 1 || N > PSFM_POSE_MAX_CTX) return fail(-1, "bad pose_from_vec args");
    MatPtrs p{};
    for (int j = 0; j < N; ++j) {
        if (!mats[j]) return fail(-1, "null pose matrix output");
        p.m[j] = mats[j];
    }
    hipLaunchKernelGGL(k_pose_fwd, dim3((B * N + 63) / 64), dim3(64), 0, (hipStream_t)stream, vec, B, N, p);
    return launch_status();
}

int psfm_pose_from_vec_bwd(const float* vec, int B, int N, const float* const* grad_mats, float* grad_vec,
                           void* stream) {
    if (!vec || !grad_mats || !grad_vec || B < 1 || N < 1 || N > PSFM_POSE_MAX_CTX)
        return fail(-1, "bad pose_from_vec_bwd args");
    ConstMatPtrs p{};
    for (int j = 0; j < N; ++j) p.m[j] = grad_mats[j];
    hipLaunchKernelGGL(k_pose_bwd, dim3((B * N + 63) / 64), dim3(64), 0, (hipStream_t)stream, vec, B, N, p,
                       grad_vec);
    return launch_status();
}

int psfm_pinhole_cam_records(const float* K, const float* ref_K, const float* T, int t_stride, int B, int N, int S,
                             float scale, float* cam, void* stream) {
    if (!K || !ref_K || !T || !cam || B < 1 || N < 1 || S < 1) return fail(-1, "bad cam_records args");
    if (t_stride != 12 && t_stride != 16) return fail(-2, "t_stride must be 12 ([3][4]) or 16 ([4][4])");
    const int n = S * N * B;
    hipLaunchKernelGGL(k_cam_records, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, K, ref_K, T, t_stride,
                       B, N, S, scale, scale != 1.0f ? 1 : 0, cam);
    return launch_status();
}

const char* psfm_pose_last_error(void) { return g_err.c_str(); }

}  // extern "C"
