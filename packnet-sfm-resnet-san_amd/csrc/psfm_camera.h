// psfm_camera.h — camera models of the sweep kernels (gfx950): pinhole (geometry/camera.py:15-190)
// and the fork's fisheye VADAS model (geometry/camera.py:194-394), as compile-time policies.
//
// A policy holds the wave-uniform parameters of one (scale, image): the target camera and, per
// context j, the context camera and T = [R|t] target -> context, and provides
//   lift(u, v, d)           pixel -> point X = d * ray(u, v) in the target frame (reconstruct)
//   project(j, lift, P&)    X -> c = R X + t -> sampling position (ix, iy) in context j
//   grad(j, P, gix, giy, gc) adjoint: (dL/dix, dL/diy) -> dL/dc (returned in gc, for dL/dT) and
//                            dL/d(depth) (returned)
// Camera records (PSFM_CAMREC floats per (scale, context, image)):
//   pinhole  [0..8] K^-1 of the target | [9..17] K of the context | [18..29] T
//   fisheye  [0..3] target s, div, ux, uy | [4..10] context k0..k6 | [11..14] context s, div,
//            ux, uy | [18..29] T
#pragma once
#include "psfm_common.h"

namespace psfm {

typedef __attribute__((address_space(4))) const float cfloat;  // scalar (s_load) reads

// wave-uniform record pointer -> constant address space (records are read-only in every kernel)
__device__ __forceinline__ cfloat* as_const(const float* p) { return reinterpret_cast<cfloat*>(reinterpret_cast<uint64_t>(p)); }

template <int NC, int MODEL>
struct Cams;

// ---------------------------------------------------------------------------------------------
template <int NC>
struct Cams<NC, PSFM_CAM_PINHOLE> {
    using P = Proj;
    float Ki[9];
    float T[NC][12];
    float Kr[NC][9];
    float wm1, rwm1, hm1, rhm1;

    // rec = record of (s, context 0, b); context j is j*B records further
    __device__ __forceinline__ void load(cfloat* rec, int B, int H, int W) {
#pragma unroll
        for (int i = 0; i < 9; ++i) Ki[i] = rec[i];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
#pragma unroll
            for (int i = 0; i < 9; ++i) Kr[j][i] = rec[(size_t)j * B * PSFM_CAMREC + 9 + i];
#pragma unroll
            for (int i = 0; i < 12; ++i) T[j][i] = rec[(size_t)j * B * PSFM_CAMREC + 18 + i];
        }
        wm1 = (float)(W - 1);
        hm1 = (float)(H - 1);
        rwm1 = rcp_nr(wm1);
        rhm1 = rcp_nr(hm1);
    }
    __device__ __forceinline__ Lift lift(float u, float v, float d) const { return psfm::lift(Ki, u, v, d); }
    __device__ __forceinline__ void project(int j, const Lift& l, Proj& r) const {
        project_lifted(T[j], Kr[j], l, wm1, rwm1, hm1, rhm1, r);
    }
    // same arithmetic as psfm::project_grad (dL/dc -> gc, returns dL/dd)
    __device__ __forceinline__ float grad(int j, const Proj& r, float gix, float giy, float (&gc)[3]) const {
        const float iz = r.iz;
        const float gp0 = gix * iz;
        const float gp1 = giy * iz;
        const float gp2 = (r.p2 >= 1e-5f) ? -(gix * r.p0 + giy * r.p1) * (iz * iz) : 0.0f;
        gc[0] = Kr[j][0] * gp0 + Kr[j][3] * gp1 + Kr[j][6] * gp2;
        gc[1] = Kr[j][1] * gp0 + Kr[j][4] * gp1 + Kr[j][7] * gp2;
        gc[2] = Kr[j][2] * gp0 + Kr[j][5] * gp1 + Kr[j][8] * gp2;
        const float gX0 = T[j][0] * gc[0] + T[j][4] * gc[1] + T[j][8] * gc[2];
        const float gX1 = T[j][1] * gc[0] + T[j][5] * gc[1] + T[j][9] * gc[2];
        const float gX2 = T[j][2] * gc[0] + T[j][6] * gc[1] + T[j][10] * gc[2];
        return gX0 * r.xn0 + gX1 * r.xn1 + gX2 * r.xn2;
    }
};

// ---------------------------------------------------------------------------------------------
// Fisheye VADAS.  reconstruct (camera.py:243-303): (xd, yd) = ((u-ux)/s, (v-uy)/div),
// r_d = |(xd, yd)|, theta = r_d (the reference's approximation), ray = (tan(r_d)/r_d) (xd, yd, 1)
// with r_d clamped below at FLT_EPS.  project (:305-394): (x, y) = c_xy / max(c_z, FLT_EPS),
// r = |(x, y)|, theta = atan r, r_d = k0 + sum_i k_i theta^i, (u, v) = (s, div) (r_d / max(r,
// FLT_EPS)) (x, y) + (ux, uy), then the same [-1, 1] normalise / grid_sample round trip.
constexpr float FLT_EPS_D = 2.220446049250313e-16f;  // sys.float_info.epsilon in fp32

struct FProj {
    float xn0, xn1, xn2;  // ray of the target pixel (dL/dd = dL/dX . ray)
    float X0, X1, X2;     // lifted point
    float c2, iZ;         // c_z and 1 / max(c_z, eps)
    float x, y, r, rs, th, poly;
    float ix, iy;
};

template <int NC>
struct Cams<NC, PSFM_CAM_FISHEYE> {
    using P = FProj;
    float ts, tdiv, tux, tuy;
    float T[NC][12];
    float k[NC][7];
    float s[NC], dv[NC], ux[NC], uy[NC];
    float wm1, rwm1, hm1, rhm1;

    __device__ __forceinline__ void load(cfloat* rec, int B, int H, int W) {
        ts = rec[0];
        tdiv = rec[1];
        tux = rec[2];
        tuy = rec[3];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            cfloat* r = rec + (size_t)j * B * PSFM_CAMREC;
#pragma unroll
            for (int i = 0; i < 7; ++i) k[j][i] = r[4 + i];
            s[j] = r[11];
            dv[j] = r[12];
            ux[j] = r[13];
            uy[j] = r[14];
#pragma unroll
            for (int i = 0; i < 12; ++i) T[j][i] = r[18 + i];
        }
        wm1 = (float)(W - 1);
        hm1 = (float)(H - 1);
        rwm1 = rcp_nr(wm1);
        rhm1 = rcp_nr(hm1);
    }
    __device__ __forceinline__ Lift lift(float u, float v, float d) const {
        const float xd = (u - tux) / ts, yd = (v - tuy) / tdiv;
        const float rd = sqrtf(xd * xd + yd * yd);
        const float r = tanf(rd);
        const float rds = rd < FLT_EPS_D ? FLT_EPS_D : rd;
        Lift l;
        l.xn0 = (r / rds) * xd;
        l.xn1 = (r / rds) * yd;
        l.xn2 = 1.0f;
        l.X0 = l.xn0 * d;
        l.X1 = l.xn1 * d;
        l.X2 = d;
        return l;
    }
    __device__ __forceinline__ void project(int j, const Lift& l, FProj& p) const {
        p.xn0 = l.xn0; p.xn1 = l.xn1; p.xn2 = l.xn2;
        p.X0 = l.X0; p.X1 = l.X1; p.X2 = l.X2;
        const float c0 = T[j][0] * l.X0 + T[j][1] * l.X1 + T[j][2] * l.X2 + T[j][3];
        const float c1 = T[j][4] * l.X0 + T[j][5] * l.X1 + T[j][6] * l.X2 + T[j][7];
        p.c2 = T[j][8] * l.X0 + T[j][9] * l.X1 + T[j][10] * l.X2 + T[j][11];
        const float Z = fmaxf(p.c2, FLT_EPS_D);
        p.iZ = 1.0f / Z;
        p.x = c0 / Z;
        p.y = c1 / Z;
        p.r = sqrtf(p.x * p.x + p.y * p.y);
        p.th = atanf(p.r);
        float poly = k[j][0], tp = 1.0f;
#pragma unroll
        for (int i = 1; i < 7; ++i) {
            tp *= p.th;
            poly += k[j][i] * tp;
        }
        p.poly = poly;
        p.rs = p.r < FLT_EPS_D ? FLT_EPS_D : p.r;
        const float u = s[j] * ((poly / p.rs) * p.x) + ux[j];
        const float v = dv[j] * ((poly / p.rs) * p.y) + uy[j];
        p.ix = norm_roundtrip(u, wm1, rwm1);
        p.iy = norm_roundtrip(v, hm1, rhm1);
    }
    __device__ __forceinline__ float grad(int j, const FProj& p, float gix, float giy, float (&gc)[3]) const {
        // d ix/du = d iy/dv = 1 (normalise round trip); u - ux = s f x, f = P(theta(r)) / rs(r)
        const float gu = gix * s[j], gv = giy * dv[j];
        const float f = p.poly / p.rs;
        float dP = 0.0f, tp = 1.0f;  // P'(theta)
#pragma unroll
        for (int i = 1; i < 7; ++i) {
            dP += (float)i * k[j][i] * tp;
            tp *= p.th;
        }
        const float dth = 1.0f / (1.0f + p.r * p.r);
        const float fr = dP * dth / p.rs - (p.r >= FLT_EPS_D ? p.poly / (p.rs * p.rs) : 0.0f);  // df/dr
        const float w = p.r > 0.0f ? fr / p.r : 0.0f;                                            // df/dr / r
        const float gx = gu * (f + p.x * p.x * w) + gv * (p.y * p.x * w);
        const float gy = gu * (p.x * p.y * w) + gv * (f + p.y * p.y * w);
        gc[0] = gx * p.iZ;
        gc[1] = gy * p.iZ;
        gc[2] = (p.c2 >= FLT_EPS_D) ? -(gx * p.x + gy * p.y) * p.iZ : 0.0f;
        const float gX0 = T[j][0] * gc[0] + T[j][4] * gc[1] + T[j][8] * gc[2];
        const float gX1 = T[j][1] * gc[0] + T[j][5] * gc[1] + T[j][9] * gc[2];
        const float gX2 = T[j][2] * gc[0] + T[j][6] * gc[1] + T[j][10] * gc[2];
        return gX0 * p.xn0 + gX1 * p.xn1 + gX2 * p.xn2;
    }
};

}  // namespace psfm
