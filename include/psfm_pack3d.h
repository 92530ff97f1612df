/*
 * psfm_pack3d.h — C-ABI of the MI355X (gfx950) fused PackNet packing / unpacking 3-D convolution.
 *
 * Replaces, in packnet_sfm/networks/layers/packnet/layers01.py:
 *   PackLayerConv3d.forward   (:217-223)  packing (space-to-depth, :126-146) -> unsqueeze(1) ->
 *                                          Conv3d(1 -> d, 3x3x3, pad 1) -> view(b, d*C, h, w)
 *   UnpackLayerConv3d.forward (:276-282)  unsqueeze(1) -> Conv3d(1 -> d, 3x3x3, pad 1) ->
 *                                          view(b, d*C, h, w) -> PixelShuffle(r)
 * (the Conv2D before / after them stays on MIOpen), and their autograd backward.  ATen runs
 * these as a permute copy + im2col + GEMM + col2im + a second permute copy with a d-times
 * larger intermediate; here one kernel reads the (virtually packed) volume once from its own
 * layout and writes the folded / pixel-shuffled result straight into the caller's layout.
 *
 * The 3-D convolution runs over the virtual volume V[b][k][y][x] (K = C*r^2 channels for pack,
 * K = C for unpack; Hv x Wv pixels) with zero padding, 8 (d) output features per voxel at
 * channel o*K + k of the folded map.  Tensors are described by element strides (any memory
 * format); `dtype` selects fp32 or bf16 storage (fp32 accumulation either way).
 *   mode PSFM_P3D_PACK:   x [B, C, Hv*r, Wv*r] -> y [B, d*C*r^2, Hv, Wv]
 *   mode PSFM_P3D_UNPACK: x [B, C, Hv, Wv]     -> y [B, d*C/r^2, Hv*r, Wv*r]
 * Weights w [d, 1, 3, 3, 3] and bias [d] are fp32 (the caller casts).  Deterministic: the
 * weight gradient is reduced from per-workgroup partials in a fixed order (fp64).
 */
#ifndef PSFM_PACK3D_H
#define PSFM_PACK3D_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum psfm_p3d_mode { PSFM_P3D_PACK = 0, PSFM_P3D_UNPACK = 1 };
enum psfm_p3d_dtype { PSFM_P3D_F32 = 0, PSFM_P3D_BF16 = 1 };

typedef struct psfm_p3d_desc {
    int mode, dtype;
    int B, C, Hv, Wv, r, d;          /* C: channels of x; Hv x Wv: the volume's pixels; d = 8 */
    int64_t xs[4];                   /* element strides of x  (b, c, h, w) */
    int64_t ys[4];                   /* element strides of y  (b, c, h, w) */
} psfm_p3d_desc;

/* y = fold(conv3d(pack(x))) / shuffle(fold(conv3d(x))) */
int psfm_p3d_fwd(const psfm_p3d_desc* t, const void* x, const float* w, const float* bias, void* y,
                 void* stream);

/* floats of the weight-gradient workspace (per-workgroup partials) */
int64_t psfm_p3d_ws_floats(const psfm_p3d_desc* t);

/* backward: dx (strides t->xs, written) from dy (strides t->ys); dw [d*27] and dbias [d] fp32
 * (written) through the workspace; dx / dw may be NULL to skip that gradient. */
int psfm_p3d_bwd(const psfm_p3d_desc* t, const void* x, const float* w, const void* dy, void* dx,
                 float* dw, float* dbias, float* ws, void* stream);

const char* psfm_p3d_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_PACK3D_H */
