/*
 * psfm_packconv.h — C-ABI of the MI355X (gfx950) composed PackNet packing layer.
 *
 * Replaces, in packnet_sfm/networks/layers/packnet/layers01.py:
 *   PackLayerConv3d.forward (:239-246)   packing (:126-146) -> unsqueeze -> Conv3d(1 -> d, 3x3x3,
 *                                         pad 1) -> view(b, d*4C, H/2, W/2) -> self.conv, whose
 *                                         Conv2D (:10-37) is ConstantPad2d(k//2) -> Conv2d(d*4C -> C, k)
 * up to the Conv2d (its bias, GroupNorm and ELU stay in psfm_gn_act), and its autograd backward.
 *
 * The packed volume never exists.  Conv3d (3x3x3, 1 -> d) followed by the k x k Conv2d is ONE
 * linear (k+2) x (k+2) convolution over the 4C packed channels P (= a 2(k+2) x 2(k+2), stride-2
 * convolution over x itself), with 4x fewer MACs than the reference chain for k = 5, d = 8
 * (4C (k+2)^2 vs d 4C k^2 per output), EXCEPT that the reference zero-pads the Conv3d output V
 * (ConstantPad2d) where the composed form would extend V = conv3d(P) + bias3 past the image.
 * The exact output is
 *     y = conv(P, Weff) + BT[row class][col class] - E_T - E_B - E_L - E_R (+ corner terms)
 * where Weff = conv3d^T-composition of (W2, w3), BT the bias3 table, and E_* are 1-D (k+2)-tap
 * convolutions of P's first / last row / column (the only P values that reach the V ring just
 * outside the image) on the frame pixels within k//2 of the border.  psfm_pc_compose builds these
 * small tensors in kernel layouts from the module's parameters (and psfm_pc_compose_bwd carries
 * their gradients back); the other kernels do the data-sized work:
 *   forward : edge convolutions (4 lines) -> corner terms -> main convolution + epilogue (bias
 *             table, edge terms) -> y (bf16, channels_last)
 *   backward: edge transposed convolutions -> corner terms -> main transposed convolution written
 *             straight into dx's packing permutation (+ edge terms) ; main and edge weight
 *             gradients (per-split partials, fixed-order reduce: deterministic) ; corner and
 *             bias-table gradients
 * Main / edge convolutions and weight gradients run on v_mfma_f32_16x16x32_bf16 (fp32 accumulate);
 * edge / corner / bias terms are fp32.
 *
 * Constraints (else the caller keeps the reference op chain): x bf16 channels_last, H and W even,
 * C % 32 == 0, k odd in {3, 5}, d in {4, 8}, H/2 >= 2 (k//2) + 1, W/2 >= 2 (k//2) + 1.
 */
#ifndef PSFM_PACKCONV_H
#define PSFM_PACKCONV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct psfm_pc_desc {
    int B, C, H, W;     /* x [B, C, H, W] bf16 channels_last; y [B, C, H/2, W/2] */
    int k;              /* the Conv2D kernel size (pad k/2); ke = k + 2, pk = k / 2 */
    int d;              /* Conv3d output features (8 PackNet01, 4 PackNetSAN01) */
    int64_t xs[4];      /* element strides of x (b, c, h, w); xs[1] == 1 */
    int64_t ys[4];      /* element strides of y and dy (b, c, h, w); ys[1] == 1 */
} psfm_pc_desc;

/* Weights in kernel layouts (bf16 unless noted).  cop(n) = n rounded up to a multiple of 64;
 * kin = s C + c is the packed channel of sub-pixel s = 2 i + j (the reference's packed channel is
 * 4 c + s); "[..][4][64][8]" is the 32-channel chunk as 4 groups of 8 per 64-column block. */
typedef struct psfm_pc_weights {
    const void* wf;      /* main forward  [cop(C)/64][4C/32][ke][ke][4][64][8]: Weff[m][kin][a][b]    */
    const void* wb;      /* main backward [4C/64][C/32][ke][ke][4][64][8]: Weff[m][kin][ke-1-a][ke-1-b] */
    const void* ef[4];   /* edge forward  (T, B, L, R) [cop(pk C)/64][4C/32][1][ke][4][64][8], column e C + m */
    const void* eb[4];   /* edge backward (T, B, L, R) [4C/64][pk C/32][1][ke][4][64][8], flipped taps */
    const float* corner; /* fp32 [4 (TL, BL, TR, BR)][pk][pk][C][4C] */
    const float* bt;     /* fp32 [2pk+1][2pk+1][C]: bias3 table by (row class, column class) */
} psfm_pc_weights;

/* floats of the workspace either direction needs */
int64_t psfm_pc_ws_floats(const psfm_pc_desc* t);

/* The composed weights, from the module's fp32 parameters W2 [C][d 4C][k][k] (Conv2D.conv_base,
 * reference layout), w3 [d][1][3][3][3] and b3 [d] (Conv3d; NULL = no bias).  Every operand is
 * rounded to bf16 first, as autocast's Conv3d / Conv2d does; the sums run in fp32.  All layouts go
 * into one caller buffer of psfm_pc_wbuf_bytes() bytes; psfm_pc_weights_of() returns the pointers
 * into it.  psfm_pc_compose_bwd() is the chain rule back to W2, w3, b3 from the composed weights'
 * gradients (those psfm_pc_bwd writes; the bf16 rounding passes gradients straight through), fp32,
 * deterministic (fixed-order reductions). */
int64_t psfm_pc_wbuf_bytes(const psfm_pc_desc* t);
int psfm_pc_weights_of(const psfm_pc_desc* t, const void* wbuf, psfm_pc_weights* out);
int psfm_pc_compose(const psfm_pc_desc* t, const float* W2, const float* w3, const float* b3, void* wbuf,
                    void* stream);
int psfm_pc_compose_bwd(const psfm_pc_desc* t, const float* W2, const float* w3, const float* b3,
                        const float* dwmain, const float* dedge, const float* dcorner, const float* dbt,
                        float* dW2, float* dw3, float* db3, float* ws, void* stream);

/* y = the Conv2d output (no Conv2d bias) of PackLayerConv3d on x */
int psfm_pc_fwd(const psfm_pc_desc* t, const psfm_pc_weights* w, const void* x, void* y, float* ws,
                void* stream);

/* backward from dy (strides t->ys): dx (bf16, strides t->xs) and the gradients of the composed
 * weights, fp32, any of them NULL to skip:
 *   dwmain  [C][ke][ke][4C]       (m, a, b, kin)
 *   dedge   [4][pk][C][ke][4C]    (edge, e, m, s, kin)
 *   dcorner [4][pk][pk][C][4C]
 *   dbt     [2pk+1][2pk+1][C] */
int psfm_pc_bwd(const psfm_pc_desc* t, const psfm_pc_weights* w, const void* x, const void* dy, void* dx,
                float* dwmain, float* dedge, float* dcorner, float* dbt, float* ws, void* stream);

const char* psfm_pc_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_PACKCONV_H */
