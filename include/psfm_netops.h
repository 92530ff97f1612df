/*
 * psfm_netops.h — C-ABI of the fused normalisation / activation kernels of the depth and pose
 * networks (gfx950).
 *
 * The reference runs these layers as separate ATen/MIOpen ops under autocast:
 *   - ResNet encoder  conv -> BatchNorm2d -> ReLU (-> + identity -> ReLU)
 *       packnet_sfm/networks/layers/resnet/resnet_encoder.py:16-98 (torchvision BasicBlock)
 *   - DepthDecoder    Conv3x3(bias) -> ReLU / Sigmoid
 *       packnet_sfm/networks/layers/resnet/depth_decoder.py:16-64, layers.py:12-72
 *   - PoseNet         Conv2d(bias) -> GroupNorm(16) -> ReLU
 *       packnet_sfm/networks/pose/PoseNet.py:15-84
 * i.e. 3 MIOpen BN kernels + ReLU + add forward and 3 + 2 backward per BN layer, bias add +
 * ReLU + a bias-gradient reduction per decoder conv.  Each entry point below fuses one such
 * chain into one or two passes over the activation.
 *
 * Layout: an activation is a bf16 matrix [M, C] row-major — the storage order of an NHWC
 * (torch.channels_last) tensor with M = N*H*W (GroupNorm: [N, HW, C]).  Statistics and
 * parameters are fp32.  Reductions are deterministic (no float atomics) and use no counters:
 * each pass writes one partial row per workgroup into `ws`, and the next launch sums what it
 * needs in a fixed order (fp64) — the GroupNorm apply pass its sample's group rows in its
 * prologue, a small column-total kernel the parameter gradients.  The kernel boundary orders
 * the partial rows before their readers, so no device-scope arrival rounds are needed.
 *
 * Conventions as include/psfm.h: device pointers, caller-owned buffers, stream-ordered,
 * graph-capturable; return 0 / <0 bad argument / >0 hipError_t, message from
 * psfm_netops_last_error().
 */
#ifndef PSFM_NETOPS_H
#define PSFM_NETOPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSFM_ACT_NONE 0
#define PSFM_ACT_RELU 1
#define PSFM_ACT_SIGMOID 2
#define PSFM_ACT_ELU 3     /* ELU(alpha = 1): GroupNorm only (PackNet Conv2D / ResidualConv) */

/* fp32 workspace floats needed by a reduction over an [M, C] activation (bias_act_bwd,
 * bn_act_fwd / bn_act_bwd), and for groupnorm over [N, HW, C] with G groups. */
size_t psfm_netops_ws_floats(int M, int C);
size_t psfm_gn_ws_floats(int N, int HW, int C, int G);

/* y = act(x + bias)   (Conv2d bias add + ReLU / Sigmoid, layers.py:44-51, depth_decoder.py:60).
 * x bf16 [M,C]; bias bf16 (bias_bf16=1) or fp32 [C]; y bf16 for NONE/RELU, fp32 for SIGMOID
 * (the sigmoid maps feed the fp32 photometric loss). */
int psfm_bias_act_fwd(const void* x, const void* bias, int bias_bf16, int M, int C, int act, void* y,
                      void* stream);

/* dx = dy * act'(y) (bf16), dbias = sum_rows dx (written in the bias dtype).  dy has y's dtype.
 * Two launches: dx + per-workgroup partial rows, then the column totals. */
int psfm_bias_act_bwd(const void* dy, const void* y, int M, int C, int act, void* dx, void* dbias,
                      int bias_bf16, float* ws, void* stream);
/* The same with dy := bf16(dy + dy1): the two gradients of an output that has two consumers (the
 * DepthDecoder's up-stage output feeds the next stage and a disparity head), summed in the load as
 * autograd's accumulation would (one bf16 rounding) — no separate add kernel.  ReLU / NONE only. */
int psfm_bias_act_bwd_sum(const void* dy, const void* dy1, const void* y, int M, int C, int act, void* dx,
                          void* dbias, int bias_bf16, float* ws, void* stream);

/* Training-mode BatchNorm2d (+ residual) (+ ReLU):  y = act(gamma (x-mu)/sqrt(var+eps) + beta [+ res]),
 * ONE launch each way where psfm_bn_act_resident(M, C) (ws may be NULL there); other shapes return
 * -3 — the two-launch "ticket" kernels (a statistics pass whose last workgroup finishes the batch
 * statistics) and the round-2 three-pass kernels both lost to MIOpen's BatchNorm and were removed
 * from the library in round 6 (git 61b4f88 holds them);
 * batch statistics over the M rows, running stats updated as torch does (momentum, unbiased
 * var), save_mean / save_invstd [C] for the backward.  res may be NULL. */
int psfm_bn_act_fwd(const void* x, const void* res, const float* gamma, const float* beta, float* run_mean,
                    float* run_var, float momentum, float eps, int M, int C, int relu, void* y, float* save_mean,
                    float* save_invstd, float* ws, void* stream);

/* 1 when an [M, C] BatchNorm runs the resident one-launch kernels (a workgroup owns 8 channels and
 * all M rows: C % 8 == 0 and M <= the BN_RES_MAXM knob, 2048 by default = the ResNet encoder's
 * layer3-4 at B = 4, 192x640; at most 8192), else 0.  Callers keep MIOpen's BatchNorm for the other
 * shapes (the three-pass kernels lose to it, and so does the resident form at larger M: DESIGN.md). */
int psfm_bn_act_resident(int M, int C);
/* 1 when psfm_bn_act_fwd / _bwd(_sum) take an [M, C] BatchNorm at all (the product: the resident
 * shapes; A/B builds: also the two-launch ticket form), else 0. */
int psfm_bn_act_fused(int M, int C);

/* Backward of psfm_bn_act_fwd: dx (bf16), dres (bf16, = ReLU-masked dy; may be NULL),
 * dgamma / dbeta (fp32 [C], written). */
int psfm_bn_act_bwd(const void* dy, const void* y, const void* x, const float* gamma, const float* save_mean,
                    const float* save_invstd, int M, int C, int relu, void* dx, void* dres, float* dgamma,
                    float* dbeta, float* ws, void* stream);
/* The same with dy := bf16(bf16(dy + dy1) + dy2) (dy1 / dy2 may be NULL): the gradients of a block
 * output with several consumers (next block's conv1 and identity / downsample, the decoder skip),
 * summed inside the kernel instead of by autograd's add kernels. */
int psfm_bn_act_bwd_sum(const void* dy, const void* dy1, const void* dy2, const void* y, const void* x,
                        const float* gamma, const float* save_mean, const float* save_invstd, int M, int C, int relu,
                        void* dx, void* dres, float* dgamma, float* dbeta, float* ws, void* stream);

/* y = act(GroupNorm(G)(x [+ res] + bias)) per sample: x / res bf16 [N, HW, C], conv bias bf16/fp32 [C]
 * or NULL, gamma/beta fp32 [C], act PSFM_ACT_NONE / RELU / ELU.  PoseNet conv_gn (conv + GN + ReLU,
 * PoseNet.py:15-19); PackNet Conv2D (conv + GN(16) + ELU, layers01.py:10-37) and ResidualConv's
 * GN(conv2 + shortcut) + ELU (res = the conv2 branch, layers01.py:40-61).  save_mean / save_invstd
 * [N*G].  Layers whose (sample, channel block) fits one 256-thread workgroup's registers run ONE launch
 * (statistics and apply in the workgroup): the block is CB = max(8, C/G) channels with C/G in
 * {1, 2, 4, 8, 16, 32} (CV = CB/8 row vectors of 8 channels per pixel), each thread holds RPT <= 4
 * pixels' row vectors, so HW <= 256 RPT / CV = 1024 / CV pixels (PackNet's 24x80 and smaller layers
 * at C/G <= 8).  Larger layers take two launches (statistics rows, then apply with the per-sample
 * reduction in its prologue). */
int psfm_gn_act_fwd(const void* x, const void* res, const void* bias, int bias_bf16, const float* gamma,
                    const float* beta, float eps, int N, int HW, int C, int G, int act, void* y, float* save_mean,
                    float* save_invstd, float* ws, void* stream);

/* Backward of psfm_gn_act_fwd: dx (bf16) and, with res, dres (a second copy: both inputs are summed),
 * dgamma / dbeta (fp32 [C]) and dbias (bias dtype, NULL with bias NULL).  dbias is the conv-bias
 * gradient sum_{n,hw} dx in CLOSED FORM, per sample k1*S1 - HW*k2 - k3*X (S1 = sum dyr, X = sum xhat
 * per channel, k1 = gamma*invstd, k2 / k3 the group terms of dx), summed over samples in fp64 from
 * fp32 partial sums before any bf16 rounding — not the column sum of the stored bf16 dx that autograd
 * would form; the two differ by the bf16 rounding noise of the N*HW summands (with one or two channels
 * per group the exact sum is ~0 and both are noise; tests/test_netops.py pins it for cpg 1 / 2 / 4 / 8+).
 * The activation's derivative is taken at its input, recomputed from x (+ res + bias), save_mean /
 * save_invstd and gamma / beta — the forward output is not read back.  Resident layers (as the
 * forward, HW <= 1024 / CV pixels, 512 / CV with res): one data launch (dy, x read once)
 * + a parameter finish over per-sample rows; others: statistics rows, then apply + parameter
 * gradients (two launches). */
int psfm_gn_act_bwd(const void* dy, const void* x, const void* res, const void* bias, int bias_bf16,
                    const float* gamma, const float* beta, const float* save_mean, const float* save_invstd,
                    int N, int HW, int C, int G, int act, void* dx, void* dres, void* dbias, float* dgamma,
                    float* dbeta, float* ws, void* stream);

/* BasicBlock tail after the BatchNorm (torchvision BasicBlock via resnet_encoder.py:61-98:
 * out = relu(bn2(conv2(.)) + identity)): y = relu(bf16(a + b)) over n bf16 elements (n % 8 == 0,
 * 16-byte aligned; any layout, a / b / y alike) — the add and the ReLU of autocast's op chain in one
 * pass; and its backward dz = (y <= 0) ? 0 : dy, ATen's threshold_backward (both inputs get dz). */
int psfm_add_relu_fwd(const void* a, const void* b, long long n, void* y, void* stream);
int psfm_relu_mask_bwd(const void* dy, const void* y, long long n, void* dz, void* stream);
/* b may be NULL in psfm_add_relu_fwd (y = relu(a): the stem's BatchNorm + ReLU, whose output has two
 * consumers); psfm_relu_mask_bwd_sum masks bf16(bf16(dy + dy1) + dy2) (dy1 / dy2 may be NULL): the
 * gradients of an output with several consumers, summed in the mask pass. */
int psfm_relu_mask_bwd_sum(const void* dy, const void* dy1, const void* dy2, const void* y, long long n, void* dz,
                           void* stream);

/* The nets' fp32 input images as the bf16 first-convolution inputs, one pass each (ATen: sub, div,
 * autocast cast / cat, cast).  psfm_normalize_bf16: y[i] = bf16((x[i] - sub) * mul) over n elements
 * of any dense layout (y keeps x's), x 16-byte and y 8-byte aligned — the depth encoder's
 * (x - 0.45) / 0.225 (resnet_encoder.py:89) with mul = 1.0f / 0.225f, which is how ATen divides by a
 * scalar.  psfm_cat_channels_bf16: NHWC concatenation along channels of k <= 4 fp32 NHWC images of
 * `pixels` pixels each (channels[q] per pixel, <= 32 in all) into bf16 y [pixels, sum channels] — PoseNet's
 * torch.cat([image, *context], 1) (PoseNet.py) + its cast. */
int psfm_normalize_bf16(const float* x, long long n, float sub, float mul, void* y, void* stream);
int psfm_cat_channels_bf16(int k, const float* const* xs, const int* channels, long long pixels, void* y,
                           void* stream);

/* The ResNet stem's ReLU + MaxPool2d(kernel 3, stride 2, padding 1) (torchvision ResNet through
 * resnet_encoder.py: relu(bn1(conv1(x))) feeds the max-pool and the decoder's first skip) in ONE pass:
 * x = the BatchNorm output, bf16 NHWC [N, H, W, C] (H, W even, C % 8 == 0); writes relu_out (same
 * shape: the skip), pool_out [N, H/2, W/2, C] and argmax (uint8 per output element: the window
 * position kh * 3 + kw of the maximum, ATen's first-maximum / NaN-propagating choice). */
int psfm_relu_maxpool_fwd(const void* x, int N, int H, int W, int C, void* relu_out, void* pool_out, void* argmax,
                          void* stream);
/* Its backward in one pass: dx = relu'(relu_out) * bf16(bf16(max-pool backward of bf16(dpool + dpool1))
 * + dskip) — ATen's max_pool2d backward (windows in (oh, ow) order, fp32, one rounding), autograd's adds
 * of the pooled output's second consumer (dpool1, may be NULL) and of the skip (dskip, may be NULL). */
int psfm_relu_maxpool_bwd(const void* dpool, const void* dpool1, const void* dskip, const void* relu_out,
                          const void* argmax, int N, int H, int W, int C, void* dx, void* stream);

const char* psfm_netops_last_error(void);

/* Decoder up-stage input: out = cat([nearest_up2(x), skip], channels)  (the reference's
 * upsample(convs[("upconv", i, 0)](x)) then torch.cat with the encoder skip,
 * packnet_sfm/networks/layers/resnet/depth_decoder.py:48-57, layers.py:60-64).
 * x bf16 NHWC [N, h, w, C1]; skip bf16 NHWC [N, 2h, 2w, C2] or NULL with C2 = 0; out bf16 NHWC
 * [N, 2h, 2w, C1 + C2].  C1 >= 8, C1 and C2 multiples of 8 (16-byte vectors). */
int psfm_upcat_fwd(const void* x, const void* skip, int N, int h, int w, int C1, int C2, void* out, void* stream);

/* Its backward: dx[n, y, x, c] = the sum of dout[n, 2y + i, 2x + j, c] over the 2x2 block (fp32,
 * fixed order, one bf16 rounding: deterministic, unlike ATen's atomic upsample backward),
 * dskip = dout[..., C1:] (NULL when C2 = 0). */
int psfm_upcat_bwd(const void* dout, int N, int h, int w, int C1, int C2, void* dx, void* dskip, void* stream);

/* The up-stage input with the stage's first ConvBlock folded in (layers.py:25-41 Conv3x3 + ReLU,
 * depth_decoder.py:48-57): out = cat([nearest_up2(relu(x + bias)), skip], channels), x = that
 * block's convolution WITHOUT its bias (bf16 NHWC [N, h, w, C1]), bias bf16 (bias_bf16 = 1) or fp32
 * [C1].  The block's output is never materialised on its own.  C1 / 8 must divide 256. */
int psfm_upcat_bias_relu_fwd(const void* x, const void* bias, int bias_bf16, const void* skip, int N, int h, int w,
                             int C1, int C2, void* out, void* stream);

/* Its backward: dx = (relu'(.) read from `out`, the forward output) * the 2x2 block sums of
 * dout[..., :C1] (fp32, one bf16 rounding), dskip = dout[..., C1:], dbias = the column sums of the
 * stored dx (bias dtype) — two launches (dx + partial rows, column totals); ws floats:
 * psfm_upcat_ws_floats(N, h, w, C1). */
int psfm_upcat_bias_relu_bwd(const void* dout, const void* out, int N, int h, int w, int C1, int C2, void* dx,
                             void* dskip, void* dbias, int bias_bf16, float* ws, void* stream);
size_t psfm_upcat_ws_floats(int N, int h, int w, int C1);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_NETOPS_H */
