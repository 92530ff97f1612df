/*
 * psfm_optim.h — C-ABI of the fused mixed-precision Adam step of the training hot path.
 *
 * Replaces, per training step (reference: packnet_sfm/models/model_wrapper.py:172-216 builds
 * torch.optim.Adam with 'Depth'/'Pose' param groups; packnet_sfm/trainers/horovod_trainer.py:
 * 222-284 runs zero_grad -> backward -> (Horovod allreduce) -> optimizer.step()):
 *   - the gradient gather into one flat buffer for the RCCL all-reduce (psfm_grad_pack),
 *   - torch.optim.Adam.step (L2 weight decay, bias-corrected moments, eps outside the sqrt) on
 *     fp32 master weights, fused with the bf16 -> fp32 widening of the gradients and the
 *     fp32 -> bf16 rounding of the model weights (psfm_adam_step).
 * One launch covers every parameter tensor: the tensors are described by a device table, the
 * work by a device chunk list (psfm_optim_plan_chunks), so the whole update is graph-capturable
 * and its argument list never changes between replays (the kernel reads the tables at run time).
 *
 * Conventions as include/psfm.h: device pointers, caller-owned buffers, stream-ordered, return
 * 0 / <0 bad argument / >0 hipError_t, message from psfm_optim_last_error().
 */
#ifndef PSFM_OPTIM_H
#define PSFM_OPTIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSFM_OPT_GRAD_BF16 1   /* grad storage is bfloat16 (else float32)             */
#define PSFM_OPT_PARAM_BF16 2  /* model parameter storage is bfloat16 (else float32)  */
#define PSFM_OPT_CHUNK 1024    /* elements per workgroup                              */

/* One parameter tensor.  Elements are addressed in STORAGE order (dense tensors; grad and
 * parameter share strides, e.g. both channels_last), element i of the tensor is element
 * offset + i of the flat fp32 master / exp_avg / exp_avg_sq / flat-gradient buffers. */
typedef struct psfm_optim_tensor {
    const void* grad;   /* autograd's gradient of the model parameter                   */
    void* param;        /* the model parameter, rewritten as round(master) every step    */
    int64_t numel;
    int64_t offset;     /* multiple of 4                                                 */
    int32_t group;      /* index into the hyper-parameter array (param_groups order)     */
    int32_t flags;      /* PSFM_OPT_*                                                    */
} psfm_optim_tensor;

/* torch.optim.Adam param_group hyper-parameters (amsgrad=False, maximize=False). */
typedef struct psfm_adam_hparams {
    float lr, beta1, beta2, eps, weight_decay;
    float pad[3];
} psfm_adam_hparams;

/* Host: split n tensors into PSFM_OPT_CHUNK-element work items.  chunks[2*k] = tensor index,
 * chunks[2*k+1] = first element.  Returns the number of chunks (chunks may be NULL to count),
 * or <0 when `cap` is too small. */
int psfm_optim_plan_chunks(int n, const int64_t* numel, int32_t* chunks, int cap);

/* flat_grad[offset + i] = float(grad[i]) for every tensor (the all-reduce buffer). */
int psfm_grad_pack(const psfm_optim_tensor* tensors, const int32_t* chunks, int nchunks,
                   float* flat_grad, void* stream);

/* One Adam step on every tensor: step[0] += 1, then with t = step[0]
 *   g = (flat_grad ? flat_grad[offset+i] * grad_scale : float(grad[i])) + wd * master
 *   m = b1*m + (1-b1)*g ;  v = b2*v + (1-b2)*g*g
 *   master -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps) ;  param[i] = round(master)
 * (ATen's fused Adam formula, in fp32).  hparams: device array indexed by tensor.group. */
int psfm_adam_step(const psfm_optim_tensor* tensors, const int32_t* chunks, int nchunks,
                   const psfm_adam_hparams* hparams, int32_t* step, const float* flat_grad,
                   float grad_scale, float* master, float* exp_avg, float* exp_avg_sq, void* stream);

const char* psfm_optim_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PSFM_OPTIM_H */
