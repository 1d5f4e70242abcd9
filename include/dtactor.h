/* dtactor.h — C-ABI of the actor-side kernels of the batched rollout
 * (SURVEY.md §8a A19-A20).
 *
 * dt_sample_norm: LeakyReLU followed by BatchNorm2d in TRAIN mode applied to
 * a batch of ONE sample, for n samples at once.  This is what every acting
 * call of the reference computes: its explorers' models are in train mode
 * (training/managers.py:264-268, training/explorers.py:46) and act on a single
 * observation (models/ddpg/model.py:74-88), so each conv layer's
 * `leaky_relu -> batch_norm_2d` (config.json actor list; ddpg.py:56) uses
 * that sample's own per-channel mean and biased variance over H x W:
 *   y = (lrelu(x) - mean_c) / sqrt(var_c + eps) * gamma_c + beta_c.
 * x, y: [n, hw, c] channels-last (NHWC) tensors, bf16 (dtype 0), f32
 * (dtype 1) or fp16 (dtype 2); c a multiple of 8, <= 64; gamma, beta: f32[c].  Statistics are
 * accumulated in f32, two-pass (mean, then squared deviations).  y may alias x.
 * Returns 0 or DT_E_ARG / DT_E_HIP; work is enqueued on `stream`.
 */
#ifndef AIDO1_AMD_DTACTOR_H
#define AIDO1_AMD_DTACTOR_H

#include <stdint.h>

#include "dtsim.h"

#ifdef __cplusplus
extern "C" {
#endif

int dt_sample_norm(const void* x, void* y, int32_t n, int32_t hw, int32_t c, const float* gamma,
                   const float* beta, float eps, float slope, int32_t dtype, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AIDO1_AMD_DTACTOR_H */
