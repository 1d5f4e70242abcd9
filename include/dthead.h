/* dthead.h — C-ABI of the DDPG update's small fully connected tails
 * (BASELINE configs[4]): config.json's critic output branch
 * concat(obs branch 256, action 2) -> linear 128 -> leaky_relu -> linear 1
 * and the actor output branch linear 2 -> tanh (models/ddpg/modules.py
 * Net.forward's torch.cat + the output MetaNet), run in train mode by
 * training/trainers.py:156-229 on batches of 64.  Each is a handful of
 * 64-row GEMMs far too small for a library GEMM's tiles (one 128x64 tile a
 * launch, ~15 us); here one launch runs the whole tail forward, one its
 * whole backward.
 *
 * The tail: x = [x0 | x1] (x1 optional: the concatenation is read in place),
 *   h = act1(x w1^T + b1)                         [m, n1]
 *   y = act2(h w2^T + b2)  (two layers)           [m, n2]   or y = h (one layer)
 * act: 0 none, 1 leaky_relu(slope), 2 tanh, 3 sigmoid.  Row-major float32,
 * w1 [n1, k0 + k1], w2 [n2, n1]; b1 / b2 may be NULL.  Forward dot products:
 * 16 strided f32 fma chains over k, then a butterfly; backward: one f32 fma
 * chain per element over the rows (dw) or the outputs (dx).  Deterministic;
 * the order differs from a library GEMM's.
 * Limits: m <= 256, k0 + k1 <= 1024, n1 <= 1024 (<= 512 with a second layer),
 * n2 <= 64, m * n1 <= 8192, m * n2 <= 2048, n2 * n1 <= 4096; DT_E_ARG otherwise.
 * leaky_relu with slope >= 0 only (its derivative is read from the sign of
 * the saved output).
 * Conventions as dtsim.h: 0 or a negative DT_E_* code; device pointers; work
 * goes on `stream`. */
#ifndef AIDO1_AMD_DTHEAD_H
#define AIDO1_AMD_DTHEAD_H

#include <stdint.h>

#include "dtsim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct DtMlp {
  int32_t m, k0, k1, n1, n2;   /* n2 = 0: one layer */
  int32_t act1, act2;
  float slope;
  const float* w1;
  const float* b1;
  const float* w2;
  const float* b2;
} DtMlp;

/* h [m, n1] (kept for the backward), y [m, n2] (two layers; NULL for one). */
int dt_mlp_fwd(const DtMlp* p, const float* x0, const float* x1, float* h, float* y, void* stream);

/* dt_mlp_fwd plus the TD target of the DDPG critic loss (training/trainers.py:
 * 166-170) in the same launch: target[r][j] = rew[r] + (notdone[r] * gamma) *
 * y[r][j] (y = h for one layer), rew / notdone [m] device f32, target [m, n_out]. */
int dt_mlp_fwd_td(const DtMlp* p, const float* x0, const float* x1, float* h, float* y,
                  const float* rew, const float* notdone, float gamma, float* target,
                  void* stream);

/* The DDPG losses in one launch each (training/trainers.py:174-177, 193-196),
 * one workgroup, a float64 sum in a fixed order:
 *   kind 0: loss = mean((a - b)^2)  (F.mse_loss, mean reduction)
 *   kind 1: loss = -mean(a)         (the actor loss, b unused)
 * dt_loss_bwd: da = (2 / m) (a - b) g (kind 0), -(g / m) (kind 1), g the
 * scalar upstream gradient (device).  m >= 1. */
int dt_loss(int32_t kind, int32_t m, const float* a, const float* b, float* loss, void* stream);
int dt_loss_bwd(int32_t kind, int32_t m, const float* a, const float* b, const float* g,
                float* da, void* stream);

/* The tail's backward from dy (= dL/dy [m, n2], or dL/dh [m, n1] for one
 * layer) and the forward's h and y: any output may be NULL (not wanted).
 *   dx0 [m, k0], dx1 [m, k1], dw1 [n1, k0 + k1], db1 [n1], dw2 [n2, n1], db2 [n2] */
int dt_mlp_bwd(const DtMlp* p, const float* x0, const float* x1, const float* h, const float* y,
               const float* dy, float* dx0, float* dx1, float* dw1, float* db1, float* dw2,
               float* db2, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AIDO1_AMD_DTHEAD_H */
