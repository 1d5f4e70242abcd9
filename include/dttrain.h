/* dttrain.h — C-ABI of the fused training-mode layer tail of the DDPG update
 * (BASELINE configs[4]).
 *
 * Every conv block of the reference's actor and critic is conv_2d ->
 * leaky_relu -> batch_norm_2d (config.json:19-170, models/ddpg/modules.py
 * MetaNet), and every network is in train mode during the update
 * (training/trainers.py:143-237, managers.py:264-268): BatchNorm normalises
 * with the batch statistics and updates its running statistics.  These two
 * calls replace, per block, torch's bias add, LeakyReLU, BatchNorm (MIOpen's
 * three kernels) and num_batches_tracked increment in the forward, and
 * BatchNorm's backward, LeakyReLU's backward and the bias-gradient reduction
 * in the backward: two kernels each way (aido1_amd/csrc/dttrain.hip).  The
 * convolution itself stays MIOpen's (called without bias).
 *
 * Layout: NHWC float32 (torch channels_last), m = N*H*W pixels of exactly 32
 * channels.  Per-channel reductions run per workgroup (Welford for the
 * statistics, plain f32 sums in the backward) and the last workgroup to
 * finish merges the partials (Chan's formula) and writes the per-channel
 * results, so one launch does the whole reduction.
 *
 *   work   device scratch, dt_train_work_floats(m) floats, zeroed ONCE before
 *          its first use (the kernels leave their counters and the partials'
 *          counts at zero again); one buffer per call site in flight (a forward
 *          and a backward of the same layer may not share one).
 *   guard  a non-finite guard block (below) or NULL.
 *
 * The hand-off: every workgroup writes its partials through to memory (`sc1`
 * stores), waits for them, and adds to a counter; the workgroup whose add
 * returns grid - 1 runs an agent-scope acquire before it reads the partials
 * (MI355X_MICROARCH.md, inter-workgroup visibility: valid at any placement
 * of the workgroups), then zeroes the partials' counts, so a partial that
 * was never written or is read stale shows up as a missing count:
 * dt_bn_leaky_fwd's last workgroup checks that the merged count is m
 * (DT_GUARD_BN_COUNT) and that mean / invstd are finite (DT_GUARD_BN_FWD);
 * dt_bn_leaky_bwd's that dgamma / dbeta / dbias are finite (DT_GUARD_BN_BWD).
 *
 * Conventions as dtsim.h: 0 or a negative DT_E_* code; device pointers; work
 * goes on `stream` (a hipStream_t).
 */
#ifndef AIDO1_AMD_DTTRAIN_H
#define AIDO1_AMD_DTTRAIN_H

#include <stdint.h>

#include "dtsim.h"

#ifdef __cplusplus
extern "C" {
#endif

int64_t dt_train_work_floats(int64_t m);

/* Forward: a = leaky_relu(z + bias, slope); y = (a - mean) * invstd * gamma +
 * beta with the batch mean and biased variance of a over the m pixels
 * (invstd = 1 / sqrt(var + eps)); running_mean / running_var move by
 * `momentum` towards mean and the unbiased variance, num_batches_tracked += 1
 * (torch.nn.BatchNorm2d.forward in train mode); `updates` >= 1 times, as
 * that many train-mode forwards over the same batch would (the trainer's
 * shared critic trunk: the actor-loss and TD-error forwards of
 * training/trainers.py:190-192,223-226 see the same weights and batch).
 *   z, y               device f32 [m, 32]
 *   a                  device f32 [m, 32] out, or NULL: the activation is not
 *                      stored (the normalisation and dt_bn_leaky_bwd recompute
 *                      it from z and bias, bit for bit)
 *   bias, gamma, beta  device f32 [32]
 *   running_mean, running_var  device f32 [32], updated in place
 *   num_batches_tracked        device int64 [1] or NULL
 *   mean_invstd        device f32 [64] out: mean[32] then invstd[32] (saved
 *                      for the backward) */
int dt_bn_leaky_fwd(int64_t m, const float* z, const float* bias, float slope, const float* gamma,
                    const float* beta, float eps, float momentum, float* running_mean,
                    float* running_var, int64_t* num_batches_tracked, int32_t updates, float* a,
                    float* y, float* mean_invstd, float* work, int32_t* guard, void* stream);

/* The normalisation half of dt_bn_leaky_fwd alone, from statistics already
 * in mean_invstd (dt_upd_conv_fwd_bn, include/dtupd.h):
 * y = (leaky_relu(z + bias) - mean) * invstd * gamma + beta. */
int dt_bn_leaky_apply(int64_t m, const float* z, const float* bias, float slope,
                      const float* mean_invstd, const float* gamma, const float* beta, float* y,
                      void* stream);

/* Backward of dt_bn_leaky_fwd given dy (device f32 [m, 32]) and the forward's
 * z and bias (a = leaky_relu(z + bias, slope) recomputed):
 *   dgamma = sum(dy * xhat), dbeta = sum(dy), xhat = (a - mean) * invstd;
 *   da = gamma * invstd * (dy - dbeta / m - xhat * dgamma / m);
 *   dz = a > 0 ? da : slope * da  (LeakyReLU's backward: a > 0 iff z + bias > 0);
 *   dbias = sum(dz).
 *   dz            device f32 [m, 32] out
 *   dbias, dgamma, dbeta  device f32 [32] out (overwritten) */
int dt_bn_leaky_bwd(int64_t m, const float* dy, const float* z, const float* bias,
                    const float* mean_invstd, const float* gamma, float slope, float* dz,
                    float* dbias, float* dgamma, float* dbeta, float* work, int32_t* guard,
                    void* stream);

/* Multi-tensor steps over a network's parameters in one launch.  `tensors`
 * is a device table, one entry per parameter (the roles of a, b, c, d per
 * call below, n elements each, float32); `chunks` a device table of
 * (tensor index, chunk index) int32 pairs, one workgroup per chunk of
 * DT_MT_CHUNK elements. */
#define DT_MT_CHUNK 4096
typedef struct dt_mt_tensor {
  float* a;
  float* b;
  float* c;
  float* d;
  int64_t n;
} dt_mt_tensor;

/* torch.optim.Adam's step (no weight decay, amsgrad or maximize;
 * trainers.py:258-268 "adam"), a = param, b = grad, c = exp_avg, d = exp_avg_sq:
 *   t = *step + 1 (*step is written back by the last workgroup);
 *   c = lerp(c, b, 1 - beta1); d = d * beta2 + (1 - beta2) * b * b;
 *   a = a - lr / (1 - beta1^t) * c / (sqrt(d) / sqrt(1 - beta2^t) + eps)
 * with the bias corrections in float64 from *step and *lr (device float64),
 * each element op rounded to float32 in torch's order.
 *   counter  device uint32, zero before the first call (left at zero)
 *   guard    a guard block or NULL: grad_bit is set if a gradient is not
 *            finite, param_bit if an updated parameter is not (-1: no bit) */
int dt_adam(int32_t n_chunks, const dt_mt_tensor* tensors, const int32_t* chunks, double* step,
            const double* lr, double beta1, double beta2, double eps, uint32_t* counter,
            int32_t* guard, int32_t grad_bit, int32_t param_bit, void* stream);

/* Soft target update (models/torch_utils.py:5-9), a = target, b = source:
 * a = a * (1 - tau) + b * tau, the two products rounded separately. */
int dt_soft_update(int32_t n_chunks, const dt_mt_tensor* tensors, const int32_t* chunks,
                   double tau, void* stream);


/* ---- Non-finite guards (SURVEY.md §5 failure detection) ----------------------------------
 * A guard block is DT_GUARD_WORDS device int32, zeroed by the caller except
 * first[] (DT_GUARD_NONE each):
 *   word 0           OR of the stage bits (1 << bit) found non-finite
 *   word 1           number of detections (one per wave that saw one)
 *   word 2           the tick: the caller's sequence number (the trainer
 *                    adds 1 per update, on the device, so captured graphs
 *                    advance it too)
 *   word 3 + bit     the smallest tick at which `bit` was set (DT_GUARD_NONE
 *                    until then)
 * The stages of the training loop (aido1_amd/guard.py names them): */
#define DT_GUARD_WORDS 36
#define DT_GUARD_NONE 0x7fffffff
enum {
  DT_GUARD_ACTOR_OUT = 0,    /* rollout actor outputs (before DDPG.act's clip) */
  DT_GUARD_ENV = 1,          /* rollout rewards */
  DT_GUARD_BATCH = 2,        /* the sampled batch: obs, action, reward, next_obs */
  DT_GUARD_TARGET = 3,       /* y = r + notdone * gamma * Q'(s', pi'(s')) */
  DT_GUARD_BN_FWD = 4,       /* a train-mode BatchNorm's batch mean / invstd */
  DT_GUARD_BN_COUNT = 5,     /* a BatchNorm's merged pixel count != m (lost partial) */
  DT_GUARD_CRITIC_LOSS = 6,
  DT_GUARD_BN_BWD = 7,       /* a BatchNorm's dgamma / dbeta / dbias */
  DT_GUARD_CRITIC_GRAD = 8,
  DT_GUARD_CRITIC_PARAM = 9,
  DT_GUARD_ACTOR_LOSS = 10,
  DT_GUARD_ACTOR_GRAD = 11,
  DT_GUARD_ACTOR_PARAM = 12,
  DT_GUARD_TD = 13           /* the TD error (-> update_priorities) */
};

/* One scan: for each of the n (<= DT_GUARD_MAX) tensors, OR (1 << bit) into
 * guard[0] if any of its count elements is NaN or +-Inf.  dtype 0 = float32,
 * 1 = float64.  The table is passed by value (captured into a HIP graph as
 * kernel arguments). */
#define DT_GUARD_MAX 8
typedef struct dt_guard_tensor {
  const void* p;
  int64_t count;
  int32_t bit;
  int32_t dtype;
} dt_guard_tensor;
int dt_guard_scan(int32_t n, const dt_guard_tensor* tensors, int32_t* guard, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AIDO1_AMD_DTTRAIN_H */
