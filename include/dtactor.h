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

/* dt_conv1: the actor's first layer, conv_2d(3 -> 32, 8x8, stride 2) + bias +
 * LeakyReLU (config.json actor; duckietown_rl/ddpg.py:36,56), read straight
 * from the observation ring: channel c of the stack is ring slot order[c]
 * (oldest first, the Transformer order).  An MFMA implicit GEMM in fp16 with
 * f32 accumulation (aido1_amd/csrc/dtconv.hip).
 *   ring      device f32 [n, slots, 120, 160]
 *   wfrag     device fp16 [16, 64, 8]: the weights as the MFMA A fragments,
 *             element [s][l][j] = w[co = l%32][c = j%4][ky = s/2]
 *             [kx = 4*(s%2) + 2*(l/32) + j/4], 0 for c = 3 (aido1_amd/actor.py)
 *   bias      device f32 [32]
 *   y         device fp16 [n, 57, 77, 32] (NHWC)
 *   partials  device f32 [n, 32, 3] or NULL (reference mode): the sample's
 *             per-channel (mean, M2, c) for dt_conv1_norm and dt_conv32 layer
 *             2.  With partials, y holds the LeakyReLU outputs CENTRED: v - c,
 *             c = the sample's pixel-0 output of the channel, and mean is the
 *             mean of the stored (centred) values; M2 is shift-free.  So the
 *             next BatchNorm's (y - mean) * invstd is the uncentred one, and a
 *             nearly flat channel (tiny std) does not amplify the fp16
 *             rounding of |v| but only of |v - c|. */
int dt_conv1(const float* ring, int32_t n, int32_t slots, const int32_t* order, const void* wfrag,
             const float* bias, void* y, float* partials, float slope, void* stream);

/* dt_conv1_norm: the train-mode batch-of-one BatchNorm after conv1 (as
 * dt_sample_norm) from dt_conv1's per-sample statistics; y is normalised in
 * place. */
int dt_conv1_norm(void* y, int32_t n, const float* partials, const float* gamma,
                  const float* beta, float eps, void* stream);

/* dt_conv32: conv2 / conv3 / conv4 of the actor (layer = 2, 3, 4: conv_2d
 * 32 -> 32, 4x4, strides 2, 2, 1) + bias + LeakyReLU, MFMA fp16 with f32
 * accumulation, NHWC fp16 in and out (aido1_amd/csrc/dtconv.hip): persistent
 * workgroups stream whole samples through an LDS ring of input rows.
 *   wfrag      device fp16 [32, 64, 8] A fragments: [s][l][j] =
 *              w[l%32][16*(s%2) + 8*(l/32) + j][(s/2)/4][(s/2)%4]
 *   prev_part  the previous layer's statistics [n, 32, 3] (dt_conv1's partials for
 *              layer 2, this call's `part` of layer 2 / 3 for 3 / 4) or NULL:
 *              with it, the previous BatchNorm (in_gamma, in_beta, in_eps) is
 *              applied per sample while the input is staged (reference mode)
 *   part       layers 2, 3 with prev_part: out [n, 32, 3], the sample's
 *              per-channel (mean, M2, c), y centred as dt_conv1's
 *   y          layers 2, 3: [n, OH, OW, 32]; layer 4: [n, 32*9*14] flattened in
 *              NCHW order, normalised by (out_gamma, out_beta, out_eps) when
 *              prev_part is given (the last BatchNorm, whole sample in-kernel)
 * Without prev_part the layer is the eval-mode one (BatchNorms folded into
 * the weights by the caller). */
int dt_conv32(int32_t layer, int32_t n, const void* x, const void* wfrag, const float* bias,
              const float* prev_part, const float* in_gamma, const float* in_beta, float in_eps,
              void* y, float* part, const float* out_gamma, const float* out_beta,
              float out_eps, float slope, void* stream);

/* A second weight set for the samples [n0, n) of one dt_conv1_split /
 * dt_conv32_split launch.  config.json:183-186 runs 7 exploring and 1
 * exploiting explorer, and the exploiters act with their own copy of the
 * weights (the target model, training/explorers.py:104-105), so one decision
 * runs the actor with two weight sets.  The persistent workgroups are split
 * in proportion to the two sample counts and each loads one set; every
 * sample's result is the one a separate launch with its set gives.  The
 * layouts are those of the launch's own arguments; in_* / out_* are
 * dt_conv32's (NULL exactly where the launch's are). */
typedef struct dt_conv_set {
  int32_t n0;               /* samples [0, n0) use the launch's weights */
  const void* wfrag;        /* [n0, n): these */
  const float* bias;
  const float* in_gamma;
  const float* in_beta;
  const float* out_gamma;
  const float* out_beta;
} dt_conv_set;

/* dt_conv1 with an optional second weight set (set2 NULL = dt_conv1). */
int dt_conv1_split(const float* ring, int32_t n, int32_t slots, const int32_t* order,
                   const void* wfrag, const float* bias, const dt_conv_set* set2, void* y,
                   float* partials, float slope, void* stream);

/* dt_conv1_split on a ring of palette-index frames (u8 [n, slots, 120, 160],
 * dt_render_io.index): each byte is decoded to its grey level
 * (dt_palette_gray) as the rows are staged, so y and partials equal
 * dt_conv1_split's on the grey ring of the same frames bit for bit, from a
 * quarter of its input bytes. */
int dt_conv1_index_split(const uint8_t* ring, int32_t n, int32_t slots, const int32_t* order,
                         const void* wfrag, const float* bias, const dt_conv_set* set2, void* y,
                         float* partials, float slope, void* stream);

/* dt_conv32 with an optional second weight set (set2 NULL = dt_conv32). */
int dt_conv32_split(int32_t layer, int32_t n, const void* x, const void* wfrag,
                    const float* bias, const float* prev_part, const float* in_gamma,
                    const float* in_beta, float in_eps, void* y, float* part,
                    const float* out_gamma, const float* out_beta, float out_eps, float slope,
                    const dt_conv_set* set2, void* stream);

/* dt_conv1x_split / dt_conv32x_split: the same four convolutions at the
 * reference's float32 accuracy (models/ddpg/model.py:79-88 acts in float32;
 * duckietown_rl/ddpg.py:44-62), reference mode only (train-mode batch-of-one
 * BatchNorms), on fp16 MFMA (aido1_amd/csrc/dtconvx.hip).  Every f32 operand x
 * is an fp16 pair hi = fp16(x), lo = fp16((x - hi) * 2^11) (x = hi + 2^-11 lo
 * to 2^-24 |x|) and every product three fp16 MFMA products accumulated in f32:
 * ah*bh + 2^-11 (ah*bl + al*bh).  Activations between layers use the "HLB"
 * layout, 4 B an element like f32: fp16 [n, H, 4, 2, P, 8], for each image row
 * 4 blocks of 8 channels, each a hi segment and a lo segment of P 8-channel
 * chunks; pixel x is chunk x of a segment when the consumer reads the image
 * at stride 1 (P = W), and chunk x / 2 (even x) or (W + 1) / 2 + x / 2 (odd x)
 * at stride 2 (P = 2 ((W + 1) / 2)), so a wave's 32 pixels of one k step are
 * contiguous.  Values are centred on the sample's pixel 0 as dt_conv1's.
 *
 * dt_conv1x_split: conv1 + bias + LeakyReLU from the frame ring, as
 * dt_conv1_split / dt_conv1_index_split (index != 0: palette-index u8 frames,
 * else grey f32).
 *   wfrag     device fp16 [2, 16, 64, 8]: dt_conv1's fragment layout, first
 *             the hi halves of the f32 weights, then the lo halves
 *   y         device fp16 HLB [n, 57, 4, 2, 78, 8] (read at stride 2), centred
 *   partials  device f32 [n, 32, 3] (required): (mean, M2, c) as dt_conv1's
 *   set2      the second weight set (wfrag in this layout) or NULL.
 * Assumes |w| < 65504 (an fp16 hi of a larger weight overflows). */
int dt_conv1x_split(const void* ring, int32_t index, int32_t n, int32_t slots,
                    const int32_t* order, const void* wfrag, const float* bias,
                    const dt_conv_set* set2, void* y, float* partials, float slope, void* stream);

/* dt_conv32x_split: conv2 / conv3 / conv4 (layer 2, 3, 4) as dt_conv32_split
 * in reference mode.  The previous layer's BatchNorm (prev_part, in_gamma,
 * in_beta, in_eps; all required) is folded per sample into the weights: w' =
 * w * sc[c] (scaled by a power of two when the sample's largest |w'| would
 * leave fp16's range), bias' = bias + sum_k w * sh[c].
 *   x      device fp16 HLB (dt_conv1x_split's y, or this call's y of layer
 *          2 / 3)
 *   wfrag  device f32 [32, 64, 8]: dt_conv32's fragment layout in float32
 *   y, part  layers 2, 3: HLB [n, 27, 4, 2, 38, 8] (read at stride 2) /
 *          [n, 12, 4, 2, 17, 8] (stride 1), centred, and (mean, M2, c)
 *          [n, 32, 3]; layer 4: f32 [n, 32*9*14] flattened in NCHW order,
 *          normalised by (out_gamma, out_beta, out_eps) (required), part NULL */
int dt_conv32x_split(int32_t layer, int32_t n, const void* x, const float* wfrag,
                     const float* bias, const float* prev_part, const float* in_gamma,
                     const float* in_beta, float in_eps, void* y, float* part,
                     const float* out_gamma, const float* out_beta, float out_eps, float slope,
                     const dt_conv_set* set2, void* stream);

/* dt_actor_head_x3: the actor's output branch at float32 accuracy, for n
 * samples in one launch (config.json actor: flatten -> dropout -> linear(4032
 * -> 512) -> leaky_relu -> linear(512 -> 2) -> tanh; duckietown_rl/ddpg.py:
 * 56-62):  out[i] = head(lrelu(x[i] . w1^T + b1) . w2^T + b2), rows [0, n0)
 * with the first weight set, [n0, n) with the second.  lin1 on fp16 MFMA as
 * dt_conv1x_split's products (x3), lin2 and the head in f32.
 *   x      device f32 [n, k], k = 4032 (dropout already applied)
 *   w1*    device fp16 [2, 16, 252, 64, 8]: lin1's weights [512, 4032] as
 *          (hi, lo) MFMA A fragments, element [q][t][s][l][j] = half q of
 *          w1[32 t + l % 32][16 s + 8 (l / 32) + j] (aido1_amd/actor.py)
 *   b1*    device f32 [512]; w2* device f32 [2, 512]; b2* device f32 [2]
 *   head   0 none, 1 tanh, 2 sigmoid; out device f32 [n, 2]
 *   work   device f32 [dt_actor_head_x3_work_floats(n)]: lin1's partial sums
 *          (four K quarters) between the two launches it makes */
int dt_actor_head_x3(int32_t n, int32_t n0, int32_t k, const float* x, const void* w1a,
                     const float* b1a, const float* w2a, const float* b2a, const void* w1b,
                     const float* b1b, const float* w2b, const float* b2b, int32_t head,
                     float slope, float* work, float* out, void* stream);
int64_t dt_actor_head_x3_work_floats(int32_t n);
/* dt_actor_head_x3 with reference mode's dropout before lin1 folded in (ABI
 * 13): x[i][j] is kept where u >= p and scaled by 1 / (1 - p), u a 16-bit
 * uniform from a counter-based hash of (seed, i * k + j) -- F.dropout(x, p)'s
 * bernoulli(1 - p) mask and scale (duckietown_rl/ddpg.py:56-62 in train mode),
 * with its own generator.  0 <= p < 1 (0: no dropout).  x is read in place,
 * the dropped rows never written. */
int dt_actor_head_x3_drop(int32_t n, int32_t n0, int32_t k, const float* x, float p,
                          uint32_t seed, const void* w1a, const float* b1a, const float* w2a,
                          const float* b2a, const void* w1b, const float* b1b, const float* w2b,
                          const float* b2b, int32_t head, float slope, float* work, float* out,
                          void* stream);
/* The fp16 fast mode's head in the same two launches (ABI 13): x device fp16
 * [n, k]; w1* the hi half of dt_actor_head_x3's fragment layout ([16, 252,
 * 64, 8] fp16 from the fp16 lin1 weights); b1*, w2*, b2* device fp16; one
 * fp16 MFMA a product with f32 accumulation, the same folded dropout; the
 * lin1 output kept in f32 (the library-GEMM path it replaces rounded it to
 * fp16).  work: dt_actor_head_x3_work_floats(n). */
int dt_actor_head_f16_drop(int32_t n, int32_t n0, int32_t k, const void* x, float p,
                           uint32_t seed, const void* w1a, const void* b1a, const void* w2a,
                           const void* b2a, const void* w1b, const void* b1b, const void* w2b,
                           const void* b2b, int32_t head, float slope, float* work, float* out,
                           void* stream);

/* dt_explore: SingleThreadExplorer's action choice for n explorers at once,
 * one fused pass replacing the torch restatement's ~25 element-wise kernels
 * (aido1_amd/explore.py explore_actions + rollout.CycleEpsilon; the same
 * operations in the same order, so the two agree bit for bit):
 *   epsilon  = clip(cycle decay of episode[i], final, initial)
 *              (training/explorers.py:92-111, utils/util.py:36-40)
 *   OU step  x += theta (mu - x) dt + max(m steps + c, sigma_min) sqrt(dt) z,
 *              steps += 1 (utils/random_process.py:42-47)
 *   action   = clip(float(actor_out + (2 if tanh) * (eps * float(x))))
 *              (models/ddpg/model.py:74-102: the noise is float64, the sum
 *              rounded once to float32, as numpy 2 evaluates it)
 *   every_second_random (coin != NULL): even explorer ids take uni[i] when
 *              coin[i] < ratio * eps in float64 (explorers.py:178-194)
 *   actor_out f32 [n, 2]; normals f64 [n, 2]; coin f64 [n], uni f32 [n, 2]
 *   ou_x f64 [n, 2] and ou_steps f64 [n] updated in place; episode i64 [n];
 *   cycle, max_step f64 [n]; explorer_id i64 [n]; actions f32 [n, 2] out. */
typedef struct DtExploreParams {
  double pi, eps_span, eps_final, eps_initial;          /* eps_span = initial - final */
  double ou_m, ou_c, ou_sigma_min, ou_sqrt_dt, ou_theta, ou_mu, ou_dt;
  double eps_ratio;                                     /* epsilon_ratio */
  int32_t head;                                         /* 0 tanh, 1 sigmoid, 2 none */
} DtExploreParams;

int dt_explore(int32_t n, const float* actor_out, const double* normals, const double* coin,
               const float* uni, double* ou_x, double* ou_steps, const int64_t* episode,
               const double* cycle, const double* max_step, const int64_t* explorer_id,
               const DtExploreParams* params, float* actions, void* stream);

/* dt_explore_done: after the step, (tanh_map) actions = actions / 2 + 0.5 in
 * place (utils/env_wrappers.py:214-216), and every explorer with done[i]
 * gets its OU state zeroed and episode[i] += 1 (explorers.py:170). */
int dt_explore_done(int32_t n, const uint8_t* done, double* ou_x, int64_t* episode,
                    float* actions, int32_t tanh_map, void* stream);

/* dt_episode_account: the explorers' per-episode accounting for n envs, after
 * each decision (training/explorers.py:118-123 start an episode at zero,
 * :202-204 add every decision's (reward, reward_modified) and one step, the
 * episode ends with done; utils/env_wrappers.py:251 keeps total_reward).
 * Replaces the Python float sums of one SingleThreadExplorer per env.
 *   reward, reward_mod  device f64 [k, n]: dt_step's outputs (k = 1), or
 *                       dt_step_many's k decisions (decision d at [d * n])
 *   done                device u8 [k, n]
 * Per env, in decision order: sums += (reward, reward_mod) in f64, decisions
 * += 1, tick += 1; on done one record (below) is written to the ring at slot
 * count % capacity (count += 1, a device atomic), and the sums restart.  An
 * env that finishes several episodes inside one k-chunk writes one record
 * for each.  Records of one call are in no particular order: (tick, env)
 * orders them.  The caller owns and zero-initialises every array.  The
 * reference's episode reward divides by reward_scale and multiplies steps by
 * repeat_actions (explorers.py:135-140); the host does that, in f64. */
typedef struct DtEpisodeRecord {
  double reward;            /* sum of the episode's decision rewards */
  double reward_modified;   /* sum of its reward_mod */
  int64_t tick;             /* the env's decisions so far, this one included */
  int64_t episode;          /* the env's episode index (0-based) */
  int32_t env;              /* env index in [0, n) */
  int32_t decisions;        /* decisions in the episode */
} DtEpisodeRecord;

typedef struct DtEpisodeState {
  double* reward;               /* [n] running sums of the current episode */
  double* reward_modified;      /* [n] */
  int64_t* tick;                /* [n] */
  int64_t* episode;             /* [n] finished episodes */
  int32_t* decisions;           /* [n] */
  uint64_t* count;              /* [1] records written since creation */
  DtEpisodeRecord* ring;        /* [capacity] */
  int64_t capacity;             /* >= 1 */
} DtEpisodeState;

int dt_episode_account(int32_t n, int32_t k, const double* reward, const double* reward_mod,
                       const uint8_t* done, const DtEpisodeState* state, void* stream);

/* dt_refresh_copy: FusedActor.refresh (reference mode) in one launch: every
 * acting tensor (the MFMA weight fragments, biases, BatchNorm affine
 * parameters, the linears in fp16) gathered and converted from the source
 * actor's float32 parameters.  table: device [n] entries; entry e writes
 * count elements of dst (in its physical order) from src (float32): element
 * i = src[map[i]] (map device int64 [count], -1 = 0.0), or src[i] with map
 * NULL; dst_dtype 0 float32, 1 fp16 (round to nearest), 2 the x3 pair of
 * dt_conv1x_split (fp16 hi = fp16(v) at dst[i], lo = fp16((v - hi) * 2^11)
 * at dst[count + i]: dst holds 2 * count fp16).  max_count: the largest
 * count (the grid's width). */
typedef struct DtCopyEntry {
  const void* src;
  void* dst;
  const int64_t* map;
  int64_t count;
  int32_t dst_dtype;
  int32_t pad;
} DtCopyEntry;

int dt_refresh_copy(int32_t n, const DtCopyEntry* table, int64_t max_count, void* stream);

/* dt_actor_head: the actor's output branch after its first linear
 * (config.json actor: leaky_relu -> linear(512 -> 2) -> tanh;
 * duckietown_rl/ddpg.py:58-62) for n samples in one launch, one wave each:
 *   out[i] = head(leaky(h[i]) . w2^T + b2), rows [0, n0) with (w2a, b2a), rows
 *   [n0, n) with (w2b, b2b) (the second weight set of dt_conv1_split).
 *   h      device fp16 [n, ld] (the first linear's output, bias included), k
 *          inputs used (k, ld multiples of 8)
 *   w2*    device fp16 [2, k]; b2* device fp16 [2]
 *   head   0 none, 1 tanh, 2 sigmoid; slope the LeakyReLU's negative slope
 *   out    device f32 [n, 2]
 * LeakyReLU is rounded to fp16 and the pre-head value to fp16, as the fp16
 * tensors of the torch path are; the dot products accumulate in f32. */
int dt_actor_head(int32_t n, int32_t n0, int32_t k, const void* h, int32_t ld, const void* w2a,
                  const void* b2a, const void* w2b, const void* b2b, int32_t head, float slope,
                  float* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AIDO1_AMD_DTACTOR_H */
