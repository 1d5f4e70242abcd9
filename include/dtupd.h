/* dtupd.h — C-ABI of the DDPG update's convolutions (SURVEY.md §8f 1,
 * BASELINE configs[4]): hand-written f32 MFMA kernels for the conv_2d layers
 * of config.json's actor and critic (3 -> 32 8x8 stride 2; 32 -> 32 4x4
 * strides 2 and 1; padding 0, no dilation or groups), forward and both
 * gradients, in place of MIOpen (training/trainers.py:143-237 runs every
 * network in train mode through torch's conv2d and its autograd).
 *
 * Layout: NHWC float32 (torch channels_last), batch n, C_out = 32.  The
 * weight is w[co][kh][kw][ci] (a channels_last [32, C_in, KS, KS] tensor),
 * i.e. [32][K] with K = KS * KS * C_in, the im2col order of an input patch.
 * OH = (IH - KS) / ST + 1, OW likewise.  Supported (C_in, KS, ST): (3, 8, 2),
 * (32, 4, 2), (32, 4, 1); DT_E_ARG otherwise.
 *
 * Numerics: v_mfma_f32_32x32x2_f32, an exact f32 fma chain per output over
 * its K products (the order differs from a CPU or MIOpen convolution, as
 * theirs differ from each other); no TF32-like rounding exists on gfx950.
 *
 * Conventions as dtsim.h: 0 or a negative DT_E_* code; device pointers; work
 * goes on `stream` (a hipStream_t).
 */
#ifndef AIDO1_AMD_DTUPD_H
#define AIDO1_AMD_DTUPD_H

#include <stdint.h>

#include "dtsim.h"

#ifdef __cplusplus
extern "C" {
#endif

/* z[n][oy][ox][co] = sum_k x[n][ST*oy + kh][ST*ox + kw][ci] * w[co][k]  (no bias)
 *   x  device f32 [n, IH, IW, C_in];  w  device f32 [32, K];  z  device f32 [n, OH, OW, 32] */
int dt_upd_conv_fwd(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                    const float* x, const float* w, float* z, void* stream);

/* dt_upd_conv_fwd plus the block's train-mode BatchNorm statistics, fused
 * into its epilogue (config.json's conv_2d -> leaky_relu -> batch_norm_2d):
 * exactly dt_bn_leaky_fwd's statistics part (include/dttrain.h) -- batch
 * mean / biased variance of a = leaky_relu(z + bias, slope) over the
 * n * OH * OW pixels into mean_invstd [64], running_mean / running_var moved
 * `updates` times, num_batches_tracked += updates, DT_GUARD_BN_* reports --
 * without a second pass over z.  dt_bn_leaky_apply then normalises.
 *   work  dt_upd_bn_work_floats() floats, zeroed once (left reusable); not
 *         shared with dt_bn_leaky_fwd's (another partial layout) */
int dt_upd_conv_fwd_bn(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                       const float* x, const float* w, const float* bias, float slope, float eps,
                       float momentum, float* running_mean, float* running_var,
                       int64_t* num_batches_tracked, int32_t updates, float* z,
                       float* mean_invstd, float* work, int32_t* guard, void* stream);

int64_t dt_upd_bn_work_floats(void);

/* ---- a chain of blocks (the conv trunk) ---------------------------------------------
 * Block j's BatchNorm statistics leave its forward as per-workgroup partials
 * and are merged by the NEXT kernel, which normalises while it loads:
 *   dt_upd_conv_fwd_part(block j + 1's conv, x = z_j, in = block j's BN) reads
 *   z_j, applies y_j = bn_j(leaky(z_j + bias_j)) to every value it loads, and
 *   writes z_{j+1} and block j + 1's partials; its first workgroup writes
 *   block j's mean_invstd, running statistics, num_batches_tracked and guard
 *   reports;
 *   dt_upd_bn_finish(last block) merges the last partials and writes y.
 * y_j itself is never stored: dt_upd_conv_wgrad_bn normalises z_j the same
 * way when it stages block j + 1's input rows.  Values equal the
 * block-by-block path's (dt_upd_conv_fwd_bn + dt_bn_leaky_apply) bit for bit:
 * same partials, same merge order, same formula. */
typedef struct DtUpdBn {
  const float* part;             /* the producer's partials [parts][32][3] */
  int32_t parts;                 /* as dt_upd_conv_fwd_part returned them */
  int64_t m;                     /* pixels the partials cover (n * OH * OW) */
  const float* bias;             /* conv bias [32] (added before leaky_relu) */
  const float* gamma;            /* BatchNorm weight [32] */
  const float* beta;             /* BatchNorm bias [32] */
  float slope, eps, momentum;
  float* running_mean;           /* [32], moved `updates` times */
  float* running_var;
  int64_t* num_batches_tracked;  /* may be NULL */
  int32_t updates;
  float* mean_invstd;            /* [64] out: batch mean, 1 / sqrt(biased var + eps) */
  int32_t* guard;                /* DT_GUARD_BN_COUNT / _FWD reports; may be NULL */
} DtUpdBn;

/* floats of one partials buffer (any layer) */
int64_t dt_upd_part_floats(void);

/* z = conv(x') with x' = x (in == NULL: the observation) or bn_in(leaky(x +
 * bias_in)) (in: the previous block); this block's statistics of
 * leaky(z + bias) go to part ([dt_upd_part_floats()]), *parts = how many. */
int dt_upd_conv_fwd_part(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                         const float* x, const DtUpdBn* in, const float* w, const float* bias,
                         float slope, float* z, float* part, int32_t* parts, void* stream);

/* y = bn(leaky(z + bias)) for the chain's last block (z [m, 32]): merges
 * bn->part and writes mean_invstd / running statistics as above.  y is laid
 * out as z (hw = 0) or NCHW, [m / hw][32][hw] (hw = pixels a sample: the
 * flatten after the trunk is then a view) */
int dt_upd_bn_finish(int64_t m, int32_t hw, const float* z, const DtUpdBn* bn, float* y,
                     void* stream);

/* dt_upd_conv_wgrad with the input x' = bn_in(leaky(x + bias_in)) made while
 * staging (in->mean_invstd as the forward wrote it; in == NULL: x as is) */
int dt_upd_conv_wgrad_bn(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                         const float* x, const DtUpdBn* in, const float* dz, float* dw,
                         float* work, void* stream);

/* Floats of scratch dt_upd_conv_wgrad needs for these dimensions (per-chunk
 * partial weight gradients, reduced in a fixed order: deterministic). */
int64_t dt_upd_wgrad_work_floats(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih,
                                 int32_t iw);

/* dw[co][k] = sum over the n * OH * OW output pixels of dz[pixel][co] * the
 * pixel's input patch x[...][k] (torch.nn.grad.conv2d_weight).
 *   dz device f32 [n, OH, OW, 32];  dw device f32 [32, K] out, 16-B aligned;
 *   work device f32 [dt_upd_wgrad_work_floats(...)], 16-B aligned */
int dt_upd_conv_wgrad(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                      const float* x, const float* dz, float* dw, float* work, void* stream);

/* dx[n][ih][iw][ci] = sum over the (co, kh, kw) with ih = ST*oy + kh,
 * iw = ST*ox + kw inside the output of dz[n][oy][ox][co] * w[co][kh][kw][ci]
 * (torch.nn.grad.conv2d_input); C_in = 32 only (the first layer's input is
 * the observation, which needs no gradient).  Every dx element is written.
 *   dz device f32 [n, OH, OW, 32];  w [32, K];  dx device f32 [n, IH, IW, 32] out */
int dt_upd_conv_dgrad(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                      const float* dz, const float* w, float* dx, void* stream);

/* ---- the linear layer after the trunk -------------------------------------------------
 * y[m][n] = act(b[n] + sum_k x[m][k] w[n][k]) (torch.nn.Linear: x [M, K],
 * w [N, K] row-major; act = the following LeakyReLU(slope) when leaky != 0,
 * else none), K split over waves and the slices summed in a fixed order
 * (deterministic); for config.json's flatten -> dropout -> linear 4032 ->
 * 256 (critic) or 512 (actor) -> leaky_relu, where the batch M is small and
 * K long.  N % 32 == 0, K % 32 == 0.
 *   work  dt_upd_linear_work_floats(m, n, k) floats;  b may be NULL */
int64_t dt_upd_linear_work_floats(int32_t m, int32_t n, int32_t k);
int dt_upd_linear_fwd(int32_t m, int32_t n, int32_t k, const float* x, const float* w,
                      const float* b, int32_t leaky, float slope, float* y, float* work,
                      void* stream);
/* dx[m][k] = sum_n g[m][n] w[n][k], g = dy through the fused LeakyReLU when
 * yact (the forward's output y) is given, else dy */
int dt_upd_linear_dgrad(int32_t m, int32_t n, int32_t k, const float* dy, const float* w,
                        const float* yact, float slope, float* dx, void* stream);
/* dw[n][k] = sum_m g[m][n] x[m][k]; db[n] = sum_m g[m][n] (db may be NULL) */
int dt_upd_linear_wgrad(int32_t m, int32_t n, int32_t k, const float* dy, const float* x,
                        const float* yact, float slope, float* dw, float* db, void* stream);

/* The forward and the input gradient with the dropout before the linear
 * folded in (config.json's flatten -> dropout(p) -> linear; ABI 12).
 *   u   device f32 [m, k] uniforms in [0, 1), 16-B aligned, or NULL (no
 *       dropout): element (i, j) of x is kept where u[i][j] >= p and then
 *       scaled by 1 / (1 - p) -- torch's F.dropout with the bernoulli(1 - p)
 *       mask {u >= p} -- on x's loads in the forward and on dx's stores in
 *       the input gradient.  0 <= p < 1.
 *   xd  device f32 [m, k] out or NULL: the dropped input, written by the
 *       forward for the weight gradient (dt_upd_linear_wgrad with x = xd).
 * Replaces the dropout + nn.Linear pair of the reference's MetaNet
 * (models/ddpg/modules.py) as training/trainers.py runs it: no separate
 * dropout kernel, no dropout backward. */
int dt_upd_linear_fwd_drop(int32_t m, int32_t n, int32_t k, const float* x, const float* u,
                           float p, float* xd, const float* w, const float* b, int32_t leaky,
                           float slope, float* y, float* work, void* stream);
int dt_upd_linear_dgrad_drop(int32_t m, int32_t n, int32_t k, const float* dy, const float* w,
                             const float* yact, float slope, const float* u, float p, float* dx,
                             void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AIDO1_AMD_DTUPD_H */
