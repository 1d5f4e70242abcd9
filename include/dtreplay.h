/* dtreplay.h — C-ABI of the GPU prioritized replay.
 *
 * Replaces, for the batched DDPG path, the index side of
 *   utils/buffers.py:140-259   PrioritizedReplayBuffer (add / sample / update_priorities)
 *   utils/segment_tree.py:94-146 SumSegmentTree + MinSegmentTree
 * The payload (observations, actions, ...) lives in caller-owned device tensors
 * indexed by the slots these calls return (aido1_amd/replay.py).
 *
 * Layout in HBM: two float64 trees of 2*capacity nodes each (node 1 = root,
 * leaf i at capacity + i, as segment_tree.py:34), an int32[capacity] scratch
 * used to resolve duplicate indices in one update, and the float64 running
 * max priority.  All state stays on the device: add / sample / update are
 * stream-ordered and never synchronise.
 *
 * Conventions as dtsim.h: every call returns 0 or a negative DT_E_* code,
 * device pointers belong to the handle's GPU, work goes on `stream`
 * (a hipStream_t, NULL = default stream).
 */
#ifndef AIDO1_AMD_DTREPLAY_H
#define AIDO1_AMD_DTREPLAY_H

#include <stdint.h>

#include "dtsim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dt_per dt_per;

/* PrioritizedReplayBuffer(size, alpha) — buffers.py:141-167: capacity = next
 * power of two >= size, sum tree 0, min tree +inf, max_priority 1. */
int dt_per_create(int64_t size, double alpha, int32_t device, dt_per** out);
void dt_per_destroy(dt_per* h);
const char* dt_per_last_error(const dt_per* h);
int64_t dt_per_capacity(const dt_per* h);
int64_t dt_per_len(const dt_per* h);      /* len(buffer._storage) */
int64_t dt_per_next_idx(const dt_per* h); /* buffer._next_idx */

/* n consecutive add() calls — buffers.py:169-174 + ReplayBuffer.add :29-36:
 * slot k = (next_idx + k) % size gets leaf max_priority**alpha in both trees.
 * slots_dev (int64[n], may be NULL) receives each add's slot; when n > size
 * later adds overwrite earlier ones, so the payload of add k belongs in
 * slots[k] only if k >= n - size. */
int dt_per_add(dt_per* h, int64_t n, int64_t* slots_dev, void* stream);

/* sample(batch, beta) — buffers.py:176-235 with random.random() replaced by
 * u_dev[batch] (float64 in [0,1)): mass = u * sum(0, len - 1) (leaves
 * 0..len-2, the reference's reduce() end quirk), idx = find_prefixsum_idx(mass)
 * (segment_tree.py:106-132), weight = (p_idx * len)^-beta / (p_min * len)^-beta.
 * Needs len >= 2 (the reference recurses forever at len 1). */
int dt_per_sample(dt_per* h, int32_t batch, const double* u_dev, double beta, int64_t* idx_dev,
                  double* weights_dev, void* stream);

/* update_priorities(idx, priorities) — buffers.py:237-259: leaf = p**alpha
 * (the last occurrence of a duplicated index wins, as the sequential loop),
 * max_priority = max(max_priority, p).  Entries the reference would reject
 * (p <= 0 or NaN, idx outside [0, len)) are skipped, flagged and counted
 * for dt_per_check. */
int dt_per_update(dt_per* h, int32_t n, const int64_t* idx_dev, const double* priorities_dev,
                  void* stream);

/* dt_per_update with priorities |td[i]| + eps (td device float32 [n], the
 * trainer's TD errors; the float32 absolute value widened to float64, then
 * + eps: what update_priorities(idx, abs(td) + eps) stores). */
int dt_per_update_td(dt_per* h, int32_t n, const int64_t* idx, const float* td, double eps,
                     void* stream);

/* Copy out the trees (float64[2*capacity] each; NULL to skip) and the max
 * priority (float64[1]) — tests and checkpointing. */
int dt_per_read(dt_per* h, double* sum_dev, double* min_dev, double* max_priority_dev,
                void* stream);

/* Synchronises; DT_E_ARG if an update since the last check held an entry the
 * reference's asserts reject (message in dt_per_last_error: the kinds and how
 * many entries were skipped). */
int dt_per_check(dt_per* h);

/* dt_frame_add: one decision of the frame store behind
 * ReplayBuffer.add_batch_ring (aido1_amd/replay.py, frame_envs).  Replaces the
 * two stacked observation copies buffers.py:29-36 stores per transition
 * (obs_t, obs_tp1; the Transformer stack of 3 frames each): a decision adds
 * ONE frame per env, and a transition keeps frame-row indices instead.
 *   src        device, env e's newest frame at src + e * src_env_stride
 *              4-byte words (the rollout ring's newest slot); frames are copied
 *              as opaque words: f32 grey, or 4 u8 palette-index pixels a word
 *              (dt_render_io.index); frame_elems words a frame, a multiple of
 *              4, src and dst 16-B aligned
 *   dst        device [n, frame_elems] words: frame rows base_row .. base_row + n - 1
 *   stack      device int32 [n, k]: each env's current stack as frame rows
 *              (oldest first), advanced in place
 *   done       device uint8 [n] or NULL: respawned envs, whose whole stack
 *              becomes the new row (the renderer refilled every slot)
 *   obs_ptr    device int32 [n, k] out: the stack before (the transition's obs)
 *   next_ptr   device int32 [n, k] out: the stack after (its next_obs) */
int dt_frame_add(int32_t n, int64_t frame_elems, const void* src, int64_t src_env_stride,
                 void* dst, int32_t k, int32_t* stack, const uint8_t* done, int32_t base_row,
                 int32_t* obs_ptr, int32_t* next_ptr, void* stream);

/* dt_frame_gather: a sampled batch of the frame store straight into the
 * update's inputs (ReplayBuffer._encode_sample, buffers.py:38-52, then
 * DDPGTrainer's float32 channels_last inputs, trainers.py:156-163), one
 * launch instead of the index_selects, the layout change, the casts and the
 * copies into the captured graph's static inputs.  For b < batch, i = idx[b]:
 *   obs[b][y][x][c] = frames[obs_ptr[i][c]][y * w + x]   (c < k; NHWC: the
 *   nxt[b][y][x][c] = frames[next_ptr[i][c]][...]         channels_last memory
 *                                                          of [batch, k, h, w])
 *   act[b][j] = action[i][j] (j < 2), rew[b] = (float)reward[i],
 *   notdone[b] = done[i] ? 0 : 1
 *   idx device i64 [batch] in [0, size) (unchecked: dt_per_sample's output);
 *   frames [rows, hw]: frame_kind 0 f32 grey, 1 u8 palette-index frames
 *   (dt_render_io.index), decoded through dt_palette_gray's table (so the
 *   output equals kind 0's on the grey frames bit for bit); obs_ptr /
 *   next_ptr i32 [size, k]; action f32 [size, 2]; reward f64 [size]; done u8
 *   [size] (torch bool); k <= 4 */
int dt_frame_gather(int32_t batch, const int64_t* idx, const void* frames, int32_t frame_kind,
                    int64_t hw, int32_t k, const int32_t* obs_ptr, const int32_t* next_ptr,
                    const float* action, const double* reward, const uint8_t* done, float* obs,
                    float* nxt, float* act, float* rew, float* notdone, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AIDO1_AMD_DTREPLAY_H */
