// libdtsim: MI355X-native batched Duckietown environment — step/reset kernels
// and the C ABI declared in include/dtsim.h.
//
// One wavefront lane per environment; 64-thread workgroups (one wave each) so
// a 4096-env batch spreads over 64 CUs instead of piling onto 16; the map's
// tile kinds, Bezier control points and headings are staged in LDS per block;
// pose state is float64 SoA in HBM (coalesced 8-B lanes); done/reset masks are
// wave ballots; resets are wave-cooperative rejection sampling (see
// dtsim_common.h wave_spawn).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "dthandle.h"

static std::string g_create_err;

namespace {

using dt::MapLds;

// Diagnostic build only (-DDTSIM_STAMPS, tools/step_stamps.sh): wave 0 of the
// first 64 step blocks records the shader clock at fixed points of the step.
#ifdef DTSIM_STAMPS
constexpr int kStamps = 16;
__device__ unsigned long long g_stamps[64 * kStamps];
#define STAMP(i)                                                                    \
  do {                                                                              \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                     \
    if (threadIdx.x == 0 && blockIdx.x < 64) g_stamps[blockIdx.x * kStamps + (i)] = _t; \
  } while (0)
__device__ unsigned long long g_rstamps[4096 * 4];  // refill blocks: entry, exit, items
#define RFSTAMP(b, i, v)                                                            \
  do {                                                                              \
    if (threadIdx.x == 0 && (b) < 4096) g_rstamps[(b) * 4 + (i)] = (v);             \
  } while (0)
#define RSTAMP(i)                                                                   \
  do {                                                                              \
    const unsigned long long _t = __builtin_amdgcn_s_memrealtime();                 \
    if (threadIdx.x == 0 && blockIdx.x < 64) g_stamps[blockIdx.x * kStamps + (i)] = _t; \
  } while (0)
// step_fan_kernel: lane 0 of each wave of the first 64 blocks, decisions 0..7:
// [block][wave][decision][point] shader clock; point 15 of decision 0 = real
// time at entry, of decision 1 = real time at exit
constexpr int kPDec = 8;
__device__ unsigned long long g_pstamps[64 * 4 * kPDec * 16];
#define PSTAMP(d, i, v)                                                             \
  do {                                                                              \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 64 && (d) >= 0 && (d) < kPDec)      \
      g_pstamps[((blockIdx.x * 4 + (threadIdx.x >> 6)) * kPDec + (d)) * 16 + (i)] = (v); \
  } while (0)
#define PSTAMPT(d, i) PSTAMP(d, i, __builtin_amdgcn_s_memtime())
// every block of step_fan_kernel: entry / exit real time, HW_ID, XCC_ID
__device__ unsigned long long g_bstamps[4096 * 4];
__device__ inline unsigned hw_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
}
__device__ inline unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v;
}
#define BSTAMP(i, v)                                                                 \
  do {                                                                              \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_bstamps[blockIdx.x * 4 + (i)] = (v); \
  } while (0)
#else
#define BSTAMP(i, v) \
  do {               \
  } while (0)
#define PSTAMP(d, i, v) \
  do {                  \
  } while (0)
#define PSTAMPT(d, i) PSTAMP(d, i, 0)
#define STAMP(i) \
  do {           \
  } while (0)
#define RSTAMP(i) STAMP(i)
#define RFSTAMP(b, i, v) STAMP(i)
#endif

__device__ inline void map_action(int mode, float a0, float a1, double& vl, double& vr) {
  if (mode == DT_ACTION_TANH) {
    // utils/env_wrappers.py:214-216: in-place float32 `action /= 2; action += 0.5`
    a0 = a0 / 2.0f;
    a0 = a0 + 0.5f;
    a1 = a1 / 2.0f;
    a1 = a1 + 0.5f;
    vl = (double)a0;
    vr = (double)a1;
  } else if (mode == DT_ACTION_STEERING) {
    // duckietown_rl/wrappers.py:138-161 then ActionWrapper :99-101 (left wheel x0.8)
    const double vel = (double)a0, ang = (double)a1;
    const double kinv_r = (1.0 + 0.0) / 27.0, kinv_l = (1.0 - 0.0) / 27.0;
    const double om_r = (vel + 0.5 * ang * 0.102) / 0.0318;
    const double om_l = (vel - 0.5 * ang * 0.102) / 0.0318;
    double ur = om_r * kinv_r, ul = om_l * kinv_l;
    ur = ur < 1.0 ? ur : 1.0;
    ur = ur > -1.0 ? ur : -1.0;
    ul = ul < 1.0 ? ul : 1.0;
    ul = ul > -1.0 ? ul : -1.0;
    vl = ul * 0.8;
    vr = ur;
  } else {
    vl = (double)a0;
    vr = (double)a1;
  }
}

// Spawn-ahead reset (A13).  Each env keeps a window of kSlots
// precomputed reset poses: key j (the episode counter the env has when it takes
// that reset) lives in slot j % kSlots, tagged with the env's launch tick at the
// time it was written.  want[e] - 1 is the env's episode counter as its last
// launch left it; the window is the keys [want - 1, want - 1 + kSlots).
//
// refill_group refills envs [e0, e0 + ne) with one 256-thread block: the first
// ne lanes read want, the slot words, tick and seed of one env each and list
// the window's missing keys; the block stages the map only when the list is
// not empty and computes the items: one with all 256 threads (spawn_block: one
// round of 256 proposals almost always holds the first accepted one), several
// with one wave each in parallel (spawn_one).
//
// Race-free against the step lanes of the same launch:
//  * a step lane consumes a slot only if an earlier launch wrote it (tag older
//    than the lane's tick; a refill of the same launch tags with the tick it
//    reads, which is >= the lane's), so it never reads a slot being written;
//  * a refill writes only slots whose key is outside the window it read, and
//    a lane moves its window (want store) only after its last slot loads
//    returned.
// A standalone refill (dt_seed, dt_reset: no step lane runs) tags tick - 1,
// usable by the next launch.
constexpr int kBlock = 256;        // step and refill blocks (4 waves)

__device__ inline void put_slot(const dt::State& st, int n, int e, uint32_t key, bool ok,
                                uint32_t tag, double x, double z, double a, double dist,
                                double arad) {
#if defined(DTSIM_DIAG_SKIP_STORES) && (DTSIM_DIAG_SKIP_STORES & 16)
  return;   // diagnostic build: no refill stores
#endif
  const size_t sl = key % (uint32_t)dt::kSlots;
  double* p = st.pre + sl * dt::kSlotRec * (size_t)n + e;
  double sa = 0.0, ca = 1.0;
  sincos(a, &sa, &ca);
  p[0] = x;
  p[(size_t)n] = z;
  p[2 * (size_t)n] = a;
  p[3 * (size_t)n] = dist;
  p[4 * (size_t)n] = arad;
  p[5 * (size_t)n] = sa;
  p[6 * (size_t)n] = ca;
  const uint64_t w = ((uint64_t)tag << 32) | (ok ? key : (key | dt::kKeyFailed));
  __hip_atomic_store(st.pre_key + sl * n + e, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#ifndef DTSIM_REFILL_ENVS
#define DTSIM_REFILL_ENVS 8
#endif
constexpr int kRefillEnvs = DTSIM_REFILL_ENVS;  // envs scanned per refill block
constexpr int kMaxItems = dt::kSlots * kRefillEnvs;

__device__ int refill_group(const dt::State& st, const dt::MapDev& md, const dt::Geo& g, int n,
                             uint32_t max_attempts, uint32_t env_base, int e0, int ne,
                             uint32_t tag_back, unsigned char* lds) {
  __shared__ int32_t item_env[kMaxItems];
  __shared__ uint32_t item_key[kMaxItems];
  __shared__ uint32_t item_tag[kMaxItems];
  __shared__ uint64_t item_seed[kMaxItems];
  __shared__ int32_t n_items;
  __shared__ double scratch[6 * (kBlock / 64)];
  const int tid = threadIdx.x;
  if (tid == 0) n_items = 0;
  __syncthreads();
  const int e = e0 + tid;
  if (tid < ne && e < n) {
    const uint32_t w = __hip_atomic_load(st.want + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t tag =
        __hip_atomic_load(st.tick + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - tag_back;
    uint32_t have[dt::kSlots];
#pragma unroll
    for (int s = 0; s < dt::kSlots; ++s)
      have[s] = (uint32_t)__hip_atomic_load(st.pre_key + (size_t)s * n + e, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t seed = st.seed[e];
#pragma unroll
    for (int i = 0; i < dt::kSlots; ++i) {
      const uint32_t key = w - 1u + (uint32_t)i;
      if ((i > 0 || w > 0u) && (have[key % (uint32_t)dt::kSlots] & ~dt::kKeyFailed) != key) {
        const int slot = atomicAdd(&n_items, 1);
        item_env[slot] = e;
        item_key[slot] = key;
        item_tag[slot] = tag;
        item_seed[slot] = seed;
      }
    }
  }
  __syncthreads();
  const int cnt = n_items;
  if (cnt == 0) return 0;  // block-uniform
  const dt::MapLds M = dt::stage_map(md, lds);
  if (cnt == 1) {  // all four waves on the one item
    double x = 0.0, z = 0.0, a = 0.0, dist = 0.0, arad = 0.0;
    const bool ok = dt::spawn_block(M, g, max_attempts, env_base + (uint32_t)item_env[0],
                                    item_seed[0], item_key[0], scratch, x, z, a, dist, arad);
    if (tid == 0) put_slot(st, n, item_env[0], item_key[0], ok, item_tag[0], x, z, a, dist, arad);
  } else {  // several: one wave per item (64 proposals per round), waves in parallel
    const int wave = tid >> 6, nw = (int)(blockDim.x >> 6);
    for (int it = wave; it < cnt; it += nw) {  // wave-uniform
      double x = 0.0, z = 0.0, a = 0.0, lp[2] = {0.0, 0.0};
      const bool ok = dt::spawn_one(M, g, max_attempts, env_base + (uint32_t)item_env[it],
                                    item_seed[it], item_key[it], x, z, a, lp);
      if ((tid & 63) == 0)
        put_slot(st, n, item_env[it], item_key[it], ok, item_tag[it], x, z, a, lp[0], lp[1]);
    }
  }
  return cnt;
}

__global__ __launch_bounds__(kBlock) void refill_kernel(dt::State st, dt::MapDev md, dt::Geo g,
                                                        int n, uint32_t max_attempts,
                                                        uint32_t env_base) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  refill_group(st, md, g, n, max_attempts, env_base, (int)blockIdx.x * kRefillEnvs, kRefillEnvs,
               1u, lds);
}

// 0, available only once v's load has returned (the asm reads v).
__device__ inline uint32_t after_load(double v) {
  uint32_t z;
  asm volatile("v_mov_b32 %0, 0 ; %1" : "=v"(z) : "v"(v));
  return z;
}

// One EnvironmentWrapper.step of one lane: repeat x frame_skip Simulator steps
// (A4 _update_pos, A11 _compute_done_reward) and the BaselineAggregation of
// their rewards (utils/env_wrappers.py:213-253).  c, s = cos, sin of ang on
// entry and on exit.
struct Decision {
  double tr, trm;  // reward sum, aggregated reward x reward_scale
  bool dn;
  unsigned nsim;   // Simulator steps run
  // lane position of the last reward computation; valid while the pose has not
  // moved since (reused for the terminal output instead of a 4th bisection)
  bool lp_fresh, lp_inl;
  double lp[4];
};

__device__ __forceinline__ void sim_decision(const MapLds& M, const dt::Geo& g, const StepCfg& sc,
                                             bool active, float2 a, double& x, double& z,
                                             double& ang, double& c, double& s,
                                             uint32_t& step_count, uint32_t& env_step,
                                             Decision& D) {
  double vl, vr;
  map_action(sc.action_mode, a.x, a.y, vl, vr);
  if (sc.clip) {  // Simulator.step: np.clip(action, -1, 1)
    vl = vl < -1.0 ? -1.0 : (vl > 1.0 ? 1.0 : vl);
    vr = vr < -1.0 ? -1.0 : (vr > 1.0 ? 1.0 : vr);
  }
  const double wl = vl * g.robot_speed * 1.0, wr = vr * g.robot_speed * 1.0;
  const bool straight = (wl == wr);
  double w_rot = 0.0, r_icc = 0.0, rot = 0.0, cr = 1.0, sr = 0.0;
  if (!straight) {  // _update_pos terms that do not depend on the pose (A4)
    const double l = g.wheel_dist;
    w_rot = (wr - wl) / l;
    r_icc = (l * (wl + wr)) / (2.0 * (wl - wr));
    rot = w_rot * g.dt;
    sincos(rot, &sr, &cr);
  }
  const double kstraight = g.dt * wl;
  STAMP(2);

  double tr = 0.0, trm = 0.0;
  bool dn = !active;
  unsigned nsim = 0;
  double* lp = D.lp;
  bool lp_fresh = false, lp_inl = false;
  for (int rep = 0; rep < sc.repeat; ++rep) {
    const bool live = !dn;
    if (live) {
      double speed = 0.0;
      for (int f = 0; f < sc.frame_skip; ++f) {
        const double ox = x, oz = z;
        if (straight) {
          x = x + kstraight * c;
          z = z + kstraight * (-s);
        } else {
          const double cx = x + r_icc * s;
          const double cz = z + r_icc * c;
          const double ddx = x - cx, ddz = z - cz;
          const double ndx = ddx * cr + ddz * sr;
          const double ndz = ddz * cr - ddx * sr;
          x = cx + ndx;
          z = cz + ndz;
          ang = ang + rot;
          sincos(ang, &s, &c);
        }
        step_count += 1u;
        nsim += 1u;
        if (rep == 1) STAMP(11);
        if (sc.speed_measured) {
          const double a1 = x - ox, a3 = z - oz;
          speed = sqrt((a1 * a1 + 0.0 * 0.0) + a3 * a3) / g.dt;
        }
      }
      // _compute_done_reward (A11).  get_lane_pos2 of the new pose is computed
      // beside _valid_pose (independent float64 chains) and used only if the
      // pose is valid.
      double lq[4] = {0.0, 0.0, 0.0, 0.0};
      const bool lq_inl = dt::lane_pos<false>(M, g, x, z, c, s, lq);
      const bool vp = dt::valid_pose(M, g, x, z, c, s, 1.0);
      if (rep == 1) STAMP(12);
      lp_fresh = false;
      double r;
      bool sd = false;
      if (!vp) {
        r = -1000.0;
        sd = true;
      } else if (step_count >= sc.max_steps) {
        r = 0.0;
        sd = true;
      } else {
        const double sp = sc.speed_measured ? speed : g.robot_speed;
        // compute_reward: proximity_penalty2 at the actual centre (0 without objects)
        const double pen =
            M.n_obj ? dt::proximity_penalty(M, g, x + g.off * c, z + g.off * (-s)) : 0.0;
        lp_fresh = true;
        lp_inl = lq_inl;
        lp[0] = lq[0];
        lp[1] = lq[1];
        lp[2] = lq[2];
        lp[3] = lq[3];
        if (rep == 1) STAMP(13);
        if (lp_inl) {
          const double ad = fabs(lp[0]);
          r = ((1.0 * sp) * lp[1] + (-10.0) * ad) + 40.0 * pen;
        } else {
          r = 40.0 * pen;
        }
      }
      // BaselineAggregationFunction (aggregation_functions.py:25-32)
      const double rm = (r == -1000.0) ? -10.0 : (r > 0.0 ? r + 10.0 : r + 4.0);
      tr = tr + r;
      trm = trm + rm;
      env_step += 1u;
      dn = sd || env_step > sc.max_env_steps;
    }
    STAMP(3 + (rep < 3 ? rep : 2));
  }
  D.tr = tr;
  D.trm = trm * sc.reward_scale;
  D.dn = dn;
  D.nsim = nsim;
  D.lp_fresh = lp_fresh;
  D.lp_inl = lp_inl;
}

// EnvironmentWrapper.step (utils/env_wrappers.py:213-253) x repeat
// Simulator.step, k decisions in one launch (dt_step: k = 1; dt_step_many).
// The pose, counters and spawn-ahead bookkeeping stay in registers across the
// decisions and the map is staged once.  Outputs of decision d are at
// [d * n + env].  Blocks past n_step_blocks are the spawn-ahead refill.
__global__ __launch_bounds__(kBlock) void step_kernel(dt::State st, dt::MapDev md, dt::Geo g,
                                                  StepCfg sc, int n, uint32_t env_base, int k,
                                                  const float2* __restrict__ act,
                                                  double* __restrict__ rew,
                                                  double* __restrict__ rewm,
                                                  uint8_t* __restrict__ done_out,
                                                  float2* __restrict__ obs,
                                                  double* __restrict__ lanepos,
                                                  int32_t* __restrict__ tile_out,
                                                  int n_step_blocks, uint32_t max_attempts,
                                                  const uint8_t* __restrict__ step_mask) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  // blocks past the step's: the spawn-ahead refill, kRefillEnvs envs each,
  // running on the CUs the step leaves idle (block-uniform branch)
  if ((int)blockIdx.x >= n_step_blocks) {
    const int rb = (int)blockIdx.x - n_step_blocks;
    RFSTAMP(rb, 0, __builtin_amdgcn_s_memrealtime());
    const int items = refill_group(st, md, g, n, max_attempts, env_base, rb * kRefillEnvs,
                                   kRefillEnvs, 0u, lds);
    RFSTAMP(rb, 1, __builtin_amdgcn_s_memrealtime());
    RFSTAMP(rb, 2, (unsigned long long)items);
    (void)items;
    return;
  }
  // the step waves win issue arbitration against refill waves sharing their SIMD
  __builtin_amdgcn_s_setprio(3);
  RSTAMP(9);
  STAMP(0);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool in_range = e < n;
  // envs outside step_mask (dt_step_masked) are left exactly as they were
  const bool active = in_range && (step_mask == nullptr || step_mask[e] != 0);
  const int ei = in_range ? e : 0;

  // state and the spawn-ahead slot words are loaded before the map is staged,
  // so their latency hides behind it
  double x = st.x[ei], z = st.z[ei], ang = st.angle[ei];
  uint32_t step_count = st.step_count[ei], env_step = st.env_step[ei];
  float2 a = act[ei];
  const uint32_t tick = st.tick[ei];
  uint32_t key = 0u;
  uint64_t seed = 0u, words[dt::kSlots];
  if (sc.auto_reset) {
    key = st.episode[ei];
    seed = st.seed[ei];
#pragma unroll
    for (int q = 0; q < dt::kSlots; ++q)
      words[q] = __hip_atomic_load(st.pre_key + (size_t)q * n + ei, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }
  const MapLds M = dt::stage_map(md, lds);
  STAMP(1);
  // bit i: key + i is ready (written by an earlier launch); of those, failed
  const uint32_t key0 = key;
  uint32_t ready = 0u, failed = 0u;
  if (sc.auto_reset) {
#pragma unroll
    for (int q = 0; q < dt::kSlots; ++q) {
      const uint32_t kw = (uint32_t)words[q], tag = (uint32_t)(words[q] >> 32);
      const uint32_t rel = (kw & ~dt::kKeyFailed) - key;
      if (rel < (uint32_t)dt::kSlots && (int32_t)(tick - tag) > 0) {
        ready |= 1u << rel;
        if (kw & dt::kKeyFailed) failed |= 1u << rel;
      }
    }
  }

  double c = 0.0, s = 0.0;
  sincos(ang, &s, &c);
  unsigned nsim_t = 0, act_t = 0, resets_t = 0, dones_t = 0;
  double rp[dt::kSlotRec] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0};
  for (int d = 0; d < k; ++d) {
    // the next decision's action and this decision's reset pose (if ready),
    // loaded while the decision runs
    const float2 an = act[(size_t)(d + 1 < k ? d + 1 : d) * n + ei];
    const uint32_t rel = key - key0;
    const bool slot_ready = rel < (uint32_t)dt::kSlots && ((ready >> rel) & 1u) != 0u;
    if (slot_ready) {
      const size_t sl = key % (uint32_t)dt::kSlots;
#pragma unroll
      for (int q = 0; q < dt::kSlotRec; ++q) rp[q] = st.pre[(sl * dt::kSlotRec + q) * (size_t)n + ei];
    }
    asm volatile("" ::: "memory");  // keep the loads here, ahead of the decision

    Decision D;
    sim_decision(M, g, sc, active, a, x, z, ang, c, s, step_count, env_step, D);

    // auto-reset (VectorEnv): a finished env takes the reset pose of its next
    // spawn key; a key not ready is computed here, the whole wave on one env
    const bool want_reset = active && D.dn && sc.auto_reset;
    bool ok = slot_ready && ((failed >> rel) & 1u) == 0u;
    uint64_t need = __ballot(want_reset && !slot_ready);
    while (need) {  // wave-uniform
      const int l = __ffsll((unsigned long long)need) - 1;
      need &= need - 1u;
      const uint32_t el = (uint32_t)__shfl(ei, l), kl = (uint32_t)__shfl((int)key, l);
      const uint64_t sd = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(seed >> 32), l) << 32) |
                          (uint64_t)(uint32_t)__shfl((int)(uint32_t)seed, l);
      double sx = 0.0, sz = 0.0, sa = 0.0, slp[2] = {0.0, 0.0};
      const bool sok = dt::spawn_one(M, g, max_attempts, env_base + el, sd, kl, sx, sz, sa, slp);
      if (lane == l) {
        rp[0] = sx;
        rp[1] = sz;
        rp[2] = sa;
        rp[3] = slp[0];
        rp[4] = slp[1];
        sincos(sa, &rp[5], &rp[6]);
        ok = sok;
      }
    }
    const bool reset_now = want_reset && ok;
    if (want_reset && !ok) atomicOr(st.err, dt::kErrSpawn);  // failed: env stays put

    // terminal lane pose: the obs of an env that stays, and the optional lanepos
    // output; an env being reset reports its reset pose's obs instead
    const bool need_lp = lanepos != nullptr || (obs != nullptr && !reset_now);
    bool inl = false;
    if (D.lp_fresh) {  // same pose as the last reward: only the angle is missing
      inl = D.lp_inl;
      if (inl && need_lp) dt::finish_angle(g, D.lp);
    } else if (active && need_lp) {
      inl = dt::lane_pos<true>(M, g, x, z, c, s, D.lp);
    }
    STAMP(6);
    if (active) {
      const size_t o = (size_t)d * n + e;
      rew[o] = D.tr;
      rewm[o] = D.trm;
      done_out[o] = (uint8_t)D.dn;
      if (lanepos) {
        const double nan = __longlong_as_double(0x7ff8000000000000LL);
        double* lo = lanepos + 4 * o;
        lo[0] = inl ? D.lp[0] : nan;
        lo[1] = inl ? D.lp[1] : nan;
        lo[2] = inl ? D.lp[2] : nan;
        lo[3] = inl ? D.lp[3] : nan;
      }
      if (tile_out) tile_out[o] = dt::tile_of(M, g, x, z);
      if (obs)
        obs[o] = reset_now ? make_float2((float)rp[3], (float)rp[4])
                           : (inl ? make_float2((float)D.lp[0], (float)D.lp[3])
                                  : make_float2(0.0f, 0.0f));
    }
    if (reset_now) {
      x = rp[0];
      z = rp[1];
      ang = rp[2];
      s = rp[5];  // sincos(ang), made with the slot
      c = rp[6];
      step_count = 0u;
      env_step = 0u;
      key += 1u;
    }
    nsim_t += D.nsim;
    act_t += active ? 1u : 0u;
    resets_t += reset_now ? 1u : 0u;
    dones_t += (active && D.dn) ? 1u : 0u;
    a = an;
  }
  STAMP(7);
  const unsigned kk = (unsigned)k;
  dt::wave_count(st.stats + 0, nsim_t, kk * (unsigned)(sc.repeat * sc.frame_skip));
  dt::wave_count(st.stats + 1, act_t, kk);
  dt::wave_count(st.stats + 2, resets_t, kk);
  dt::wave_count(st.stats + 3, dones_t, kk);
  if (in_range) {
    if (active) {
      st.x[e] = x;
      st.z[e] = z;
      st.angle[e] = ang;
      st.step_count[e] = step_count;
      st.env_step[e] = env_step;
    }
    __hip_atomic_store(st.tick + e, tick + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (key != key0) {
      st.episode[e] = key;
      // the window moves past the consumed keys only once the slot loads have
      // returned: the store's value depends on the last of them (loads return
      // in order)
      __hip_atomic_store(st.want + e, key + 1u + after_load(rp[dt::kSlotRec - 1]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  STAMP(8);
  RSTAMP(10);
}

// dt_step_many in fan mode (the default): 16 envs per 256-thread workgroup,
// each env on one lane quad of each of the block's four waves.  Within a
// decision the poses of the repeat (<= 3) Simulator steps do not depend on any
// validity or lane-pose result (those only decide whether a step is kept), so
// every wave computes the pose chain -- the quad computes the decision's
// sincos(rot) and the three sincos(angle) on its four lanes at once -- and the
// step math fans out: wave 0 runs _valid_pose of the three poses (a drivable
// probe per lane), wave r (1..3) get_lane_pos2 of pose r (three bisection
// levels per round on the quad) and its acos.  One barrier per decision swaps
// the results through LDS; then every wave runs the same reward / done /
// aggregation chain over the steps actually taken, the same reset, and writes
// its share of the outputs.  4096 envs are 1024 waves, one per SIMD.
// Bit-identical to step_kernel (the same operations on the same operands;
// tests/test_gpu_step.py runs all three kernels).
constexpr int kFanEnvs = 16;                // envs per workgroup
constexpr int kFanBlock = 4 * 64;           // four waves
constexpr int kFanSteps = 3;                // repeat * frame_skip handled
constexpr int kFanMaxK = 64;                // decisions per launch (actions staged in LDS)

struct FanX {  // [parity][env][step], rows padded to 4 for wide LDS reads
  double dist[2][kFanEnvs][4], dot[2][kFanEnvs][4], arad[2][kFanEnvs][4], pen[2][kFanEnvs][4];
  uint8_t inl[2][kFanEnvs][4], vp[2][kFanEnvs][4];
  double park[kFanBlock][9];   // a lane's values across an in-loop spawn
};

// kLean: the common configuration as compile-time facts (wheel-velocity
// actions clipped to [-1, 1], the nominal speed in the reward, auto-reset, no
// collidable objects); the generic instantiation reads them from StepCfg / the map
template <bool kLean>
__global__ __launch_bounds__(kFanBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void step_fan_kernel(dt::State st, dt::MapDev md,
                                                             dt::Geo g, StepCfg sc, int n,
                                                             uint32_t env_base, int k,
                                                             const float2* __restrict__ act,
                                                             double* __restrict__ rew,
                                                             double* __restrict__ rewm,
                                                             uint8_t* __restrict__ done_out,
                                                             float2* __restrict__ obs,
                                                             double* __restrict__ pose_out,
                                                             int n_step_blocks,
                                                             uint32_t max_attempts,
                                                             uint32_t map_lds_offset) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
#ifdef DTSIM_STAMPS
  BSTAMP(0, __builtin_amdgcn_s_memrealtime());
  BSTAMP(2, hw_id());
  BSTAMP(3, xcc_id());
#endif
  if ((int)blockIdx.x >= n_step_blocks) {  // spawn-ahead refill blocks
    refill_group(st, md, g, n, max_attempts, env_base,
                 ((int)blockIdx.x - n_step_blocks) * kRefillEnvs, kRefillEnvs, 0u, lds);
    BSTAMP(1, __builtin_amdgcn_s_memrealtime());
    return;
  }
  __shared__ FanX X;
  __builtin_amdgcn_s_setprio(3);
  PSTAMP(0, 15, __builtin_amdgcn_s_memrealtime());
  PSTAMP(3, 15, __builtin_amdgcn_s_memtime());
  const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const int q = lane & 3, le = lane >> 2;
  const int e = (int)blockIdx.x * kFanEnvs + le;
  const bool active = e < n;
  const int ei = active ? e : 0;
  const bool lead = q == 0;   // the lane of the quad that stores

  double x = st.x[ei], z = st.z[ei], ang = st.angle[ei];
  uint32_t step_count = st.step_count[ei], env_step = st.env_step[ei];
  const uint32_t tick = st.tick[ei];
  uint32_t key = 0u;
  uint64_t seed = 0u, words[dt::kSlots];
  if (sc.auto_reset) {
    key = st.episode[ei];
    seed = st.seed[ei];
#pragma unroll
    for (int j = 0; j < dt::kSlots; ++j)
      words[j] = __hip_atomic_load(st.pre_key + (size_t)j * n + ei, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  }
  // staged in LDS behind the map image: the block's spawn-ahead slot records
  // (the whole window; a lane reads only slots an earlier launch wrote, which
  // no block of this launch rewrites) and its actions of all k decisions
  // (k <= kFanMaxK; the host splits longer runs) -- no global load and no
  // prefetch register in the decision loop
  double* sslot = reinterpret_cast<double*>(lds + map_lds_offset);   // [kSlots*kSlotRec][16]
  float2* sact = reinterpret_cast<float2*>(sslot + dt::kSlots * dt::kSlotRec * kFanEnvs);
  {
    const int e0 = (int)blockIdx.x * kFanEnvs;
    for (int i = (int)threadIdx.x; i < k * kFanEnvs; i += kFanBlock) {
      const int dd = i / kFanEnvs, j = i % kFanEnvs;
      if (e0 + j < n) sact[i] = act[(size_t)dd * n + e0 + j];
    }
    if (sc.auto_reset)
      for (int i = (int)threadIdx.x; i < dt::kSlots * dt::kSlotRec * kFanEnvs; i += kFanBlock) {
        const int row = i / kFanEnvs, j = i % kFanEnvs;
        if (e0 + j < n) sslot[i] = st.pre[(size_t)row * n + e0 + j];
      }
  }
  const MapLds M = dt::stage_map(md, lds);   // its barrier also covers sact
  const uint32_t key0 = key;
  uint32_t ready = 0u, failed = 0u;
  if (sc.auto_reset) {
#pragma unroll
    for (int j = 0; j < dt::kSlots; ++j) {
      const uint32_t kw = (uint32_t)words[j], tag = (uint32_t)(words[j] >> 32);
      const uint32_t rel = (kw & ~dt::kKeyFailed) - key;
      if (rel < (uint32_t)dt::kSlots && (int32_t)(tick - tag) > 0) {
        ready |= 1u << rel;
        if (kw & dt::kKeyFailed) failed |= 1u << rel;
      }
    }
  }

  double c = 0.0, s = 0.0;
  sincos(ang, &s, &c);
  unsigned nsim_t = 0, act_t = 0, resets_t = 0, dones_t = 0;
  double rp[dt::kSlotRec] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0};
  const int R = sc.repeat;
  const int act_mode = kLean ? DT_ACTION_WHEELS : sc.action_mode;
  const bool clip = kLean ? true : sc.clip != 0;
  const bool speed_measured = kLean ? false : sc.speed_measured != 0;
  const bool auto_reset = kLean ? true : sc.auto_reset != 0;
  const bool objs = kLean ? false : M.n_obj != 0;
  for (int d = 0; d < k; ++d) {
    const int par = d & 1;
    const float2 a = sact[d * kFanEnvs + le];
    const uint32_t rel = key - key0;
    const bool slot_ready = rel < (uint32_t)dt::kSlots && ((ready >> rel) & 1u) != 0u;
    PSTAMPT(d, 0);

    // ---- the pose chain (every wave) ----
    double vl, vr;
    map_action(act_mode, a.x, a.y, vl, vr);
    if (clip) {
      vl = vl < -1.0 ? -1.0 : (vl > 1.0 ? 1.0 : vl);
      vr = vr < -1.0 ? -1.0 : (vr > 1.0 ? 1.0 : vr);
    }
    const double wl = vl * g.robot_speed * 1.0, wr = vr * g.robot_speed * 1.0;
    const bool straight = (wl == wr);
    double r_icc = 0.0, rot = 0.0;
    if (!straight) {
      const double l = g.wheel_dist;
      const double w_rot = (wr - wl) / l;
      r_icc = (l * (wl + wr)) / (2.0 * (wl - wr));
      rot = w_rot * g.dt;
    }
    const double kstraight = g.dt * wl;
    // the angles of the three steps and the sincos of rot / angle 1..3, one per lane
    const double a1 = ang + rot, a2 = a1 + rot, a3 = a2 + rot;
    double sq = 0.0, cq = 1.0;
    if (!straight) sincos(q == 0 ? rot : (q == 1 ? a1 : (q == 2 ? a2 : a3)), &sq, &cq);
    const double sr = dt::qget<0>(sq), cr = dt::qget<0>(cq);
    double px[kFanSteps + 1], pz[kFanSteps + 1], pa[kFanSteps + 1], pc[kFanSteps + 1],
        ps[kFanSteps + 1], spd[kFanSteps + 1];
    px[0] = x;
    pz[0] = z;
    pa[0] = ang;
    pc[0] = c;
    ps[0] = s;
    spd[0] = 0.0;
    if (straight) {
#pragma unroll
      for (int r = 1; r <= kFanSteps; ++r) {
        px[r] = px[r - 1] + kstraight * c;
        pz[r] = pz[r - 1] + kstraight * (-s);
        pa[r] = ang;
        pc[r] = c;
        ps[r] = s;
      }
    } else {
      pa[1] = a1;
      pa[2] = a2;
      pa[3] = a3;
      ps[1] = dt::qget<1>(sq);
      pc[1] = dt::qget<1>(cq);
      ps[2] = dt::qget<2>(sq);
      pc[2] = dt::qget<2>(cq);
      ps[3] = dt::qget<3>(sq);
      pc[3] = dt::qget<3>(cq);
#pragma unroll
      for (int r = 1; r <= kFanSteps; ++r) {
        const double xo = px[r - 1], zo = pz[r - 1];
        const double cx = xo + r_icc * ps[r - 1];
        const double cz = zo + r_icc * pc[r - 1];
        const double ddx = xo - cx, ddz = zo - cz;
        const double ndx = ddx * cr + ddz * sr;
        const double ndz = ddz * cr - ddx * sr;
        px[r] = cx + ndx;
        pz[r] = cz + ndz;
      }
    }
    if (speed_measured) {
#pragma unroll
      for (int r = 1; r <= kFanSteps; ++r) {
        const double a1d = px[r] - px[r - 1], a3d = pz[r] - pz[r - 1];
        spd[r] = sqrt((a1d * a1d + 0.0 * 0.0) + a3d * a3d) / g.dt;
      }
    }

    PSTAMPT(d, 1);
    // ---- the step math, fanned out over the waves ----
    if (wave == 0) {
#pragma unroll
      for (int r = 1; r <= kFanSteps; ++r) {
        const bool vp = dt::valid_pose_q<!kLean>(M, g, q, px[r], pz[r], pc[r], ps[r], 1.0);
        const double pen = objs ? dt::proximity_penalty(M, g, px[r] + g.off * pc[r],
                                                        pz[r] + g.off * (-ps[r]))
                                : 0.0;
        if (lead) {
          X.vp[par][le][r - 1] = vp ? 1 : 0;
          X.pen[par][le][r - 1] = pen;
        }
      }
    } else {
      const int r = wave;
      double lp[4] = {0.0, 0.0, 0.0, 0.0};
      const bool inl = dt::lane_pos_q(M, g, q, px[r], pz[r], pc[r], ps[r], lp);
      if (lead) {
        X.inl[par][le][r - 1] = inl ? 1 : 0;
        X.dist[par][le][r - 1] = lp[0];
        X.dot[par][le][r - 1] = lp[1];
        X.arad[par][le][r - 1] = lp[3];
      }
    }
    PSTAMPT(d, 2);
    __syncthreads();
    PSTAMPT(d, 3);

    // ---- reward / done / aggregation over the steps taken (every wave) ----
    // every exchanged value is read at once (one wait), then the chain runs
    // on registers
    double xd[kFanSteps], xo[kFanSteps], xa[kFanSteps], xp[kFanSteps];
    bool xi[kFanSteps], xv[kFanSteps];
    {
      const uint32_t vpw = *reinterpret_cast<const uint32_t*>(X.vp[par][le]);
      const uint32_t inw = *reinterpret_cast<const uint32_t*>(X.inl[par][le]);
#pragma unroll
      for (int r = 0; r < kFanSteps; ++r) {
        xd[r] = X.dist[par][le][r];
        xo[r] = X.dot[par][le][r];
        xa[r] = X.arad[par][le][r];
        xp[r] = X.pen[par][le][r];
        xv[r] = ((vpw >> (8 * r)) & 0xFFu) != 0u;
        xi[r] = ((inw >> (8 * r)) & 0xFFu) != 0u;
      }
    }
    // branch-free: every step's reward is formed and kept only if the step
    // was taken (the same operations on the same operands as sim_decision)
    double tr = 0.0, trm = 0.0;
    bool dn = !active;
    unsigned nsim = 0;
    int last = 0;   // the pose the env ends the decision on (0: none taken)
    const double kR = g.robot_speed;
#pragma unroll
    for (int r = 1; r <= kFanSteps; ++r) {
      const bool live = !dn && r <= R;
      const uint32_t sc1 = step_count + 1u;
      const bool vp = xv[r - 1];
      const bool cap = sc1 >= sc.max_steps;
      const double sp = speed_measured ? spd[r] : kR;
      const double pen = xp[r - 1];
      const double ad = fabs(xd[r - 1]);
      const double rin = ((1.0 * sp) * xo[r - 1] + (-10.0) * ad) + 40.0 * pen;
      const double rout = 40.0 * pen;
      double rr = xi[r - 1] ? rin : rout;
      rr = cap ? 0.0 : rr;
      rr = vp ? rr : -1000.0;
      const bool sd = !vp || cap;
      const double rm = (rr == -1000.0) ? -10.0 : (rr > 0.0 ? rr + 10.0 : rr + 4.0);
      const double tr1 = tr + rr, trm1 = trm + rm;
      const uint32_t es1 = env_step + 1u;
      tr = live ? tr1 : tr;
      trm = live ? trm1 : trm;
      step_count = live ? sc1 : step_count;
      env_step = live ? es1 : env_step;
      nsim += live ? 1u : 0u;
      last = live ? r : last;
      dn = live ? (sd || es1 > sc.max_env_steps) : dn;
    }
    trm = trm * sc.reward_scale;
    double fx = x, fz = z, fa = ang, fc = c, fs = s;
    bool inl_last = false;
    double dist_last = 0.0, arad_last = 0.0;
#pragma unroll
    for (int r = 1; r <= kFanSteps; ++r)
      if (last == r) {
        fx = px[r];
        fz = pz[r];
        fa = pa[r];
        fc = pc[r];
        fs = ps[r];
        inl_last = xi[r - 1];
        dist_last = xd[r - 1];
        arad_last = xa[r - 1];
      }
    x = fx;
    z = fz;
    ang = fa;
    c = fc;
    s = fs;

    PSTAMPT(d, 4);
    // ---- auto-reset ----
    const bool want_reset = active && dn && auto_reset;
    bool ok = slot_ready && ((failed >> rel) & 1u) == 0u;
    if (want_reset && slot_ready) {
      const int sl = (int)(key % (uint32_t)dt::kSlots);
#pragma unroll
      for (int j = 0; j < dt::kSlotRec; ++j) rp[j] = sslot[(sl * dt::kSlotRec + j) * kFanEnvs + le];
    }
    uint64_t need = __ballot(want_reset && !slot_ready && lead);
    const bool parked = need != 0u;
    if (parked) {
      // the rare in-loop spawn needs ~60 more registers than the rest of the
      // loop: the decision's values that live across it wait in LDS (the
      // memory clobbers keep the compiler from forwarding them), else the
      // kernel spills to scratch on every launch
      double* pk = X.park[threadIdx.x];
      pk[0] = x; pk[1] = z; pk[2] = ang; pk[3] = c; pk[4] = s;
      pk[5] = tr; pk[6] = trm; pk[7] = dist_last; pk[8] = arad_last;
      asm volatile("" ::: "memory");
    }
    while (need) {  // wave-uniform; every wave computes the same spawns
      const int l = __ffsll((unsigned long long)need) - 1;
      need &= need - 1u;
      const uint32_t el = (uint32_t)__shfl(ei, l), kl = (uint32_t)__shfl((int)key, l);
      const uint64_t sd = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(seed >> 32), l) << 32) |
                          (uint64_t)(uint32_t)__shfl((int)(uint32_t)seed, l);
      double sx = 0.0, sz = 0.0, sa = 0.0, slp[2] = {0.0, 0.0};
      const bool sok = dt::spawn_one(M, g, max_attempts, env_base + el, sd, kl, sx, sz, sa, slp);
      if (le == (l >> 2)) {
        rp[0] = sx;
        rp[1] = sz;
        rp[2] = sa;
        rp[3] = slp[0];
        rp[4] = slp[1];
        sincos(sa, &rp[5], &rp[6]);
        ok = sok;
      }
    }
    if (parked) {
      asm volatile("" ::: "memory");
      const double* pk = X.park[threadIdx.x];
      x = pk[0]; z = pk[1]; ang = pk[2]; c = pk[3]; s = pk[4];
      tr = pk[5]; trm = pk[6]; dist_last = pk[7]; arad_last = pk[8];
    }
    const bool reset_now = want_reset && ok;
    if (wave == 0 && lead && want_reset && !ok) atomicOr(st.err, dt::kErrSpawn);

#ifndef DTSIM_DIAG_SKIP_STORES
#define DTSIM_DIAG_SKIP_STORES 0   // diagnostic builds only (tools/step_write_diag.sh)
#endif
    if (active && lead) {
      // 32-bit element indices (zero-extended into global_store's vector
      // offset): a size_t e kept its 64-bit form live through the loop
      const uint32_t o = (uint32_t)(d * n + e);
      if (wave == 0) {
        if (!(DTSIM_DIAG_SKIP_STORES & 1)) rew[o] = tr;
        if (!(DTSIM_DIAG_SKIP_STORES & 2)) rewm[o] = trm;
      } else if (wave == 1) {
        if (!(DTSIM_DIAG_SKIP_STORES & 4)) done_out[o] = (uint8_t)dn;
      } else if (wave == 2 && obs && !(DTSIM_DIAG_SKIP_STORES & 8)) {
        obs[o] = reset_now ? make_float2((float)rp[3], (float)rp[4])
                           : (inl_last ? make_float2((float)dist_last, (float)arad_last)
                                       : make_float2(0.0f, 0.0f));
      } else if (wave == 3 && pose_out) {
        // the pose the decision ends in (the reset pose after a respawn): what a
        // render of this decision draws, [d][x | z | angle][env]
        // 32-bit indices: a hoisted pose_out + e was another spill
        const uint32_t pi = (uint32_t)(d * 3 * n + e);
        pose_out[pi] = reset_now ? rp[0] : x;
        pose_out[pi + (uint32_t)n] = reset_now ? rp[1] : z;
        pose_out[pi + 2u * (uint32_t)n] = reset_now ? rp[2] : ang;
      }
    }
    x = reset_now ? rp[0] : x;
    z = reset_now ? rp[1] : z;
    ang = reset_now ? rp[2] : ang;
    s = reset_now ? rp[5] : s;
    c = reset_now ? rp[6] : c;
    step_count = reset_now ? 0u : step_count;
    env_step = reset_now ? 0u : env_step;
    key += reset_now ? 1u : 0u;
    nsim_t += nsim;
    act_t += active ? 1u : 0u;
    resets_t += reset_now ? 1u : 0u;
    dones_t += (active && dn) ? 1u : 0u;
    PSTAMPT(d, 5);
  }
  PSTAMP(1, 15, __builtin_amdgcn_s_memrealtime());
  PSTAMP(2, 15, __builtin_amdgcn_s_memtime());
  BSTAMP(1, __builtin_amdgcn_s_memrealtime());
  // every wave is past its last slot read before wave 0 moves the window
  __syncthreads();
  if (wave != 0) return;
  const unsigned kk = (unsigned)k;
  const unsigned m = lead ? 1u : 0u;
  dt::wave_count(st.stats + 0, nsim_t * m, kk * (unsigned)(sc.repeat * sc.frame_skip));
  dt::wave_count(st.stats + 1, act_t * m, kk);
  dt::wave_count(st.stats + 2, resets_t * m, kk);
  dt::wave_count(st.stats + 3, dones_t * m, kk);
  if (active && lead) {
    const uint32_t eu = (uint32_t)e;
    st.x[eu] = x;
    st.z[eu] = z;
    st.angle[eu] = ang;
    st.step_count[eu] = step_count;
    st.env_step[eu] = env_step;
    // tick re-read (only this lane writes it): kept live through the loop it
    // was a scratch spill
    const uint32_t tick_end = __hip_atomic_load(st.tick + eu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(st.tick + eu, tick_end + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (key != key0) {
      // the slot records were read into LDS before the staging barrier, so
      // the window can move
      st.episode[eu] = key;
      __hip_atomic_store(st.want + eu, key + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Simulator.reset + EnvironmentWrapper.reset counters (A13) for dt_reset: one
// 256-thread workgroup per env (flags NULL = every env, else envs with
// flags[e] != 0), so the envs respawn in parallel across the chip.  Afterwards
// want = the new counter + 1 and refill_kernel tops up the spawn-ahead slots.
constexpr int kSpawnThreads = 256;  // proposals per round: one accept in ~37, so ~1 round

__global__ __launch_bounds__(kSpawnThreads) void spawn_kernel(dt::State st, dt::MapDev md, dt::Geo g,
                                                   uint32_t max_attempts, uint32_t env_base,
                                                   const uint8_t* __restrict__ flags) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ double scratch[6 * (kSpawnThreads / 64)];
  if (flags != nullptr && flags[blockIdx.x] == 0) return;  // block-uniform
  const MapLds M = dt::stage_map(md, lds);
  const int e = (int)blockIdx.x;
  double x = 0.0, z = 0.0, ang = 0.0, dist = 0.0, arad = 0.0;
  const uint32_t episode = st.episode[e];
  const bool ok = dt::spawn_block(M, g, max_attempts, env_base + (uint32_t)e, st.seed[e], episode,
                                  scratch, x, z, ang, dist, arad);
  if (threadIdx.x == 0) {
    if (!ok) {
      atomicOr(st.err, dt::kErrSpawn);
    } else {
      st.x[e] = x;
      st.z[e] = z;
      st.angle[e] = ang;
      st.step_count[e] = 0u;
      st.env_step[e] = 0u;
      st.episode[e] = episode + 1u;
      st.want[e] = episode + 2u;
      atomicAdd(st.stats + 2, 1ull);
    }
  }
}

__global__ __launch_bounds__(64) void lane_pos_kernel(dt::State st, dt::MapDev md, dt::Geo g,
                                                      int n, double* __restrict__ lanepos,
                                                      int32_t* __restrict__ tile_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const MapLds M = dt::stage_map(md, lds);
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const double x = st.x[e], z = st.z[e], ang = st.angle[e];
  double s, c;
  sincos(ang, &s, &c);
  double lp[4];
  const bool inl = dt::lane_pos(M, g, x, z, c, s, lp);
  const double nan = __longlong_as_double(0x7ff8000000000000LL);
  if (lanepos) {
    for (int q = 0; q < 4; ++q) lanepos[4 * (size_t)e + q] = inl ? lp[q] : nan;
  }
  if (tile_out) tile_out[e] = dt::tile_of(M, g, x, z);
}

int grid_of(int n) { return (n + dt::kWave - 1) / dt::kWave; }
int refill_grid(int n, int ne) { return (n + ne - 1) / ne; }

}  // namespace

extern "C" {

#ifdef DTSIM_STAMPS
int dt_diag_stamps(unsigned long long* out) {  // 64 x kStamps shader-clock stamps
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) == hipSuccess ? 0 : -1;
}
int dt_diag_pstamps(unsigned long long* out) {  // step_fan_kernel per-wave stamps (g_pstamps)
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pstamps), sizeof(g_pstamps)) == hipSuccess ? 0 : -1;
}
int dt_diag_bstamps(unsigned long long* out) {  // step_fan_kernel per-block stamps
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bstamps), sizeof(g_bstamps)) == hipSuccess ? 0 : -1;
}
int dt_diag_rstamps(unsigned long long* out) {  // refill blocks: entry, exit (real time), items
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rstamps), sizeof(g_rstamps)) == hipSuccess ? 0
                                                                                          : -1;
}
#endif

int32_t dt_abi_version(void) { return DT_ABI_VERSION; }

int32_t dt_n_envs(const dt_handle* h) { return h ? h->n : -1; }

const char* dt_last_error(const dt_handle* h) {
  return h ? h->err.c_str() : g_create_err.c_str();
}

int dt_create(const dt_config* cfg, const dt_map* map, uint64_t seed, int32_t n_envs,
              int32_t device, dt_handle** out) {
  g_create_err.clear();
  if (!cfg || !map || !out || n_envs <= 0 || !map->kind || !map->curves || !map->headings ||
      !map->curve_start || map->width <= 0 || map->height <= 0) {
    g_create_err = "dt_create: bad argument";
    return DT_E_ARG;
  }
  const int T = map->width * map->height;
  if (T > dt::kMaxLdsTiles) {  // (also the render's LDS kind table)
    g_create_err = "dt_create: map larger than the LDS staging limit (256 tiles)";
    return DT_E_ARG;
  }
  if (cfg->repeat_actions < 1 || cfg->frame_skip < 1 || cfg->road_tile_size <= 0) {
    g_create_err = "dt_create: bad config";
    return DT_E_ARG;
  }
  // curve table: monotone, a drivable tile has curves, an off-road tile none
  if (map->curve_start[0] != 0) {
    g_create_err = "dt_create: curve_start[0] must be 0";
    return DT_E_ARG;
  }
  for (int t = 0; t < T; ++t) {
    const int32_t k = map->curve_start[t + 1] - map->curve_start[t];
    if (k < 0 || k > 12 || (map->kind[t] > 0) != (k > 0)) {
      g_create_err = "dt_create: tile " + std::to_string(t) + " has " + std::to_string(k) +
                     " curves for kind " + std::to_string(map->kind[t]);
      return DT_E_ARG;
    }
  }
  const int C = map->curve_start[T];
  // ground-plane curve records (dt::kCurveRec); the step math drops the y terms
  std::vector<double> rec((size_t)C * dt::kCurveRec);
  for (int k = 0; k < C; ++k) {
    const double* cp = map->curves + 12 * (size_t)k;
    const double* hd = map->headings + 3 * (size_t)k;
    if (cp[1] != 0.0 || cp[4] != 0.0 || cp[7] != 0.0 || cp[10] != 0.0 || hd[1] != 0.0) {
      g_create_err = "dt_create: curve " + std::to_string(k) + " leaves the ground plane (y != 0)";
      return DT_E_ARG;
    }
    double* r = rec.data() + (size_t)k * dt::kCurveRec;
    for (int i = 0; i < 4; ++i) {
      r[2 * i] = cp[3 * i];
      r[2 * i + 1] = cp[3 * i + 2];
    }
    for (int i = 0; i < 3; ++i) {  // bezier_tangent's differences, as it computes them
      r[8 + 2 * i] = cp[3 * (i + 1)] - cp[3 * i];
      r[8 + 2 * i + 1] = cp[3 * (i + 1) + 2] - cp[3 * i + 2];
    }
    r[14] = hd[0];
    r[15] = hd[2];
  }
  const int NO = map->n_objects, NS = map->n_spawn_objects;
  if (NO < 0 || NO > 256 || NS < 0 || NS > 256 || (NO > 0 && !map->objects) ||
      (NS > 0 && !map->spawn_objects)) {
    g_create_err = "dt_create: bad object tables (n_objects / n_spawn_objects in 0..256)";
    return DT_E_ARG;
  }
  if (NO > 0 && !(cfg->safety_rad_mult > 0.0)) {
    g_create_err = "dt_create: objects need safety_rad_mult > 0";
    return DT_E_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
    g_create_err = "dt_create: no HIP device " + std::to_string(device);
    return DT_E_NODEV;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    g_create_err = "dt_create: hipGetDeviceProperties failed";
    return DT_E_NODEV;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    g_create_err = std::string("dt_create: device is ") + prop.gcnArchName + ", need gfx950";
    return DT_E_NODEV;
  }
  std::vector<int16_t> drv;
  for (int t = 0; t < T; ++t)
    if (map->kind[t] > 0) drv.push_back((int16_t)t);
  if (drv.empty()) {
    g_create_err = "dt_create: map has no drivable tile";
    return DT_E_ARG;
  }

  dt_handle* h = new dt_handle();
  h->device = device;
  h->n = n_envs;
  h->cfg = *cfg;
  dt::Geo& g = h->geo;
  g.ts = cfg->road_tile_size;
  g.inv_ts = 1.0 / cfg->road_tile_size;
  g.wheel_dist = cfg->wheel_dist;
  g.dt = cfg->delta_time;
  g.off = cfg->camera_forward_dist - (cfg->robot_length / 2);
  g.robot_width = cfg->robot_width;
  g.front = cfg->front_probe_length ? cfg->robot_length : cfg->robot_width;
  g.rad2deg = cfg->rad2deg;
  g.two_pi = cfg->two_pi;
  g.accept_deg = cfg->accept_start_angle_deg;
  g.reset_safety = cfg->reset_safety;
  g.robot_speed = cfg->robot_speed;
  g.robot_length = cfg->robot_length;
  g.agent_safety_rad =
      ((cfg->robot_length > cfg->robot_width ? cfg->robot_length : cfg->robot_width) / 2) *
      cfg->safety_rad_mult;
  StepCfg& sc = h->sc;
  sc.repeat = cfg->repeat_actions;
  sc.frame_skip = cfg->frame_skip;
  sc.action_mode = cfg->action_mode;
  sc.clip = cfg->clip_action;
  sc.speed_measured = cfg->reward_speed_measured;
  sc.auto_reset = cfg->auto_reset;
  sc.max_steps = cfg->max_steps;
  sc.max_env_steps = cfg->max_env_steps;
  sc.max_spawn_attempts = cfg->max_spawn_attempts;
  sc.reward_scale = cfg->reward_scale;

  int rc = 0;
  auto fail = [&](const std::string& m) {
    g_create_err = m;
    if (h->map_buf) (void)hipFree(h->map_buf);
    if (h->st_buf) (void)hipFree(h->st_buf);
    delete h;
    return DT_E_HIP;
  };
  if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice failed");
  // map image: curve records | objects | spawn objects | curve_start (u16) | kind |
  // drivable
  const size_t lds = dt::map_lds_bytes(T, (int)drv.size(), C, NO, NS);
  if (lds > dt::kMaxMapLdsBytes) {
    g_create_err = "dt_create: map image over the LDS budget (" + std::to_string(lds) + " B)";
    delete h;
    return DT_E_ARG;
  }
  std::vector<uint16_t> cs(T + 1);
  for (int t = 0; t <= T; ++t) cs[t] = (uint16_t)map->curve_start[t];
  const size_t cb = rec.size() * 8,
               ob = (size_t)NO * DT_OBJ_STRIDE * 8, spb = (size_t)NS * 4 * 8,
               sb16 = ((size_t)(T + 1) * 2 + 15) & ~15ul, kb = ((size_t)T + 15) & ~15ul,
               db = (drv.size() * 2 + 15) & ~15ul;
  if (hipMalloc(&h->map_buf, cb + ob + spb + sb16 + kb + db) != hipSuccess)
    return fail("hipMalloc(map)");
  char* mb = (char*)h->map_buf;
  char* m_cs = mb + cb + ob + spb;
  if ((cb && hipMemcpy(mb, rec.data(), cb, hipMemcpyHostToDevice) != hipSuccess) ||
      (ob && hipMemcpy(mb + cb, map->objects, ob, hipMemcpyHostToDevice) != hipSuccess) ||
      (spb && hipMemcpy(mb + cb + ob, map->spawn_objects, spb, hipMemcpyHostToDevice) !=
                  hipSuccess) ||
      hipMemcpy(m_cs, cs.data(), (size_t)(T + 1) * 2, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(m_cs + sb16, map->kind, (size_t)T, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(m_cs + sb16 + kb, drv.data(), drv.size() * 2, hipMemcpyHostToDevice) !=
          hipSuccess)
    return fail("hipMemcpy(map)");
  h->map.width = map->width;
  h->map.height = map->height;
  h->map.n_tiles = T;
  h->map.n_drivable = (int)drv.size();
  h->map.n_curves = C;
  h->map.n_obj = NO;
  h->map.n_spawn_obj = NS;
  h->map.curves = (const double*)mb;
  h->map.obj = (const double*)(mb + cb);
  h->map.spawn_obj = (const double*)(mb + cb + ob);
  h->map.curve_start = (const uint16_t*)m_cs;
  h->map.kind = (const int8_t*)(m_cs + sb16);
  h->map.drivable = (const int16_t*)(m_cs + sb16 + kb);
  h->lds_bytes = lds;

  // state: x z angle seed (8 B) | step_count env_step episode (4 B) | err | stats |
  // spawn-ahead: pre (kSlots x kSlotRec x 8 B) | pre_key (kSlots x 8 B) | want tick (4 B)
  const size_t N = (size_t)n_envs, N8 = N * 8, N4 = (N * 4 + 255) & ~255ul;
  const size_t S = (size_t)dt::kSlots;
  const size_t spawn_at = 4 * N8 + 3 * N4 + 512;
  const size_t R = (size_t)dt::kSlotRec;
  const size_t total = spawn_at + (R + 1) * S * N8 + 2 * N4;
  if (hipMalloc(&h->st_buf, total) != hipSuccess) return fail("hipMalloc(state)");
  if (hipMemset(h->st_buf, 0, total) != hipSuccess) return fail("hipMemset(state)");
  char* sb = (char*)h->st_buf;
  h->st.x = (double*)sb;
  h->st.z = (double*)(sb + N8);
  h->st.angle = (double*)(sb + 2 * N8);
  h->st.seed = (uint64_t*)(sb + 3 * N8);
  h->st.step_count = (uint32_t*)(sb + 4 * N8);
  h->st.env_step = (uint32_t*)(sb + 4 * N8 + N4);
  h->st.episode = (uint32_t*)(sb + 4 * N8 + 2 * N4);
  h->st.err = (uint32_t*)(sb + 4 * N8 + 3 * N4);
  h->st.stats = (unsigned long long*)(sb + 4 * N8 + 3 * N4 + 256);
  h->st.pre = (double*)(sb + spawn_at);
  h->st.pre_key = (uint64_t*)(sb + spawn_at + R * S * N8);
  h->st.want = (uint32_t*)(sb + spawn_at + (R + 1) * S * N8);
  h->st.tick = (uint32_t*)(sb + spawn_at + (R + 1) * S * N8 + N4);
  *out = h;
  rc = dt_render_init(h, map);
  if (rc == DT_OK) rc = dt_seed(h, nullptr, seed, 0);
  if (rc) {
    std::string m = h->err;
    dt_destroy(h);
    *out = nullptr;
    g_create_err = m;
    return rc;
  }
  return DT_OK;
}

int dt_destroy(dt_handle* h) {
  if (!h) return DT_E_ARG;
  (void)hipSetDevice(h->device);
  dt_render_free(h);
  if (h->map_buf) (void)hipFree(h->map_buf);
  if (h->st_buf) (void)hipFree(h->st_buf);
  delete h;
  return DT_OK;
}

// Spawn-ahead after the seeds or episode counters changed: drop every slot of
// envs [e0, e1), want = counter + 1, then fill the window (synchronous).
static int refill_from_counters(dt_handle* h, int e0, int e1) {
  const size_t n = (size_t)h->n, m = (size_t)(e1 - e0);
  std::vector<uint32_t> ep(m), want(m);
  HIP_OR_FAIL(h, hipMemcpy(ep.data(), h->st.episode + e0, m * 4, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < m; ++i) want[i] = ep[i] + 1u;
  HIP_OR_FAIL(h, hipMemcpy(h->st.want + e0, want.data(), m * 4, hipMemcpyHostToDevice));
  for (size_t q = 0; q < (size_t)dt::kSlots; ++q)
    HIP_OR_FAIL(h, hipMemset(h->st.pre_key + q * n + e0, 0xFF, m * 8));
  hipLaunchKernelGGL(refill_kernel, dim3(refill_grid(h->n, kRefillEnvs)), dim3(kBlock), h->lds_bytes, (hipStream_t)0,
                     h->st, h->map, h->geo, h->n, h->sc.max_spawn_attempts, h->env_base);
  HIP_OR_FAIL(h, hipGetLastError());
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  return DT_OK;
}

int dt_seed(dt_handle* h, const uint64_t* seeds, uint64_t base, uint32_t env_id_base) {
  if (!h) return DT_E_ARG;
  h->env_base = env_id_base;
  HIP_OR_FAIL(h, hipSetDevice(h->device));
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  std::vector<uint64_t> s(h->n);
  for (int i = 0; i < h->n; ++i) s[i] = seeds ? seeds[i] : base;
  HIP_OR_FAIL(h, hipMemcpy(h->st.seed, s.data(), s.size() * 8, hipMemcpyHostToDevice));
  HIP_OR_FAIL(h, hipMemset(h->st.episode, 0, (size_t)h->n * 4));
  return refill_from_counters(h, 0, h->n);
}

int dt_seed_env(dt_handle* h, int32_t env, uint64_t seed) {
  if (!h || env < 0 || env >= h->n) return DT_E_ARG;
  HIP_OR_FAIL(h, hipSetDevice(h->device));
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  const uint32_t zero = 0;
  HIP_OR_FAIL(h, hipMemcpy(h->st.seed + env, &seed, 8, hipMemcpyHostToDevice));
  HIP_OR_FAIL(h, hipMemcpy(h->st.episode + env, &zero, 4, hipMemcpyHostToDevice));
  return refill_from_counters(h, env, env + 1);
}

int dt_reset(dt_handle* h, const uint8_t* mask, void* stream) {
  if (!h) return DT_E_ARG;
  DevGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(spawn_kernel, dim3(h->n), dim3(kSpawnThreads), h->lds_bytes, s, h->st,
                     h->map, h->geo, h->sc.max_spawn_attempts, h->env_base, mask);
  HIP_OR_FAIL(h, hipGetLastError());
  hipLaunchKernelGGL(refill_kernel, dim3(refill_grid(h->n, kRefillEnvs)), dim3(kBlock), h->lds_bytes, s, h->st, h->map,
                     h->geo, h->n, h->sc.max_spawn_attempts, h->env_base);
  HIP_OR_FAIL(h, hipGetLastError());
  return DT_OK;
}

int dt_step_masked(dt_handle* h, const uint8_t* mask, const float* actions, double* reward,
                   double* reward_mod, uint8_t* done, float* obs, double* lanepos, int32_t* tile,
                   void* stream) {
  if (!h) return DT_E_ARG;
  if (!actions || !reward || !reward_mod || !done) {
    h->err = "dt_step: actions, reward, reward_mod and done are required";
    return DT_E_ARG;
  }
  DevGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  // step blocks, then (auto-reset) refill blocks of kRefillEnvs envs: this
  // decision's resets use poses computed in earlier launches, and the refill of
  // the ones consumed last decision overlaps this decision's step
  const int gs = (h->n + kBlock - 1) / kBlock;
  const int grid = gs + (h->sc.auto_reset ? refill_grid(h->n, kRefillEnvs) : 0);
  hipLaunchKernelGGL(step_kernel, dim3(grid), dim3(kBlock), h->lds_bytes, s, h->st, h->map,
                     h->geo, h->sc, h->n, h->env_base, 1, (const float2*)actions, reward,
                     reward_mod, done, (float2*)obs, lanepos, tile, gs, h->sc.max_spawn_attempts,
                     mask);
  HIP_OR_FAIL(h, hipGetLastError());
  return DT_OK;
}

int dt_step(dt_handle* h, const float* actions, double* reward, double* reward_mod,
            uint8_t* done, float* obs, double* lanepos, int32_t* tile, void* stream) {
  return dt_step_masked(h, nullptr, actions, reward, reward_mod, done, obs, lanepos, tile, stream);
}

int dt_step_many(dt_handle* h, int32_t k, const float* actions, double* reward,
                 double* reward_mod, uint8_t* done, float* obs, double* pose, void* stream) {
  if (!h) return DT_E_ARG;
  if (k < 1 || !actions || !reward || !reward_mod || !done) {
    h->err = "dt_step_many: k >= 1, actions, reward, reward_mod and done are required";
    return DT_E_ARG;
  }
  // step_fan_kernel indexes one launch's outputs with 32-bit offsets (pose:
  // 3 doubles an env a decision, kFanMaxK decisions a launch)
  if ((int64_t)3 * kFanMaxK * h->n >= (int64_t(1) << 31)) {
    h->err = "dt_step_many: n too large for one handle (3 * 64 * n must stay below 2^31)";
    return DT_E_ARG;
  }
  DevGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  const int rb = h->sc.auto_reset ? refill_grid(h->n, kRefillEnvs) : 0;
  if (h->sc.repeat * h->sc.frame_skip <= kFanSteps && h->sc.frame_skip == 1) {
    // step_fan_kernel: 16 envs x 4 waves per workgroup
    const int gs = (h->n + kFanEnvs - 1) / kFanEnvs;
    const size_t off = (h->lds_bytes + 15) & ~(size_t)15;
    const size_t slots = (size_t)dt::kSlots * dt::kSlotRec * kFanEnvs * sizeof(double);
    // runs of more than kFanMaxK decisions: consecutive launches (the state,
    // counters and spawn window carry over exactly as between calls)
    const bool lean = h->sc.action_mode == DT_ACTION_WHEELS && h->sc.clip && !h->sc.speed_measured &&
                      h->sc.auto_reset && h->map.n_obj == 0;
    for (int d0 = 0; d0 < k; d0 += kFanMaxK) {
      const int kk = k - d0 < kFanMaxK ? k - d0 : kFanMaxK;
      const size_t o = (size_t)d0 * h->n;
      hipLaunchKernelGGL(lean ? step_fan_kernel<true> : step_fan_kernel<false>, dim3(gs + rb),
                         dim3(kFanBlock),
                         off + slots + (size_t)kk * kFanEnvs * sizeof(float2), s, h->st, h->map,
                         h->geo,
                         h->sc, h->n, h->env_base, kk, (const float2*)actions + o, reward + o,
                         reward_mod + o, done + o, obs ? (float2*)obs + o : (float2*)nullptr,
                         pose ? pose + 3 * o : (double*)nullptr, gs, h->sc.max_spawn_attempts,
                         (uint32_t)off);
      HIP_OR_FAIL(h, hipGetLastError());
    }
    return DT_OK;
  }
  // the generic path (more than three Simulator steps per decision, or
  // frame_skip > 1): step_kernel over the k decisions, or one launch per
  // decision when the poses are asked for
  const int gs = (h->n + kBlock - 1) / kBlock;
  for (int d0 = 0; d0 < k; d0 += pose ? 1 : k) {
    const int kk = pose ? 1 : k;
    const size_t o = (size_t)d0 * h->n;
    hipLaunchKernelGGL(step_kernel, dim3(gs + rb), dim3(kBlock), h->lds_bytes, s, h->st,
                       h->map, h->geo, h->sc, h->n, h->env_base, kk,
                       (const float2*)actions + o, reward + o, reward_mod + o, done + o,
                       obs ? (float2*)obs + o : (float2*)nullptr, (double*)nullptr,
                       (int32_t*)nullptr, gs, h->sc.max_spawn_attempts, (const uint8_t*)nullptr);
    HIP_OR_FAIL(h, hipGetLastError());
    if (pose)
      HIP_OR_FAIL(h, hipMemcpyAsync(pose + 3 * o, h->st.x, 3 * (size_t)h->n * sizeof(double),
                                    hipMemcpyDeviceToDevice, s));
  }
  return DT_OK;
}

int dt_lane_pos(dt_handle* h, double* lanepos, int32_t* tile, void* stream) {
  if (!h) return DT_E_ARG;
  DevGuard dg(h->device);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(lane_pos_kernel, dim3(grid_of(h->n)), dim3(dt::kWave), h->lds_bytes, s,
                     h->st, h->map, h->geo, h->n, lanepos, tile);
  HIP_OR_FAIL(h, hipGetLastError());
  return DT_OK;
}

int dt_get_state(dt_handle* h, double* x, double* z, double* angle, uint32_t* step_count,
                 uint32_t* env_step, uint32_t* episode) {
  if (!h) return DT_E_ARG;
  HIP_OR_FAIL(h, hipSetDevice(h->device));
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  const size_t N = (size_t)h->n;
  if (x) HIP_OR_FAIL(h, hipMemcpy(x, h->st.x, N * 8, hipMemcpyDeviceToHost));
  if (z) HIP_OR_FAIL(h, hipMemcpy(z, h->st.z, N * 8, hipMemcpyDeviceToHost));
  if (angle) HIP_OR_FAIL(h, hipMemcpy(angle, h->st.angle, N * 8, hipMemcpyDeviceToHost));
  if (step_count)
    HIP_OR_FAIL(h, hipMemcpy(step_count, h->st.step_count, N * 4, hipMemcpyDeviceToHost));
  if (env_step) HIP_OR_FAIL(h, hipMemcpy(env_step, h->st.env_step, N * 4, hipMemcpyDeviceToHost));
  if (episode) HIP_OR_FAIL(h, hipMemcpy(episode, h->st.episode, N * 4, hipMemcpyDeviceToHost));
  return DT_OK;
}

int dt_set_state(dt_handle* h, const double* x, const double* z, const double* angle,
                 const uint32_t* step_count, const uint32_t* env_step, const uint32_t* episode) {
  if (!h) return DT_E_ARG;
  HIP_OR_FAIL(h, hipSetDevice(h->device));
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  const size_t N = (size_t)h->n;
  if (x) HIP_OR_FAIL(h, hipMemcpy(h->st.x, x, N * 8, hipMemcpyHostToDevice));
  if (z) HIP_OR_FAIL(h, hipMemcpy(h->st.z, z, N * 8, hipMemcpyHostToDevice));
  if (angle) HIP_OR_FAIL(h, hipMemcpy(h->st.angle, angle, N * 8, hipMemcpyHostToDevice));
  if (step_count)
    HIP_OR_FAIL(h, hipMemcpy(h->st.step_count, step_count, N * 4, hipMemcpyHostToDevice));
  if (env_step) HIP_OR_FAIL(h, hipMemcpy(h->st.env_step, env_step, N * 4, hipMemcpyHostToDevice));
  if (episode) {
    HIP_OR_FAIL(h, hipMemcpy(h->st.episode, episode, N * 4, hipMemcpyHostToDevice));
    return refill_from_counters(h, 0, h->n);   // spawn-ahead keys follow the counters
  }
  return DT_OK;
}

int dt_stats(dt_handle* h, uint64_t out[4], int32_t reset) {
  if (!h || !out) return DT_E_ARG;
  HIP_OR_FAIL(h, hipSetDevice(h->device));
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  HIP_OR_FAIL(h, hipMemcpy(out, h->st.stats, 32, hipMemcpyDeviceToHost));
  if (reset) HIP_OR_FAIL(h, hipMemset(h->st.stats, 0, 32));
  return DT_OK;
}

int dt_check(dt_handle* h, uint32_t* flags) {
  if (!h) return DT_E_ARG;
  HIP_OR_FAIL(h, hipSetDevice(h->device));
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  uint32_t f = 0;
  HIP_OR_FAIL(h, hipMemcpy(&f, h->st.err, 4, hipMemcpyDeviceToHost));
  HIP_OR_FAIL(h, hipMemset(h->st.err, 0, 4));
  if (flags) *flags = f;
  if (f & dt::kErrSpawn) {
    h->err = "reset: could not find a valid starting pose after max_spawn_attempts";
    return DT_E_SPAWN;
  }
  return DT_OK;
}

}  // extern "C"

#ifdef DTSIM_STAMPS
// Diagnostic build only: cycles of one wave (64 envs, their current poses)
// per call of a step-math piece, in a loop on the LDS-staged map.
namespace {
__device__ unsigned long long g_micro[64];
__global__ __launch_bounds__(64) void micro_kernel(dt::State st, dt::MapDev md, dt::Geo g,
                                                   int iters, int which) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const MapLds M = dt::stage_map(md, lds);
  const int lane = threadIdx.x;
  double x = st.x[lane], z = st.z[lane], a = st.angle[lane];
  double s, c;
  sincos(a, &s, &c);
  double acc = 0.0;
  const double* cv = dt::closest_curve(M, g, x, z, c, s);
  if (!cv) cv = M.curves;
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if (which == 0) {
      double lp[4];
      const bool in = dt::lane_pos<false>(M, g, x, z, c, s, lp);
      acc = acc + (in ? lp[0] : 1.0);
    } else if (which == 1) {
      acc = acc + (dt::valid_pose(M, g, x, z, c, s, 1.0) ? 1.0 : 2.0);
    } else if (which == 2) {
      double s2, c2;
      sincos(x, &s2, &c2);
      acc = acc + s2 + c2;
    } else if (which == 3) {
      acc = acc + dt::bezier_closest(cv, x, z);
    } else if (which == 4) {
      const double* cc = dt::closest_curve(M, g, x, z, c, s);
      acc = acc + (cc ? cc[0] : 1.0);
    } else if (which == 5) {
      acc = acc + (double)dt::tile_of(M, g, x, z);
    } else if (which == 6) {
      double lp[4];
      dt::lane_pose_at<false>(g, cv, 0.3, x, z, c, s, lp);
      acc = acc + lp[0];
    } else if (which == 7) {
      acc = acc + (dt::drivable(M, g, x, z) ? 1.0 : 2.0);
    } else if (which == 8) {
      double lp[4];
      const bool in = dt::lane_pos_lean<false>(M, g, x, z, c, s, lp);
      acc = acc + (in ? lp[0] : 1.0);
    } else if (which == 9) {
      acc = acc + (dt::valid_pose_lean(M, g, x, z, c, s, 1.0) ? 1.0 : 2.0);
    } else if (which == 10) {
      bool nr = false;
      acc = acc + dt::bezier_closest_fast(cv, x, z, nr) + (nr ? 1.0 : 0.0);
    } else if (which == 11) {
      bool nr = false;
      acc = acc + (double)dt::tile_of_fast(M, g, x, z, nr) + (nr ? 1.0 : 0.0);
    } else if (which == 12) {
      bool nr = false;
      const double* cc = dt::closest_curve_fast(M, g, x, z, c, s, nr);
      acc = acc + (cc ? cc[0] : 1.0) + (nr ? 1.0 : 0.0);
    } else if (which == 13) {
      double lp[4];
      const bool in = dt::lane_pos_q(M, g, lane & 3, x, z, c, s, lp);
      acc = acc + (in ? lp[0] + lp[3] : 1.0);
    } else if (which == 14) {
      bool nr = false;
      acc = acc + dt::bezier_closest_q(cv, lane & 3, x, z, nr) + (nr ? 1.0 : 0.0);
    } else if (which == 15) {
      double lp[4];
      dt::lane_pose_at<true>(g, cv, 0.3 + acc * 1e-300, x, z, c, s, lp);
      acc = acc + lp[0] + lp[3];
    } else if (which == 16) {
      acc = acc + (dt::valid_pose_q(M, g, lane & 3, x, z, c, s, 1.0) ? 1.0 : 2.0);
    } else if (which == 18) {
      acc = acc + sqrt(x * x + 1.0);
    } else if (which == 19) {
      acc = acc + 1.0 / (x + 2.0);
    } else if (which == 20) {
      double v = x;
#pragma unroll
      for (int j = 0; j < 7; ++j) v = v * 1.0000001 + 1e-3;
      acc = acc + v;
    } else if (which == 21) {
      const double tm = 0.3 + acc * 1e-300;
      const double u = 1.0 - tm;
      const double a0 = 3.0 * (u * u), a1 = 6.0 * u * tm, a2 = 3.0 * (tm * tm);
      double tx = a0 * cv[8], tz = a0 * cv[9];
      tx = tx + a1 * cv[10];
      tz = tz + a1 * cv[11];
      tx = tx + a2 * cv[12];
      tz = tz + a2 * cv[13];
      const double nn = sqrt(tx * tx + tz * tz);
      acc = acc + tx / nn + tz / nn;
    } else if (which == 22) {
      double bx, bz;
      dt::bez_xz(cv, 0.3 + acc * 1e-300, bx, bz);
      acc = acc + bx + bz;
    } else if (which == 23) {
      acc = acc + acos(x * 1e-3);
    } else if (which == 17) {
      double lp[4];
      dt::lane_pose_at<false>(g, cv, 0.3 + acc * 1e-300, x, z, c, s, lp);
      acc = acc + lp[0] + lp[2];
    }
    x = x + acc * 1e-300;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  st.x[lane] = x;  // keep the loop live (the pose moves by < 1 ulp)
  if (lane == 0) g_micro[0] = t1 - t0;
}
}  // namespace

extern "C" int dt_diag_micro(dt_handle* h, int iters, int which, unsigned long long* out) {
  HIP_OR_FAIL(h, hipSetDevice(h->device));
  hipLaunchKernelGGL(micro_kernel, dim3(1), dim3(64), h->lds_bytes, 0, h->st, h->map, h->geo,
                     iters, which);
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_micro), 8) == hipSuccess ? 0 : -1;
}
#endif
