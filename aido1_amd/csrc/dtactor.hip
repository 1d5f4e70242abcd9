// Per-sample (batch-of-one, train-mode) LeakyReLU + BatchNorm2d over NHWC
// activations — see include/dtactor.h.  One workgroup per sample: the sample's
// [hw, c] slab is read three times (sum, squared deviations, normalise) — the
// first read from HBM, the next two mostly from L2 / MALL — and written once.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/dtactor.h"

namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;  // channels per thread per pixel (16 B of bf16)

__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);  // round to nearest even
  return u >> 16;
}

template <typename T>
struct Io;

template <>
struct Io<uint16_t> {  // bf16
  static __device__ __forceinline__ void load(const uint16_t* p, float* f) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f[2 * k] = bf16_to_f32(w[k] & 0xFFFFu);
      f[2 * k + 1] = bf16_to_f32(w[k] >> 16);
    }
  }
  static __device__ __forceinline__ void store(uint16_t* p, const float* f) {
    uint4 v;
    v.x = f32_to_bf16(f[0]) | (f32_to_bf16(f[1]) << 16);
    v.y = f32_to_bf16(f[2]) | (f32_to_bf16(f[3]) << 16);
    v.z = f32_to_bf16(f[4]) | (f32_to_bf16(f[5]) << 16);
    v.w = f32_to_bf16(f[6]) | (f32_to_bf16(f[7]) << 16);
    *reinterpret_cast<uint4*>(p) = v;
  }
};

template <>
struct Io<__half> {
  static __device__ __forceinline__ void load(const __half* p, float* f) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    const __half2* h = reinterpret_cast<const __half2*>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float2 t = __half22float2(h[k]);
      f[2 * k] = t.x;
      f[2 * k + 1] = t.y;
    }
  }
  static __device__ __forceinline__ void store(__half* p, const float* f) {
    uint4 v;
    __half2* h = reinterpret_cast<__half2*>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) h[k] = __floats2half2_rn(f[2 * k], f[2 * k + 1]);
    *reinterpret_cast<uint4*>(p) = v;
  }
};

template <>
struct Io<float> {
  static __device__ __forceinline__ void load(const float* p, float* f) {
    const float4 a = reinterpret_cast<const float4*>(p)[0];
    const float4 b = reinterpret_cast<const float4*>(p)[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
    f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float* f) {
    reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
  }
};

__device__ __forceinline__ float lrelu(float v, float slope) { return v > 0.0f ? v : v * slope; }

// Sum over the threads that own the same channel group (t % groups) of
// acc[kVec] (idle threads hold zeros); returns, in s_out[c], the per-channel
// totals.
__device__ void reduce_channels(const float* acc, float (*s_part)[kVec], float* s_out, int groups,
                                int c) {
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < kVec; ++k) s_part[t][k] = acc[k];
  __syncthreads();
  if (t < c) {
    const int g = t / kVec, k = t % kVec;
    float s = 0.0f;
    for (int u = g; u < kThreads; u += groups) s += s_part[u][k];
    s_out[t] = s;
  }
  __syncthreads();
}

template <typename T>
__global__ void __launch_bounds__(kThreads)
sample_norm_kernel(const T* x, T* y, int hw, int c,  // y may alias x
                   const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                   float slope) {
  __shared__ float s_part[kThreads][kVec];
  __shared__ float s_mean[64], s_scale[64], s_shift[64];
  const int groups = c / kVec;          // threads per pixel
  const int per_iter = kThreads / groups;
  const int t = threadIdx.x;
  const int g = t % groups;
  const size_t base = (size_t)blockIdx.x * hw * c;
  const T* xs = x + base;
  T* ys = y + base;
  const int active = per_iter * groups;  // threads beyond this idle (c not dividing 256)
  float v[kVec], acc[kVec];

#pragma unroll
  for (int k = 0; k < kVec; ++k) acc[k] = 0.0f;
  if (t < active)
    for (int p = t / groups; p < hw; p += per_iter) {
      Io<T>::load(xs + (size_t)p * c + g * kVec, v);
#pragma unroll
      for (int k = 0; k < kVec; ++k) acc[k] += lrelu(v[k], slope);
    }
  reduce_channels(acc, s_part, s_mean, groups, c);
  if (t < c) s_mean[t] = s_mean[t] / (float)hw;
  __syncthreads();

  float mu[kVec];
#pragma unroll
  for (int k = 0; k < kVec; ++k) {
    mu[k] = s_mean[g * kVec + k];
    acc[k] = 0.0f;
  }
  if (t < active)
    for (int p = t / groups; p < hw; p += per_iter) {
      Io<T>::load(xs + (size_t)p * c + g * kVec, v);
#pragma unroll
      for (int k = 0; k < kVec; ++k) {
        const float d = lrelu(v[k], slope) - mu[k];
        acc[k] += d * d;
      }
    }
  reduce_channels(acc, s_part, s_scale, groups, c);
  if (t < c) {
    const float var = s_scale[t] / (float)hw;
    const float sc = gamma[t] / sqrtf(var + eps);
    s_scale[t] = sc;
    s_shift[t] = beta[t] - s_mean[t] * sc;
  }
  __syncthreads();

  float sc[kVec], sh[kVec];
#pragma unroll
  for (int k = 0; k < kVec; ++k) {
    sc[k] = s_scale[g * kVec + k];
    sh[k] = s_shift[g * kVec + k];
  }
  if (t < active)
    for (int p = t / groups; p < hw; p += per_iter) {
      Io<T>::load(xs + (size_t)p * c + g * kVec, v);
#pragma unroll
      for (int k = 0; k < kVec; ++k) v[k] = lrelu(v[k], slope) * sc[k] + sh[k];
      Io<T>::store(ys + (size_t)p * c + g * kVec, v);
    }
}

}  // namespace

extern "C" int dt_sample_norm(const void* x, void* y, int32_t n, int32_t hw, int32_t c,
                              const float* gamma, const float* beta, float eps, float slope,
                              int32_t dtype, void* stream) {
  if (!x || !y || !gamma || !beta || n < 0 || hw <= 0 || c <= 0 || c % kVec || c > 64 ||
      dtype < 0 || dtype > 2)
    return DT_E_ARG;
  if (n == 0) return DT_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == 0)
    sample_norm_kernel<uint16_t><<<n, kThreads, 0, s>>>((const uint16_t*)x, (uint16_t*)y, hw, c,
                                                        gamma, beta, eps, slope);
  else if (dtype == 1)
    sample_norm_kernel<float><<<n, kThreads, 0, s>>>((const float*)x, (float*)y, hw, c, gamma,
                                                     beta, eps, slope);
  else
    sample_norm_kernel<__half><<<n, kThreads, 0, s>>>((const __half*)x, (__half*)y, hw, c, gamma,
                                                      beta, eps, slope);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// ---- dt_explore / dt_explore_done: the rollout's per-decision action choice --------------
// One lane per explorer; every operation is the one (and in the order) the
// torch restatement in aido1_amd/explore.py + rollout.CycleEpsilon performs,
// so the two agree bit for bit given the same normals and uniforms
// (-ffp-contract=off: no fused multiply-adds).
namespace {

__global__ void __launch_bounds__(256)
explore_kernel(int n, const float* __restrict__ actor_out, const double* __restrict__ normals,
               const double* __restrict__ coin, const float* __restrict__ uni,
               double* __restrict__ ou_x, double* __restrict__ ou_steps,
               const int64_t* __restrict__ episode, const double* __restrict__ cycle,
               const double* __restrict__ max_step, const int64_t* __restrict__ explorer_id,
               DtExploreParams p, float* __restrict__ actions) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // epsilon: CycleEpsilon (explorers.py:92-111 over utils/util.py:36-40)
  const double ep = (double)episode[i], cl = cycle[i];
  const double rel = 1.0 - ep / max_step[i];
  const double cosv = 0.5 * (cos(p.pi * fmod(ep, cl) / cl) + 1.0);
  double eps = cosv * p.eps_span * rel + p.eps_final;
  eps = eps < p.eps_final ? p.eps_final : eps;
  eps = eps > p.eps_initial ? p.eps_initial : eps;
  // OU sample (utils/random_process.py:42-47): sigma annealed, then the step
  double sigma = p.ou_m * ou_steps[i] + p.ou_c;
  sigma = sigma < p.ou_sigma_min ? p.ou_sigma_min : sigma;
  const double sd = sigma * p.ou_sqrt_dt;
  const double2 x = reinterpret_cast<const double2*>(ou_x)[i];
  const double2 z = reinterpret_cast<const double2*>(normals)[i];
  const double x0 = x.x + p.ou_theta * (p.ou_mu - x.x) * p.ou_dt + sd * z.x;
  const double x1 = x.y + p.ou_theta * (p.ou_mu - x.y) * p.ou_dt + sd * z.y;
  reinterpret_cast<double2*>(ou_x)[i] = make_double2(x0, x1);
  ou_steps[i] = ou_steps[i] + 1.0;
  // DDPG.act (models/ddpg/model.py:74-102): the sample is float32; epsilon is
  // an np.float64, so noise = epsilon * sample is float64 (numpy 2, NEP 50),
  // doubled for a tanh head, and `action += noise` adds in float64 and rounds
  // once to the float32 action (tests/golden/explorer.json pins this)
  const double nz0 = eps * (double)(float)x0, nz1 = eps * (double)(float)x1;
  const float2 o = reinterpret_cast<const float2*>(actor_out)[i];
  float a0, a1;
  if (p.head == 0) {          // tanh: noise doubled, clipped to [-1, 1]
    a0 = fminf(fmaxf((float)((double)o.x + 2.0 * nz0), -1.0f), 1.0f);
    a1 = fminf(fmaxf((float)((double)o.y + 2.0 * nz1), -1.0f), 1.0f);
  } else if (p.head == 1) {   // sigmoid: clipped to [0, 1]
    a0 = fminf(fmaxf((float)((double)o.x + nz0), 0.0f), 1.0f);
    a1 = fminf(fmaxf((float)((double)o.y + nz1), 0.0f), 1.0f);
  } else {
    a0 = (float)((double)o.x + nz0);
    a1 = (float)((double)o.y + nz1);
  }
  // every_second_random (explorers.py:178-194): even ids act uniformly at
  // random when random.uniform(0, 1) < epsilon_ratio * epsilon (float64)
  if (coin && (explorer_id[i] & 1) == 0 && coin[i] < p.eps_ratio * eps) {
    const float2 u = reinterpret_cast<const float2*>(uni)[i];
    a0 = u.x;
    a1 = u.y;
  }
  reinterpret_cast<float2*>(actions)[i] = make_float2(a0, a1);
}

__global__ void __launch_bounds__(256)
explore_done_kernel(int n, const uint8_t* __restrict__ done, double* __restrict__ ou_x,
                    int64_t* __restrict__ episode, float* __restrict__ actions, int tanh_map) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (tanh_map) {   // the wrapper's in-place a / 2 + 0.5 (env_wrappers.py:214-216)
    float2 a = reinterpret_cast<float2*>(actions)[i];
    a.x = a.x / 2.0f + 0.5f;
    a.y = a.y / 2.0f + 0.5f;
    reinterpret_cast<float2*>(actions)[i] = a;
  }
  if (done[i]) {    // explorers.py:170 reset_states + the episode count
    reinterpret_cast<double2*>(ou_x)[i] = make_double2(0.0, 0.0);
    episode[i] = episode[i] + 1;
  }
}

}  // namespace

extern "C" int dt_explore(int32_t n, const float* actor_out, const double* normals,
                          const double* coin, const float* uni, double* ou_x, double* ou_steps,
                          const int64_t* episode, const double* cycle, const double* max_step,
                          const int64_t* explorer_id, const DtExploreParams* params,
                          float* actions, void* stream) {
  if (n < 0 || !params || (params->head < 0 || params->head > 2)) return DT_E_ARG;
  if (n == 0) return DT_OK;
  if (!actor_out || !normals || !ou_x || !ou_steps || !episode || !cycle || !max_step ||
      !actions || (coin && (!uni || !explorer_id)))
    return DT_E_ARG;
  explore_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(
      n, actor_out, normals, coin, uni, ou_x, ou_steps, episode, cycle, max_step, explorer_id,
      *params, actions);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

extern "C" int dt_explore_done(int32_t n, const uint8_t* done, double* ou_x, int64_t* episode,
                               float* actions, int32_t tanh_map, void* stream) {
  if (n < 0 || (n > 0 && (!done || !ou_x || !episode || (tanh_map && !actions))))
    return DT_E_ARG;
  if (n == 0) return DT_OK;
  explore_done_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(n, done, ou_x, episode,
                                                                        actions, tanh_map);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// ---- dt_episode_account: the explorers' episode sums and finished-episode ring -------------
// One lane per env walks its k decisions in order (the f64 sums are the
// explorer's `episode_metrics[...] += ...` in the same order); a finished
// episode takes a ring slot from one device-wide counter.  Finished episodes
// are ~10 % of the envs a decision, so the per-lane atomic is not contended
// enough to aggregate.
namespace {

__global__ void __launch_bounds__(256)
episode_account_kernel(int n, int k, const double* __restrict__ reward,
                       const double* __restrict__ reward_mod, const uint8_t* __restrict__ done,
                       DtEpisodeState st) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double r = st.reward[i], m = st.reward_modified[i];
  int64_t tick = st.tick[i], ep = st.episode[i];
  int32_t len = st.decisions[i];
  for (int d = 0; d < k; ++d) {
    const size_t o = (size_t)d * n + i;
    r = r + reward[o];
    m = m + reward_mod[o];
    tick += 1;
    len += 1;
    if (done[o]) {
      const unsigned long long slot =
          atomicAdd(reinterpret_cast<unsigned long long*>(st.count), 1ull);
      DtEpisodeRecord rec;
      rec.reward = r;
      rec.reward_modified = m;
      rec.tick = tick;
      rec.episode = ep;
      rec.env = i;
      rec.decisions = len;
      st.ring[slot % (unsigned long long)st.capacity] = rec;
      r = 0.0;
      m = 0.0;
      len = 0;
      ep += 1;
    }
  }
  st.reward[i] = r;
  st.reward_modified[i] = m;
  st.tick[i] = tick;
  st.episode[i] = ep;
  st.decisions[i] = len;
}

}  // namespace

extern "C" int dt_episode_account(int32_t n, int32_t k, const double* reward,
                                  const double* reward_mod, const uint8_t* done,
                                  const DtEpisodeState* state, void* stream) {
  if (n < 0 || k < 1 || !state) return DT_E_ARG;
  if (n == 0) return DT_OK;
  if (!reward || !reward_mod || !done || !state->reward || !state->reward_modified ||
      !state->tick || !state->episode || !state->decisions || !state->count || !state->ring ||
      state->capacity < 1)
    return DT_E_ARG;
  episode_account_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(
      n, k, reward, reward_mod, done, *state);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// ---- the actor head after the first linear: LeakyReLU -> lin2 -> output ---------------
// (config.json actor output branch: linear 512 -> 2, tanh; ddpg.py:58-62).  One
// wave a sample: each lane takes 8 of the K inputs (16-B loads), LeakyReLU in
// f32 rounded to fp16 (F.leaky_relu on the fp16 tensor), the two dot products
// in f32, a wave reduction, then + bias rounded to fp16 (the fp16 GEMM's
// output), the head in f32.  Rows [0, n0) use set a, [n0, n) set b.
namespace {
constexpr int kHeadWaves = 4;

__global__ void __launch_bounds__(64 * kHeadWaves)
actor_head_kernel(int n, int n0, int k, const __half* __restrict__ h, int ld,
                  const __half* __restrict__ w2a, const __half* __restrict__ b2a,
                  const __half* __restrict__ w2b, const __half* __restrict__ b2b, int head,
                  float slope, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kHeadWaves + (threadIdx.x >> 6);
  if (row >= n) return;   // wave-uniform
  const bool first = row < n0;
  const __half* w2 = first ? w2a : w2b;
  const __half* b2 = first ? b2a : b2b;
  float acc0 = 0.0f, acc1 = 0.0f;
  for (int c = 8 * lane; c < k; c += 8 * 64) {
    float x[8], u[8], v[8];
    Io<__half>::load(h + (size_t)row * ld + c, x);
    Io<__half>::load(w2 + c, u);
    Io<__half>::load(w2 + k + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = __half2float(__float2half(x[j] > 0.0f ? x[j] : x[j] * slope));
      acc0 += a * u[j];
      acc1 += a * v[j];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    acc0 += __shfl_xor(acc0, o);
    acc1 += __shfl_xor(acc1, o);
  }
  if (lane == 0) {
    float y[2] = {__half2float(__float2half(acc0 + __half2float(b2[0]))),
                  __half2float(__float2half(acc1 + __half2float(b2[1])))};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (head == 1) y[j] = tanhf(y[j]);
      else if (head == 2) y[j] = 1.0f / (1.0f + expf(-y[j]));
    }
    *reinterpret_cast<float2*>(out + 2 * (size_t)row) = make_float2(y[0], y[1]);
  }
}
}  // namespace

extern "C" int dt_actor_head(int32_t n, int32_t n0, int32_t k, const void* h, int32_t ld,
                             const void* w2a, const void* b2a, const void* w2b, const void* b2b,
                             int32_t head, float slope, float* out, void* stream) {
  if (n < 0 || n0 < 0 || n0 > n || k < 8 || (k & 7) != 0 || ld < k || (ld & 7) != 0 || !h ||
      !w2a || !b2a || !out || head < 0 || head > 2 || (n0 < n && (!w2b || !b2b)))
    return DT_E_ARG;
  if (((reinterpret_cast<uintptr_t>(h) | reinterpret_cast<uintptr_t>(w2a) |
        (w2b ? reinterpret_cast<uintptr_t>(w2b) : 0)) & 15) ||
      (reinterpret_cast<uintptr_t>(out) & 7))
    return DT_E_ARG;
  if (n == 0) return DT_OK;
  hipLaunchKernelGGL(actor_head_kernel, dim3((n + kHeadWaves - 1) / kHeadWaves),
                     dim3(64 * kHeadWaves), 0, (hipStream_t)stream, n, n0, k,
                     (const __half*)h, ld, (const __half*)w2a, (const __half*)b2a,
                     (const __half*)w2b, (const __half*)b2b, head, slope, out);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// ---- the acting copies' refresh in one launch (dt_refresh_copy) --------------------
namespace {

constexpr int kCopyThreads = 256;

// entry e of the table, element i: dst[i] = cast(src[map ? map[i] : i]), 0 where
// map[i] < 0; blockIdx.y = entry, x-blocks stride over its elements.  dst_dtype
// 0 f32, 1 fp16, 2 the x3 pair (include/dtactor.h dt_conv1x_split): fp16 hi =
// fp16(v) at dst[i], lo = fp16((v - hi) * 2^11) at dst[count + i]
__global__ void __launch_bounds__(kCopyThreads)
refresh_copy_kernel(int32_t n, const DtCopyEntry* __restrict__ table) {
  const DtCopyEntry t = table[blockIdx.y];
  const float* src = static_cast<const float*>(t.src);
  for (int64_t i = (int64_t)blockIdx.x * kCopyThreads + threadIdx.x; i < t.count;
       i += (int64_t)gridDim.x * kCopyThreads) {
    float v;
    if (t.map) {
      const int64_t j = t.map[i];
      v = j >= 0 ? src[j] : 0.0f;
    } else {
      v = src[i];
    }
    if (t.dst_dtype == 1) {
      static_cast<__half*>(t.dst)[i] = __float2half(v);   // round to nearest, as .half()
    } else if (t.dst_dtype == 2) {
      const __half h = __float2half(v);
      static_cast<__half*>(t.dst)[i] = h;
      static_cast<__half*>(t.dst)[t.count + i] = __float2half((v - __half2float(h)) * 2048.0f);
    } else {
      static_cast<float*>(t.dst)[i] = v;
    }
  }
}

}  // namespace

extern "C" int dt_refresh_copy(int32_t n, const DtCopyEntry* table, int64_t max_count,
                               void* stream) {
  if (n < 0 || n > 65535 || (n > 0 && !table) || max_count < 0) return DT_E_ARG;
  if (n == 0 || max_count == 0) return DT_OK;
  int64_t gx = (max_count + kCopyThreads * 4 - 1) / (kCopyThreads * 4);
  gx = gx < 1 ? 1 : (gx > 2048 ? 2048 : gx);
  hipLaunchKernelGGL(refresh_copy_kernel, dim3((unsigned)gx, (unsigned)n), dim3(kCopyThreads), 0,
                     (hipStream_t)stream, n, table);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}
