// The fused training-mode tail of a conv block (bias + LeakyReLU + BatchNorm
// with batch statistics) for the DDPG update: see include/dttrain.h.
//
// Each kernel is one grid-stride pass over the NHWC f32 activation, one
// float4 (4 channels of one pixel) per thread and step: 1024 threads (16
// waves, one workgroup a CU) cover 128 pixels a step and a thread always holds
// the same 4 channels (tid & 7).  At most 256 workgroups, so the last one
// merges at most 256 partials a channel: 32 threads a channel, 8 each.
// The per-channel reductions are per-thread partials -> the workgroup's (via
// LDS) -> global partials; the workgroup that finishes last (a counter in the
// scratch, reset by that workgroup) merges them and writes the channel
// results, so no second launch and no host round trip is needed.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/dttrain.h"
#include "dtsync.h"

namespace {

constexpr int C = 32;          // channels (every conv of config.json's actor / critic)
constexpr int kT = 1024;       // threads a workgroup
constexpr int kSlots = kT / 8; // pixels a workgroup step covers
constexpr int kMaxGrid = 256;
constexpr int kFin = kT / C;   // threads a channel in the final merge
constexpr int kCounters = 16;  // floats at the end of the scratch holding the counters

int grid_of(int64_t m) {
  const int64_t q = m * 8;                           // float4 items
  int64_t g = (q + 2 * kT - 1) / (2 * kT);           // >= 2 items a thread
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return (int)g;
}

__device__ __forceinline__ float4 ld4(const float* p, int64_t q) {
  return reinterpret_cast<const float4*>(p)[q];
}
__device__ __forceinline__ void st4(float* p, int64_t q, float4 v) {
  reinterpret_cast<float4*>(p)[q] = v;
}

// a = leaky_relu(z + bias): the block's activation, recomputed from the
// convolution output wherever it is read (never stored), the same two
// roundings each time
__device__ __forceinline__ void leaky4(float4 v, float4 b, float slope, float (&x)[4]) {
  x[0] = v.x + b.x;
  x[1] = v.y + b.y;
  x[2] = v.z + b.z;
  x[3] = v.w + b.w;
#pragma unroll
  for (int k = 0; k < 4; ++k) x[k] = x[k] > 0.0f ? x[k] : x[k] * slope;
}

// ---- forward 1: a = leaky(z + bias) and the batch statistics of a --------------------
__global__ void __launch_bounds__(kT)
bn_stats_kernel(int64_t m, const float* __restrict__ z, const float* __restrict__ bias, float slope,
                float eps, float momentum, float* __restrict__ running_mean,
                float* __restrict__ running_var, int64_t* __restrict__ nbt, int updates,
                float* __restrict__ a, float* __restrict__ mean_invstd,
                float* __restrict__ work, int32_t* __restrict__ guard) {
  __shared__ float red[kSlots][C][3];
  const int tid = threadIdx.x, cg = tid & 7, slot = tid >> 3;
  const float4 b = ld4(bias, cg);
  float n = 0.0f, mean[4] = {0, 0, 0, 0}, m2[4] = {0, 0, 0, 0};
  const int64_t items = m * 8, stride = (int64_t)gridDim.x * kT;
  for (int64_t q = (int64_t)blockIdx.x * kT + tid; q < items; q += stride) {
    float x[4];
    leaky4(ld4(z, q), b, slope, x);
    if (a) st4(a, q, make_float4(x[0], x[1], x[2], x[3]));
    n += 1.0f;
    const float inv = 1.0f / n;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = x[k] - mean[k];
      mean[k] += d * inv;
      m2[k] += d * (x[k] - mean[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    red[slot][4 * cg + k][0] = n;
    red[slot][4 * cg + k][1] = mean[k];
    red[slot][4 * cg + k][2] = m2[k];
  }
  __syncthreads();
  float* part = work;   // [grid][C][3]
  // 128 slots a channel: kFin threads a channel merge 4 each, then one thread
  __shared__ float red2[kFin][C][3];
  {
    const int ch = tid & (C - 1), j = tid / C;
    float cn = 0.0f, cm = 0.0f, cm2 = 0.0f;
    for (int s = j; s < kSlots; s += kFin) chan(cn, cm, cm2, red[s][ch][0], red[s][ch][1], red[s][ch][2]);
    red2[j][ch][0] = cn;
    red2[j][ch][1] = cm;
    red2[j][ch][2] = cm2;
  }
  __syncthreads();
  if (tid < C) {
    float cn = 0.0f, cm = 0.0f, cm2 = 0.0f;
    for (int s = 0; s < kFin; ++s) chan(cn, cm, cm2, red2[s][tid][0], red2[s][tid][1], red2[s][tid][2]);
    float* p = part + ((size_t)blockIdx.x * C + tid) * 3;
    st_wt(p, cn);
    st_wt(p + 1, cm);
    st_wt(p + 2, cm2);
  }
  unsigned int* counters = reinterpret_cast<unsigned int*>(work + (size_t)kMaxGrid * C * 3);
  if (!last_arrival(&counters[0])) return;
  acquire_partials();
  // the last workgroup: kFin threads a channel over the partials, then one
  {
    const int ch = tid & (C - 1), j = tid / C;
    float cn = 0.0f, cm = 0.0f, cm2 = 0.0f;
    constexpr int kPer = kMaxGrid / kFin;   // 8: all loads issued before the merges
    float pn[kPer], pm[kPer], pq[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int g = j + k * kFin;
      const float* p = part + ((size_t)(g < (int)gridDim.x ? g : 0) * C + ch) * 3;
      pn[k] = g < (int)gridDim.x ? ld_wt(p) : 0.0f;
      pm[k] = ld_wt(p + 1);
      pq[k] = ld_wt(p + 2);
    }
    // counts back to zero: a partial the next launch fails to deliver (or
    // that is read stale) then shows as a missing count below
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int g = j + k * kFin;
      if (g < (int)gridDim.x) st_wt(part + ((size_t)g * C + ch) * 3, 0.0f);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) chan(cn, cm, cm2, pn[k], pm[k], pq[k]);
    red2[j][ch][0] = cn;
    red2[j][ch][1] = cm;
    red2[j][ch][2] = cm2;
  }
  __syncthreads();
  if (tid < C) {
    float cn = 0.0f, cm = 0.0f, cm2 = 0.0f;
    for (int s = 0; s < kFin; ++s) chan(cn, cm, cm2, red2[s][tid][0], red2[s][tid][1], red2[s][tid][2]);
    const float var = cm2 / cn;                       // biased: the normalisation
    const float invstd = 1.0f / sqrtf(var + eps);
    mean_invstd[tid] = cm;
    mean_invstd[C + tid] = invstd;
    // the merged count is every pixel exactly (float integers up to 2^24)
    const bool lost = m < (int64_t(1) << 24) ? cn != (float)m
                                              : fabsf(cn - (float)m) > 1e-6f * (float)m;
    guard_raise(guard, DT_GUARD_BN_COUNT, lost);
    guard_raise(guard, DT_GUARD_BN_FWD, !finitef(cm) || !finitef(invstd));
    const float unbiased = cn > 1.0f ? cm2 / (cn - 1.0f) : var;
    // one running-statistics update per reference forward over this batch
    // (the same batch statistics each time: a shared trunk, trainer.py)
    float rm = running_mean[tid], rv = running_var[tid];
    for (int u = 0; u < updates; ++u) {
      rm = (1.0f - momentum) * rm + momentum * cm;
      rv = (1.0f - momentum) * rv + momentum * unbiased;
    }
    running_mean[tid] = rm;
    running_var[tid] = rv;
    if (tid == 0 && nbt) nbt[0] += updates;
  }
}

// ---- forward 2: y = (a - mean) * invstd * gamma + beta -------------------------------
__global__ void __launch_bounds__(kT)
bn_apply_kernel(int64_t m, const float* __restrict__ z, const float* __restrict__ bias, float slope,
                const float* __restrict__ mean_invstd, const float* __restrict__ gamma,
                const float* __restrict__ beta, float* __restrict__ y) {
  const int cg = threadIdx.x & 7;
  const float4 b = ld4(bias, cg);
  const float4 mu = ld4(mean_invstd, cg), is = ld4(mean_invstd + C, cg);
  const float4 g = ld4(gamma, cg), bt = ld4(beta, cg);
  const float4 sc = make_float4(is.x * g.x, is.y * g.y, is.z * g.z, is.w * g.w);
  const int64_t items = m * 8, stride = (int64_t)gridDim.x * kT;
  for (int64_t q = (int64_t)blockIdx.x * kT + threadIdx.x; q < items; q += stride) {
    float v[4];
    leaky4(ld4(z, q), b, slope, v);
    st4(y, q, make_float4((v[0] - mu.x) * sc.x + bt.x, (v[1] - mu.y) * sc.y + bt.y,
                          (v[2] - mu.z) * sc.z + bt.z, (v[3] - mu.w) * sc.w + bt.w));
  }
}

// sums of kN per-channel values over the workgroup's threads -> part[block][C][kN]
template <int kN>
__device__ void block_sums(float (&acc)[kN][4], float* __restrict__ part) {
  __shared__ float red[kSlots][C][kN];
  __shared__ float red2[kFin][C][kN];
  const int tid = threadIdx.x, cg = tid & 7, slot = tid >> 3;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < kN; ++j) red[slot][4 * cg + k][j] = acc[j][k];
  __syncthreads();
  {
    const int ch = tid & (C - 1), q = tid / C;
#pragma unroll
    for (int j = 0; j < kN; ++j) {
      float t = 0.0f;
      for (int sl = q; sl < kSlots; sl += kFin) t += red[sl][ch][j];
      red2[q][ch][j] = t;
    }
  }
  __syncthreads();
  if (tid < C) {
#pragma unroll
    for (int j = 0; j < kN; ++j) {
      float t = 0.0f;
      for (int q = 0; q < kFin; ++q) t += red2[q][tid][j];
      st_wt(part + ((size_t)blockIdx.x * C + tid) * kN + j, t);
    }
  }
}

// the last workgroup: per-channel totals of the kN partial columns -> out[j][C]
template <int kN>
__device__ void final_sums(const float* __restrict__ part, float* const (&out)[kN],
                           int32_t* __restrict__ guard) {
  __shared__ float red[kFin][C][kN];
  const int tid = threadIdx.x, ch = tid & (C - 1), q = tid / C;
  float s[kN];
#pragma unroll
  for (int j = 0; j < kN; ++j) s[j] = 0.0f;
  constexpr int kPer = kMaxGrid / kFin;   // 8: all loads issued before the sums
  float v[kPer][kN];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int g = q + k * kFin;
#pragma unroll
    for (int j = 0; j < kN; ++j)
      v[k][j] = g < (int)gridDim.x ? ld_wt(part + ((size_t)g * C + ch) * kN + j) : 0.0f;
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k)
#pragma unroll
    for (int j = 0; j < kN; ++j) s[j] += v[k][j];
#pragma unroll
  for (int j = 0; j < kN; ++j) red[q][ch][j] = s[j];
  __syncthreads();
  if (tid < C) {
    bool bad = false;
#pragma unroll
    for (int j = 0; j < kN; ++j) {
      float t = 0.0f;
      for (int k = 0; k < kFin; ++k) t += red[k][tid][j];
      out[j][tid] = t;
      bad = bad || !finitef(t);
    }
    guard_raise(guard, DT_GUARD_BN_BWD, bad);
  }
}

// ---- backward 1: dbeta = sum(dy), dgamma = sum(dy * xhat) ---------------------------
__global__ void __launch_bounds__(kT)
bn_bwd_reduce_kernel(int64_t m, const float* __restrict__ dy, const float* __restrict__ z,
                     const float* __restrict__ bias, float slope,
                     const float* __restrict__ mean_invstd, float* __restrict__ dgamma,
                     float* __restrict__ dbeta, float* __restrict__ work,
                     int32_t* __restrict__ guard) {
  const int cg = threadIdx.x & 7;
  const float4 b = ld4(bias, cg);
  const float4 mu = ld4(mean_invstd, cg), is = ld4(mean_invstd + C, cg);
  const float mus[4] = {mu.x, mu.y, mu.z, mu.w}, iss[4] = {is.x, is.y, is.z, is.w};
  float acc[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  const int64_t items = m * 8, stride = (int64_t)gridDim.x * kT;
  for (int64_t q = (int64_t)blockIdx.x * kT + threadIdx.x; q < items; q += stride) {
    const float4 g4 = ld4(dy, q);
    const float g[4] = {g4.x, g4.y, g4.z, g4.w};
    float x[4];
    leaky4(ld4(z, q), b, slope, x);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[0][k] += g[k];
      acc[1][k] += g[k] * ((x[k] - mus[k]) * iss[k]);
    }
  }
  block_sums<2>(acc, work);
  unsigned int* counters = reinterpret_cast<unsigned int*>(work + (size_t)kMaxGrid * C * 3);
  if (!last_arrival(&counters[1])) return;
  acquire_partials();
  float* const out[2] = {dbeta, dgamma};
  final_sums<2>(work, out, guard);
}

// ---- backward 2: dz, and dbias = sum(dz) ----------------------------------------------
__global__ void __launch_bounds__(kT)
bn_bwd_apply_kernel(int64_t m, const float* __restrict__ dy, const float* __restrict__ z,
                    const float* __restrict__ bias,
                    const float* __restrict__ mean_invstd, const float* __restrict__ gamma,
                    const float* __restrict__ dgamma, const float* __restrict__ dbeta, float slope,
                    float* __restrict__ dz, float* __restrict__ dbias, float* __restrict__ work,
                    int32_t* __restrict__ guard) {
  const int cg = threadIdx.x & 7;
  const float inv_m = 1.0f / (float)m;
  float mu[4], is[4], k1[4], k2[4], k3[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * cg + k;
    mu[k] = mean_invstd[c];
    is[k] = mean_invstd[C + c];
    k1[k] = gamma[c] * is[k];          // da = k1 * (dy - k2 - xhat * k3)
    k2[k] = dbeta[c] * inv_m;
    k3[k] = dgamma[c] * inv_m;
  }
  const float4 b = ld4(bias, cg);
  float acc[1][4] = {{0, 0, 0, 0}};
  const int64_t items = m * 8, stride = (int64_t)gridDim.x * kT;
  for (int64_t q = (int64_t)blockIdx.x * kT + threadIdx.x; q < items; q += stride) {
    const float4 g4 = ld4(dy, q);
    const float g[4] = {g4.x, g4.y, g4.z, g4.w};
    float x[4];
    leaky4(ld4(z, q), b, slope, x);
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = (x[k] - mu[k]) * is[k];
      const float da = k1[k] * (g[k] - k2[k] - xh * k3[k]);
      o[k] = x[k] > 0.0f ? da : da * slope;
      acc[0][k] += o[k];
    }
    st4(dz, q, make_float4(o[0], o[1], o[2], o[3]));
  }
  float* part = work + (size_t)kMaxGrid * C * 2;   // beside backward 1's partials
  block_sums<1>(acc, part);
  unsigned int* counters = reinterpret_cast<unsigned int*>(work + (size_t)kMaxGrid * C * 3);
  if (!last_arrival(&counters[2])) return;
  acquire_partials();
  float* const out[1] = {dbias};
  final_sums<1>(part, out, guard);
}

// ---- multi-tensor Adam and soft update -------------------------------------------------
constexpr int kMtThreads = 256;

__global__ void __launch_bounds__(kMtThreads)
adam_kernel(const dt_mt_tensor* __restrict__ tensors, const int32_t* __restrict__ chunks,
            double* __restrict__ step, const double* __restrict__ lr, double beta1, double beta2,
            double eps, unsigned int* __restrict__ counter, int32_t* __restrict__ guard,
            int grad_bit, int param_bit) {
  const dt_mt_tensor t = tensors[chunks[2 * blockIdx.x]];
  const int64_t start = (int64_t)chunks[2 * blockIdx.x + 1] * DT_MT_CHUNK;
  const int64_t end = start + DT_MT_CHUNK < t.n ? start + DT_MT_CHUNK : t.n;
  const double st = *step + 1.0;
  // torch: step_size = -(lr / (1 - b1^t)), bc2_sqrt = (1 - b2^t)^0.5, Python
  // doubles passed to float32 element ops
  const float step_size = (float)(-(*lr / (1.0 - pow(beta1, st))));
  const float bc2_sqrt = (float)sqrt(1.0 - pow(beta2, st));
  const float w = (float)(1.0 - beta1), b2 = (float)beta2, ob2 = (float)(1.0 - beta2);
  const float fe = (float)eps;
  bool bad_g = false, bad_p = false;
  for (int64_t i = start + threadIdx.x; i < end; i += kMtThreads) {
    const float g = t.b[i];
    bad_g = bad_g || !finitef(g);
    float m = t.c[i];
    m = w < 0.5f ? m + w * (g - m) : g - (g - m) * (1.0f - w);          // lerp
    float v = t.d[i] * b2;                                              // mul_
    v = v + ob2 * g * g;                                                // addcmul_
    const float den = sqrtf(v) / bc2_sqrt + fe;                         // sqrt, div_, add_
    const float p = t.a[i] + step_size * (m / den);                    // addcdiv_
    bad_p = bad_p || !finitef(p);
    t.a[i] = p;
    t.c[i] = m;
    t.d[i] = v;
  }
  guard_raise(guard, grad_bit, bad_g);
  guard_raise(guard, param_bit, bad_p);
  // the step count moves once every workgroup has read it
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int old =
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(step, st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void __launch_bounds__(kMtThreads)
soft_update_kernel(const dt_mt_tensor* __restrict__ tensors, const int32_t* __restrict__ chunks,
                   float keep, float tau) {
  const dt_mt_tensor t = tensors[chunks[2 * blockIdx.x]];
  const int64_t start = (int64_t)chunks[2 * blockIdx.x + 1] * DT_MT_CHUNK;
  const int64_t end = start + DT_MT_CHUNK < t.n ? start + DT_MT_CHUNK : t.n;
  for (int64_t i = start + threadIdx.x; i < end; i += kMtThreads) {
    const float x = t.a[i] * keep;
    const float y = t.b[i] * tau;
    t.a[i] = x + y;
  }
}

// ---- non-finite guard scan ------------------------------------------------------------
struct GuardSet {
  int n;
  dt_guard_tensor t[DT_GUARD_MAX];
};
constexpr int kGuardThreads = 256;

__global__ void __launch_bounds__(kGuardThreads)
guard_scan_kernel(GuardSet set, int32_t* __restrict__ guard) {
  const int64_t tid = (int64_t)blockIdx.x * kGuardThreads + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kGuardThreads;
  for (int k = 0; k < set.n; ++k) {
    const dt_guard_tensor t = set.t[k];
    bool bad = false;
    if (t.dtype == 0) {
      const float* p = static_cast<const float*>(t.p);
      const int64_t n4 = ((uintptr_t)p & 15) == 0 ? t.count / 4 : 0;
      for (int64_t i = tid; i < n4; i += stride) {
        const float4 v = reinterpret_cast<const float4*>(p)[i];
        bad = bad || !finitef(v.x) || !finitef(v.y) || !finitef(v.z) || !finitef(v.w);
      }
      for (int64_t i = 4 * n4 + tid; i < t.count; i += stride) bad = bad || !finitef(p[i]);
    } else {
      const double* p = static_cast<const double*>(t.p);
      for (int64_t i = tid; i < t.count; i += stride) bad = bad || !(fabs(p[i]) <= 1.79769313486231570e308);
    }
    guard_raise(guard, t.bit, bad);
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" {

int64_t dt_train_work_floats(int64_t m) {
  (void)m;
  return (int64_t)kMaxGrid * C * 3 + kCounters;
}

int dt_bn_leaky_fwd(int64_t m, const float* z, const float* bias, float slope, const float* gamma,
                    const float* beta, float eps, float momentum, float* running_mean,
                    float* running_var, int64_t* num_batches_tracked, int32_t updates, float* a,
                    float* y, float* mean_invstd, float* work, int32_t* guard, void* stream) {
  if (updates < 1) return DT_E_ARG;
  if (m < 1 || !z || !bias || !gamma || !beta || !running_mean || !running_var || !y ||
      !mean_invstd || !work)
    return DT_E_ARG;
  if (!aligned16(z) || (a && !aligned16(a)) || !aligned16(y) || !aligned16(bias) ||
      !aligned16(mean_invstd) || !aligned16(gamma) || !aligned16(beta))
    return DT_E_ARG;
  const int g = grid_of(m);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(g), dim3(kT), 0, s, m, z, bias, slope, eps, momentum,
                     running_mean, running_var, num_batches_tracked, (int)updates, a, mean_invstd, work,
                     guard);
  hipLaunchKernelGGL(bn_apply_kernel, dim3(g), dim3(kT), 0, s, m, z, bias, slope, mean_invstd,
                     gamma, beta, y);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_bn_leaky_apply(int64_t m, const float* z, const float* bias, float slope,
                      const float* mean_invstd, const float* gamma, const float* beta, float* y,
                      void* stream) {
  if (m < 1 || !z || !bias || !mean_invstd || !gamma || !beta || !y) return DT_E_ARG;
  if (!aligned16(z) || !aligned16(y) || !aligned16(bias) || !aligned16(mean_invstd) ||
      !aligned16(gamma) || !aligned16(beta))
    return DT_E_ARG;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(grid_of(m)), dim3(kT), 0, (hipStream_t)stream, m, z,
                     bias, slope, mean_invstd, gamma, beta, y);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_bn_leaky_bwd(int64_t m, const float* dy, const float* z, const float* bias,
                    const float* mean_invstd, const float* gamma, float slope, float* dz,
                    float* dbias, float* dgamma, float* dbeta, float* work, int32_t* guard,
                    void* stream) {
  if (m < 1 || !dy || !z || !bias || !mean_invstd || !gamma || !dz || !dbias || !dgamma ||
      !dbeta || !work)
    return DT_E_ARG;
  if (!aligned16(dy) || !aligned16(z) || !aligned16(bias) || !aligned16(dz) ||
      !aligned16(mean_invstd))
    return DT_E_ARG;
  const int g = grid_of(m);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(g), dim3(kT), 0, s, m, dy, z, bias, slope,
                     mean_invstd, dgamma, dbeta, work, guard);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(g), dim3(kT), 0, s, m, dy, z, bias, mean_invstd,
                     gamma, dgamma, dbeta, slope, dz, dbias, work, guard);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_adam(int32_t n_chunks, const dt_mt_tensor* tensors, const int32_t* chunks, double* step,
            const double* lr, double beta1, double beta2, double eps, uint32_t* counter,
            int32_t* guard, int32_t grad_bit, int32_t param_bit, void* stream) {
  if (n_chunks < 0 || (n_chunks > 0 && (!tensors || !chunks || !step || !lr || !counter)))
    return DT_E_ARG;
  if (n_chunks == 0) return DT_OK;
  hipLaunchKernelGGL(adam_kernel, dim3(n_chunks), dim3(kMtThreads), 0, (hipStream_t)stream,
                     tensors, chunks, step, lr, beta1, beta2, eps, counter, guard, (int)grad_bit,
                     (int)param_bit);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_soft_update(int32_t n_chunks, const dt_mt_tensor* tensors, const int32_t* chunks,
                   double tau, void* stream) {
  if (n_chunks < 0 || (n_chunks > 0 && (!tensors || !chunks))) return DT_E_ARG;
  if (n_chunks == 0) return DT_OK;
  // torch: target * (1.0 - tau) + param * tau with the Python doubles as float32 scalars
  hipLaunchKernelGGL(soft_update_kernel, dim3(n_chunks), dim3(kMtThreads), 0, (hipStream_t)stream,
                     tensors, chunks, (float)(1.0 - tau), (float)tau);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_guard_scan(int32_t n, const dt_guard_tensor* tensors, int32_t* guard, void* stream) {
  if (n < 0 || n > DT_GUARD_MAX || !guard || (n > 0 && !tensors)) return DT_E_ARG;
  GuardSet set{};
  set.n = n;
  int64_t most = 0;
  for (int k = 0; k < n; ++k) {
    const dt_guard_tensor& t = tensors[k];
    if (t.count < 0 || (t.count > 0 && !t.p) || t.bit < 0 || t.bit > 31 || t.dtype < 0 ||
        t.dtype > 1)
      return DT_E_ARG;
    set.t[k] = t;
    most = t.count > most ? t.count : most;
  }
  if (most == 0) return DT_OK;
  // ~4 elements a thread (a float4 or four doubles): a 4096-double reward
  // scan takes 4 workgroups, not one walking 16 strided loads a thread
  int64_t g = (most + kGuardThreads * 4 - 1) / (kGuardThreads * 4);
  g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
  hipLaunchKernelGGL(guard_scan_kernel, dim3((unsigned)g), dim3(kGuardThreads), 0,
                     (hipStream_t)stream, set, guard);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

}  // extern "C"
