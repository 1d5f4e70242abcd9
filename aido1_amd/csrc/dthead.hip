// The DDPG update's small fully connected tails (include/dthead.h): the
// critic's concat -> linear 128 -> leaky_relu -> linear 1 and the actor's
// linear 2 -> tanh at batch 64, forward in one launch and backward in one.
//
// Forward: a workgroup takes kRows rows of x (staged in LDS, the two inputs
// side by side as torch.cat lays them out); each wave computes outputs in
// groups of kGrp lanes per output (strided partial sums over k, then a
// butterfly within the group), kRows rows at once so each weight is read once
// per workgroup; layer 1's outputs stay in LDS for layer 2.
// Backward: every workgroup first rebuilds the output gradients of layer 2
// (g2 = dy act2'(y)) and layer 1 (g1 = (g2 w2) act1'(h)) in LDS (a few
// thousand products), then takes a block of the flattened dw1 / dx elements
// (one dot product over the m rows, or over n1, per element); workgroup 0
// also the bias and layer-2 weight gradients.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/dthead.h"

namespace {

constexpr int kThreads = 256;
constexpr int kRows = 8;          // rows a forward workgroup
constexpr int kGrp = 16;          // lanes per output (forward)
constexpr int kMaxM = 256, kMaxK = 1024, kMaxN1 = 1024, kMaxN2 = 64;
constexpr int kMaxH = 512;        // n1 of a two-layer tail (its outputs stay in LDS)
constexpr int kMaxG1 = 8192;      // m * n1 (backward: layer 1's output gradient in LDS)
constexpr int kMaxG2 = 2048;      // m * n2
constexpr int kBwdPer = 4;        // elements a thread (backward)

enum { kActNone = 0, kActLeaky = 1, kActTanh = 2, kActSigmoid = 3 };

__device__ __forceinline__ float act_fwd(int a, float v, float s) {
  switch (a) {
    case kActLeaky: return v > 0.0f ? v : v * s;   // torch: x if x > 0 else x * slope
    case kActTanh: return tanhf(v);
    case kActSigmoid: return 1.0f / (1.0f + expf(-v));
    default: return v;
  }
}
// the derivative from the OUTPUT (slope >= 0: the output's sign is the input's)
__device__ __forceinline__ float act_bwd(int a, float out, float s) {
  switch (a) {
    case kActLeaky: return out > 0.0f ? 1.0f : s;
    case kActTanh: return 1.0f - out * out;
    case kActSigmoid: return out * (1.0f - out);
    default: return 1.0f;
  }
}

// out[r][n] = act(b[n] + sum_k in[r][k] w[n][k]) for the workgroup's rows:
// lane group (kGrp lanes) per output n, kRows accumulators a lane
__device__ __forceinline__ void layer_fwd(const float* in, int K, const float* __restrict__ w,
                                          const float* __restrict__ b, int N, int act, float s,
                                          int rows, float* out_lds, float* out, int ldo) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / kGrp, gl = lane % kGrp;
  constexpr int kPerWave = 64 / kGrp;
  for (int n0 = wave * kPerWave; n0 < N; n0 += (kThreads / 64) * kPerWave) {
    const int n = n0 + grp;
    const bool on = n < N;
    float acc[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) acc[r] = 0.0f;
    if (on) {
      const float* wr = w + (size_t)n * K;
      for (int k = gl; k < K; k += kGrp) {
        const float wv = wr[k];
#pragma unroll
        for (int r = 0; r < kRows; ++r) acc[r] = fmaf(in[r * K + k], wv, acc[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r)
#pragma unroll
      for (int o = kGrp / 2; o > 0; o >>= 1) acc[r] += __shfl_xor(acc[r], o, kGrp);
    if (on) {
      const float bias = b ? b[n] : 0.0f;
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        if (gl == r && r < rows) {
          const float v = act_fwd(act, acc[r] + bias, s);
          if (out_lds) out_lds[r * N + n] = v;
          if (out) out[(size_t)r * ldo + n] = v;
        }
      }
    }
  }
}

__global__ void __launch_bounds__(kThreads) mlp_fwd_kernel(DtMlp p, const float* __restrict__ x0,
                                                           const float* __restrict__ x1,
                                                           float* __restrict__ h,
                                                           float* __restrict__ y) {
  __shared__ float xs[kRows * kMaxK];
  __shared__ float hs[kRows * kMaxH];
  const int r0 = blockIdx.x * kRows;
  const int rows = p.m - r0 < kRows ? p.m - r0 : kRows;
  const int K = p.k0 + p.k1;
  for (int i = threadIdx.x; i < kRows * K; i += kThreads) {
    const int r = i / K, k = i - r * K;
    float v = 0.0f;
    if (r < rows)
      v = k < p.k0 ? x0[(size_t)(r0 + r) * p.k0 + k] : x1[(size_t)(r0 + r) * p.k1 + (k - p.k0)];
    xs[i] = v;
  }
  __syncthreads();
  layer_fwd(xs, K, p.w1, p.b1, p.n1, p.act1, p.slope, rows, p.n2 > 0 ? hs : nullptr,
            h + (size_t)r0 * p.n1, p.n1);
  if (p.n2 > 0) {
    __syncthreads();
    layer_fwd(hs, p.n1, p.w2, p.b2, p.n2, p.act2, p.slope, rows, nullptr, y + (size_t)r0 * p.n2,
              p.n2);
  }
}

struct BwdOut {
  float *dx0, *dx1, *dw1, *db1, *dw2, *db2;
  int blocks_w1;   // workgroups on dw1 (the rest on dx)
};

__global__ void __launch_bounds__(kThreads) mlp_bwd_kernel(DtMlp p, const float* __restrict__ x0,
                                                           const float* __restrict__ x1,
                                                           const float* __restrict__ h,
                                                           const float* __restrict__ y,
                                                           const float* __restrict__ dy,
                                                           BwdOut o) {
  __shared__ float g1[kMaxG1];
  __shared__ float g2[kMaxG2];
  const int tid = threadIdx.x;
  const int m = p.m, n1 = p.n1, n2 = p.n2, K = p.k0 + p.k1;
  // output gradients of both layers (every workgroup: a few thousand products)
  if (n2 > 0) {
    for (int i = tid; i < m * n2; i += kThreads) g2[i] = dy[i] * act_bwd(p.act2, y[i], p.slope);
    __syncthreads();
    for (int i = tid; i < m * n1; i += kThreads) {
      const int r = i / n1, n = i - r * n1;
      float a = 0.0f;
      for (int j = 0; j < n2; ++j) a = fmaf(g2[r * n2 + j], p.w2[(size_t)j * n1 + n], a);
      g1[i] = a * act_bwd(p.act1, h[i], p.slope);
    }
  } else {
    for (int i = tid; i < m * n1; i += kThreads) g1[i] = dy[i] * act_bwd(p.act1, h[i], p.slope);
  }
  __syncthreads();
  auto xat = [&](int r, int k) __attribute__((always_inline)) {
    return k < p.k0 ? x0[(size_t)r * p.k0 + k] : x1[(size_t)r * p.k1 + (k - p.k0)];
  };
  const int b = blockIdx.x;
  if (b < o.blocks_w1) {   // dw1[n][k] = sum_r g1[r][n] x[r][k]
    const int base = b * kThreads * kBwdPer;
#pragma unroll
    for (int e = 0; e < kBwdPer; ++e) {
      const int i = base + e * kThreads + tid;
      if (i >= n1 * K) break;
      const int n = i / K, k = i - n * K;
      float a = 0.0f;
      for (int r = 0; r < m; ++r) a = fmaf(g1[r * n1 + n], xat(r, k), a);
      o.dw1[i] = a;
    }
  } else if (o.dx0 || o.dx1) {   // dx[r][k] = sum_n g1[r][n] w1[n][k]
    const int base = (b - o.blocks_w1) * kThreads * kBwdPer;
#pragma unroll
    for (int e = 0; e < kBwdPer; ++e) {
      const int i = base + e * kThreads + tid;
      if (i >= m * K) break;
      const int r = i / K, k = i - r * K;
      float* dst = k < p.k0 ? o.dx0 : o.dx1;
      if (!dst) continue;
      float a = 0.0f;
      for (int n = 0; n < n1; ++n) a = fmaf(g1[r * n1 + n], p.w1[(size_t)n * K + k], a);
      if (k < p.k0)
        dst[(size_t)r * p.k0 + k] = a;
      else
        dst[(size_t)r * p.k1 + (k - p.k0)] = a;
    }
  }
  if (b == 0) {   // the bias gradients and layer 2's weights
    if (o.db1)
      for (int n = tid; n < n1; n += kThreads) {
        float a = 0.0f;
        for (int r = 0; r < m; ++r) a += g1[r * n1 + n];
        o.db1[n] = a;
      }
    if (n2 > 0 && o.dw2)
      for (int i = tid; i < n2 * n1; i += kThreads) {
        const int j = i / n1, n = i - j * n1;
        float a = 0.0f;
        for (int r = 0; r < m; ++r) a = fmaf(g2[r * n2 + j], h[(size_t)r * n1 + n], a);
        o.dw2[i] = a;
      }
    if (n2 > 0 && o.db2)
      for (int j = tid; j < n2; j += kThreads) {
        float a = 0.0f;
        for (int r = 0; r < m; ++r) a += g2[r * n2 + j];
        o.db2[j] = a;
      }
  }
}

bool mlp_ok(const DtMlp* p) {
  if (!p) return false;
  const int K = p->k0 + p->k1;
  return p->m >= 1 && p->m <= kMaxM && p->k0 >= 1 && p->k1 >= 0 && K <= kMaxK && p->n1 >= 1 &&
         p->n1 <= kMaxN1 && p->n2 >= 0 && p->n2 <= kMaxN2 && p->m * p->n1 <= kMaxG1 &&
         p->m * p->n2 <= kMaxG2 && (p->n2 == 0 || p->n1 <= kMaxH) && p->act1 >= 0 && p->act1 <= 3 && p->act2 >= 0 &&
         p->act2 <= 3 && p->slope >= 0.0f && p->w1 && (p->n2 == 0 || p->w2);
}

}  // namespace

extern "C" {

int dt_mlp_fwd(const DtMlp* p, const float* x0, const float* x1, float* h, float* y,
               void* stream) {
  if (!mlp_ok(p) || !x0 || (p->k1 > 0 && !x1) || !h || (p->n2 > 0 && !y)) return DT_E_ARG;
  hipLaunchKernelGGL(mlp_fwd_kernel, dim3((p->m + kRows - 1) / kRows), dim3(kThreads), 0,
                     (hipStream_t)stream, *p, x0, x1, h, y);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_mlp_bwd(const DtMlp* p, const float* x0, const float* x1, const float* h, const float* y,
               const float* dy, float* dx0, float* dx1, float* dw1, float* db1, float* dw2,
               float* db2, void* stream) {
  if (!mlp_ok(p) || !h || !dy || (p->n2 > 0 && !y) || (dw1 && (!x0 || (p->k1 > 0 && !x1))) ||
      (dx1 && p->k1 == 0))
    return DT_E_ARG;
  const int K = p->k0 + p->k1;
  const int per = kThreads * kBwdPer;
  BwdOut o{dx0, dx1, dw1, db1, p->n2 > 0 ? dw2 : nullptr, p->n2 > 0 ? db2 : nullptr, 0};
  o.blocks_w1 = dw1 ? (p->n1 * K + per - 1) / per : 0;
  const int bx = (dx0 || dx1) ? (p->m * K + per - 1) / per : 0;
  const int grid = o.blocks_w1 + bx > 0 ? o.blocks_w1 + bx : 1;
  hipLaunchKernelGGL(mlp_bwd_kernel, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, *p, x0,
                     x1, h, y, dy, o);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

}  // extern "C"
