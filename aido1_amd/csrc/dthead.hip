// The DDPG update's small fully connected tails (include/dthead.h): the
// critic's concat -> linear 128 -> leaky_relu -> linear 1 and the actor's
// linear 2 -> tanh at batch 64, forward in one launch and backward in one.
// At these sizes every step is a global-load latency (~1 us), not bandwidth
// or FLOPs, so both kernels are built to keep that chain short: operands are
// staged into LDS with each thread's loads all issued before its stores, and
// the forward keeps the next output's weights in flight while it multiplies.
//
// Forward: a workgroup takes kRows rows of x (staged in LDS, the two inputs
// side by side as torch.cat lays them out); lane groups of kGrp lanes compute
// one output each (strided partial sums over k, then a butterfly), kRows rows
// at once so each weight is read once per workgroup; layer 1's outputs stay in
// LDS for layer 2.
// Backward: every workgroup rebuilds the output gradients of layer 2
// (g2 = dy act2'(y)) and layer 1 (g1 = (g2 w2) act1'(h)) in LDS, then owns a
// block of input columns of dw1 or of dx (its x or w1 columns staged in LDS);
// workgroup 0 also writes the bias and layer-2 weight gradients.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/dthead.h"

namespace {

// rows a forward workgroup (tools/ab.sh variants)
#ifndef DTHEAD_ROWS
#define DTHEAD_ROWS 1
#endif
constexpr int kRows = DTHEAD_ROWS;
constexpr int kGrp = 16;          // lanes per output (forward)
constexpr int kMaxM = 256, kMaxK = 1024, kMaxN1 = 1024, kMaxN2 = 64;
constexpr int kMaxH = 512;        // n1 of a two-layer tail (its outputs stay in LDS)
constexpr int kMaxG1 = 8192;      // m * n1 (backward: layer 1's output gradient in LDS)
constexpr int kMaxG2 = 2048;      // m * n2
constexpr int kMaxW2 = 4096;      // n2 * n1 (backward: w2 in LDS)
constexpr int kBwdThreads = 1024;
constexpr int kKB = 32;           // input columns a backward workgroup (at most)
constexpr int kStage = 8192;      // floats of staged x or w1 columns (m * kw, n1 * kw)
constexpr int kU = 8;             // staging loads in flight a thread

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

// LDS staging: element i of [0, total) is fetch(i, dst) stored at *dst; a
// thread issues kU fetches before any of its stores.
template <int NT, class Fetch>
__device__ __forceinline__ void stage(int total, Fetch fetch) {
  for (int base = threadIdx.x; base < total; base += kU * NT) {
    float v[kU];
    float* d[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int i = base + u * NT;
      d[u] = nullptr;
      v[u] = i < total ? fetch(i, d[u]) : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (d[u]) *d[u] = v[u];
  }
}

// A lane's KW weights of output n (k = gl, gl + kGrp, ...; K <= kGrp KW).
template <int KW>
__device__ __forceinline__ void load_w(float (&wv)[KW], const float* __restrict__ w, int K, int N,
                                       int n, int gl) {
  const bool on = n < N;
  const float* wr = w + (size_t)(on ? n : 0) * K;
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const int k = gl + kGrp * j;
    wv[j] = (on && k < K) ? wr[k] : 0.0f;
  }
}

// The TD target epilogue (dt_mlp_fwd_td): out[r][n] = rew[r] + (notdone[r] *
// gamma) * y[r][n], the trainer's y = r + notdone * gamma * Q'(s', a') in its
// operation order (training/trainers.py:166-170); pointers at the workgroup's
// first row.
struct Td {
  const float* rew;
  const float* notdone;
  float gamma;
  float* out;
};

// out[r][n] = act(b[n] + sum_k in[r][k] w[n][k]) for the workgroup's rows:
// lane group (kGrp lanes) per output n, kRows accumulators a lane.  wa holds
// the lane's weights of its first output (load_w); the next output's are in
// flight while this one's products run.
template <int KW, int NT>
__device__ __forceinline__ void layer_fwd(float (&wa)[KW], const float* in, int K,
                                          const float* __restrict__ w, const float* __restrict__ b,
                                          int N, int act, float s, int rows, float* out_lds,
                                          float* out, int ldo, const Td* td = nullptr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane / kGrp, gl = lane % kGrp;
  constexpr int kPerWave = 64 / kGrp;
  constexpr int kStep = (NT / 64) * kPerWave;
  for (int n0 = wave * kPerWave; n0 < N; n0 += kStep) {
    const int n = n0 + grp;
    float wb[KW];
    const bool more = n0 + kStep < N;
    if (more) load_w<KW>(wb, w, K, N, n + kStep, gl);
    const float bias = (b && n < N) ? b[n] : 0.0f;
    float acc[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) acc[r] = 0.0f;
#pragma unroll
    for (int j = 0; j < KW; ++j) {
      const int k = gl + kGrp * j;
      if (k < K)
#pragma unroll
        for (int r = 0; r < kRows; ++r) acc[r] = fmaf(in[r * K + k], wa[j], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r)
#pragma unroll
      for (int o = kGrp / 2; o > 0; o >>= 1) acc[r] += __shfl_xor(acc[r], o, kGrp);
    if (n < N) {
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        if (gl == r && r < rows) {
          const float v = act_fwd(act, acc[r] + bias, s);
          if (out_lds) out_lds[r * N + n] = v;
          if (out) out[(size_t)r * ldo + n] = v;
          if (td) td->out[(size_t)r * N + n] = td->rew[r] + (td->notdone[r] * td->gamma) * v;
        }
      }
    }
    if (more)
#pragma unroll
      for (int j = 0; j < KW; ++j) wa[j] = wb[j];
  }
}

template <int KW1, int KW2, int NT>
__global__ void __launch_bounds__(NT) mlp_fwd_kernel(DtMlp p, const float* __restrict__ x0,
                                                     const float* __restrict__ x1,
                                                     float* __restrict__ h,
                                                     float* __restrict__ y, Td td) {
  __shared__ float xs[kRows * kMaxK];
  __shared__ float hs[kRows * kMaxH];
  const int r0 = blockIdx.x * kRows;
  const int rows = p.m - r0 < kRows ? p.m - r0 : kRows;
  const int K = p.k0 + p.k1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float wa[KW1];   // layer 1's first weights, in flight while x is staged
  load_w<KW1>(wa, p.w1, K, p.n1, wave * (64 / kGrp) + lane / kGrp, lane % kGrp);
  stage<NT>(kRows * K, [&](int i, float*& d) __attribute__((always_inline)) {
    const int r = i / K, k = i - r * K;
    d = xs + i;
    if (r >= rows) return 0.0f;
    return k < p.k0 ? x0[(size_t)(r0 + r) * p.k0 + k] : x1[(size_t)(r0 + r) * p.k1 + (k - p.k0)];
  });
  __syncthreads();
  const int nout = p.n2 > 0 ? p.n2 : p.n1;
  const Td tdr{td.rew + r0, td.notdone + r0, td.gamma, td.out + (size_t)r0 * nout};
  const Td* tdp = td.out ? &tdr : nullptr;
  layer_fwd<KW1, NT>(wa, xs, K, p.w1, p.b1, p.n1, p.act1, p.slope, rows,
                     p.n2 > 0 ? hs : nullptr, h + (size_t)r0 * p.n1, p.n1,
                     p.n2 > 0 ? nullptr : tdp);
  if (p.n2 > 0) {
    float w2[KW2];
    load_w<KW2>(w2, p.w2, p.n1, p.n2, wave * (64 / kGrp) + lane / kGrp, lane % kGrp);
    __syncthreads();
    layer_fwd<KW2, NT>(w2, hs, p.n1, p.w2, p.b2, p.n2, p.act2, p.slope, rows, nullptr,
                       y + (size_t)r0 * p.n2, p.n2, tdp);
  }
}

// ---- backward ---------------------------------------------------------------------
struct BwdOut {
  float *dx0, *dx1, *dw1, *db1, *dw2, *db2;
  int blocks_w1;   // workgroups on dw1 (the rest on dx)
  int kw;          // input columns a workgroup: kStage / max(m, n1), at most kKB
};

// Workgroup b < blocks_w1 owns dw1[:, kb:kb+kw] (x's columns staged:
// dw1[n][k] = sum_r g1[r][n] x[r][k]), the others dx[:, kb:kb+kw] (w1's
// columns staged: dx[r][k] = sum_n g1[r][n] w1[n][k]).
__global__ void __launch_bounds__(kBwdThreads) mlp_bwd_kernel(DtMlp p, const float* __restrict__ x0,
                                                              const float* __restrict__ x1,
                                                              const float* __restrict__ h,
                                                              const float* __restrict__ y,
                                                              const float* __restrict__ dy,
                                                              BwdOut o) {
  __shared__ float g1[kMaxG1];
  __shared__ float hs[kMaxG1];
  __shared__ float g2[kMaxG2];
  __shared__ float w2s[kMaxW2];
  __shared__ float st[kStage];
  const int tid = threadIdx.x;
  const int m = p.m, n1 = p.n1, n2 = p.n2, K = p.k0 + p.k1;
  const int b = blockIdx.x;
  const bool wgrad = b < o.blocks_w1;
  const bool dx = !wgrad && (o.dx0 || o.dx1);
  const int kW = o.kw;
  const int kb = (wgrad ? b : b - o.blocks_w1) * kW;   // the block's first column
  const int kn = K - kb < kW ? K - kb : kW;
  // one staging pass: the block's operand columns, then h, w2 and g2 (two
  // layers) or g1 straight from dy and h (one layer)
  const int s0 = wgrad ? m * kW : (dx ? n1 * kW : 0);
  const int s1 = s0 + m * n1;
  const int s2 = s1 + (n2 > 0 ? n2 * n1 : 0);
  const int s3 = s2 + m * n2;
  stage<kBwdThreads>(s3, [&](int i, float*& d) __attribute__((always_inline)) {
    if (i < s0) {
      d = st + i;
      if (wgrad) {
        const int r = i / kW, c = i - r * kW, k = kb + c;
        if (c >= kn) return 0.0f;
        return k < p.k0 ? x0[(size_t)r * p.k0 + k] : x1[(size_t)r * p.k1 + (k - p.k0)];
      }
      const int n = i / kW, c = i - n * kW;
      return c < kn ? p.w1[(size_t)n * K + kb + c] : 0.0f;
    }
    if (i < s1) {
      const int j = i - s0;
      if (n2 > 0) {
        d = hs + j;
        return h[j];
      }
      d = g1 + j;
      return dy[j] * act_bwd(p.act1, h[j], p.slope);
    }
    if (i < s2) {
      d = w2s + (i - s1);
      return p.w2[i - s1];
    }
    const int j = i - s2;
    d = g2 + j;
    return dy[j] * act_bwd(p.act2, y[j], p.slope);
  });
  __syncthreads();
  if (n2 > 0) {
    for (int i = tid; i < m * n1; i += kBwdThreads) {
      const int r = i / n1, n = i - r * n1;
      float a = 0.0f;
      for (int j = 0; j < n2; ++j) a = fmaf(g2[r * n2 + j], w2s[j * n1 + n], a);
      g1[i] = a * act_bwd(p.act1, hs[i], p.slope);
    }
    __syncthreads();
  }
  if (wgrad) {   // dw1[n][kb + c] = sum_r g1[r][n] x[r][kb + c]
    for (int i = tid; i < n1 * kn; i += kBwdThreads) {
      const int n = i / kn, c = i - n * kn;
      float a = 0.0f;
      for (int r = 0; r < m; ++r) a = fmaf(g1[r * n1 + n], st[r * kW + c], a);
      o.dw1[(size_t)n * K + kb + c] = a;
    }
  } else if (dx) {   // dx[r][kb + c] = sum_n g1[r][n] w1[n][kb + c]
    for (int i = tid; i < m * kn; i += kBwdThreads) {
      const int r = i / kn, c = i - r * kn, k = kb + c;
      float* dst = k < p.k0 ? o.dx0 : o.dx1;
      if (!dst) continue;
      float a = 0.0f;
      for (int n = 0; n < n1; ++n) a = fmaf(g1[r * n1 + n], st[n * kW + c], a);
      if (k < p.k0)
        dst[(size_t)r * p.k0 + k] = a;
      else
        dst[(size_t)r * p.k1 + (k - p.k0)] = a;
    }
  }
  if (b == 0) {   // the bias gradients and layer 2's weights
    if (o.db1)
      for (int n = tid; n < n1; n += kBwdThreads) {
        float a = 0.0f;
        for (int r = 0; r < m; ++r) a += g1[r * n1 + n];
        o.db1[n] = a;
      }
    if (n2 > 0 && o.dw2)
      for (int i = tid; i < n2 * n1; i += kBwdThreads) {
        const int j = i / n1, n = i - j * n1;
        float a = 0.0f;
        for (int r = 0; r < m; ++r) a = fmaf(g2[r * n2 + j], hs[r * n1 + n], a);
        o.dw2[i] = a;
      }
    if (n2 > 0 && o.db2)
      for (int j = tid; j < n2; j += kBwdThreads) {
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
         p->m * p->n2 <= kMaxG2 && (p->n2 == 0 || (p->n1 <= kMaxH && p->n2 * p->n1 <= kMaxW2)) &&
         p->act1 >= 0 && p->act1 <= 3 && p->act2 >= 0 &&
         p->act2 <= 3 && p->slope >= 0.0f && p->w1 && (p->n2 == 0 || p->w2);
}

int mlp_fwd(const DtMlp* p, const float* x0, const float* x1, float* h, float* y, Td td,
            void* stream) {
  if (!mlp_ok(p) || !x0 || (p->k1 > 0 && !x1) || !h || (p->n2 > 0 && !y)) return DT_E_ARG;
  const int kw1 = (p->k0 + p->k1 + kGrp - 1) / kGrp, kw2 = (p->n1 + kGrp - 1) / kGrp;
  const dim3 grid((p->m + kRows - 1) / kRows);
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto kern, int nt) {
    hipLaunchKernelGGL(kern, grid, dim3(nt), 0, s, *p, x0, x1, h, y, td);
  };
  const bool two = p->n2 > 0;
  if (kw1 <= 16 && (!two || kw2 <= 8)) go(mlp_fwd_kernel<16, 8, 1024>, 1024);
  else if (kw1 <= 32 && (!two || kw2 <= 8)) go(mlp_fwd_kernel<32, 8, 1024>, 1024);
  else if (kw1 <= 32) go(mlp_fwd_kernel<32, 32, 1024>, 1024);
  else go(mlp_fwd_kernel<64, 32, 512>, 512);   // 64 weights a lane: half the lanes
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// ---- the two DDPG losses (training/trainers.py:174-177, 193-196) -------------------
// One workgroup: the f64 sum of the m terms in a fixed tree order, then / m.
constexpr int kLossThreads = 256;

__device__ double block_sum(double v) {
  __shared__ double part[kLossThreads / 64];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < kLossThreads / 64; ++w) t += part[w];
  return t;
}

// kind 0: mean((a - b)^2) (F.mse_loss); kind 1: -mean(a) (the actor loss)
__global__ void __launch_bounds__(kLossThreads) loss_kernel(int kind, int m, const float* a,
                                                            const float* b, float* loss) {
  double acc = 0.0;
  for (int i = threadIdx.x; i < m; i += kLossThreads) {
    const float d = kind == 0 ? a[i] - b[i] : a[i];
    acc += kind == 0 ? (double)(d * d) : (double)d;
  }
  const double t = block_sum(acc);
  if (threadIdx.x == 0) *loss = kind == 0 ? (float)(t / m) : (float)(-(t / m));
}

// d loss / d a for a scalar upstream gradient *g: kind 0: g * 2 (a - b) / m;
// kind 1: -g / m (both as torch's backward formulas order them)
__global__ void __launch_bounds__(kLossThreads) loss_bwd_kernel(int kind, int m, const float* a,
                                                                const float* b, const float* g,
                                                                float* da) {
  const float gv = *g;
  const float norm = 2.0f / (float)m;
  for (int i = blockIdx.x * kLossThreads + threadIdx.x; i < m; i += gridDim.x * kLossThreads)
    da[i] = kind == 0 ? norm * (a[i] - b[i]) * gv : -(gv / (float)m);
}

}  // namespace

extern "C" {


int dt_mlp_fwd(const DtMlp* p, const float* x0, const float* x1, float* h, float* y,
               void* stream) {
  return mlp_fwd(p, x0, x1, h, y, Td{nullptr, nullptr, 0.0f, nullptr}, stream);
}

int dt_mlp_fwd_td(const DtMlp* p, const float* x0, const float* x1, float* h, float* y,
                  const float* rew, const float* notdone, float gamma, float* target,
                  void* stream) {
  if (!rew || !notdone || !target) return DT_E_ARG;
  return mlp_fwd(p, x0, x1, h, y, Td{rew, notdone, gamma, target}, stream);
}

int dt_loss(int32_t kind, int32_t m, const float* a, const float* b, float* loss, void* stream) {
  if (kind < 0 || kind > 1 || m < 1 || !a || (kind == 0 && !b) || !loss) return DT_E_ARG;
  hipLaunchKernelGGL(loss_kernel, dim3(1), dim3(kLossThreads), 0, (hipStream_t)stream, kind, m,
                     a, b, loss);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_loss_bwd(int32_t kind, int32_t m, const float* a, const float* b, const float* g,
                float* da, void* stream) {
  if (kind < 0 || kind > 1 || m < 1 || !a || (kind == 0 && !b) || !g || !da) return DT_E_ARG;
  const int grid = (m + kLossThreads - 1) / kLossThreads;
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(grid < 64 ? grid : 64), dim3(kLossThreads), 0,
                     (hipStream_t)stream, kind, m, a, b, g, da);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_mlp_bwd(const DtMlp* p, const float* x0, const float* x1, const float* h, const float* y,
               const float* dy, float* dx0, float* dx1, float* dw1, float* db1, float* dw2,
               float* db2, void* stream) {
  if (!mlp_ok(p) || !h || !dy || (p->n2 > 0 && !y) || (dw1 && (!x0 || (p->k1 > 0 && !x1))) ||
      (dx1 && p->k1 == 0))
    return DT_E_ARG;
  const int K = p->k0 + p->k1;
  const int big = p->m > p->n1 ? p->m : p->n1;
  const int kw = kStage / big < kKB ? kStage / big : kKB;   // >= 8 (m <= 256, n1 <= 1024)
  const int blocks = (K + kw - 1) / kw;
  BwdOut o{dx0, dx1, dw1, db1, p->n2 > 0 ? dw2 : nullptr, p->n2 > 0 ? db2 : nullptr, 0, kw};
  o.blocks_w1 = dw1 ? blocks : 0;
  const int bx = (dx0 || dx1) ? blocks : 0;
  const int grid = o.blocks_w1 + bx > 0 ? o.blocks_w1 + bx : 1;
  hipLaunchKernelGGL(mlp_bwd_kernel, dim3(grid), dim3(kBwdThreads), 0, (hipStream_t)stream, *p, x0,
                     x1, h, y, dy, o);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

}  // extern "C"
