// GPU prioritized replay: the sum/min segment trees of utils/segment_tree.py
// and the index logic of utils/buffers.py:140-259 (PrioritizedReplayBuffer),
// batched.  See include/dtreplay.h for the contract.
//
// Exactness: every tree node is combined from its two children exactly as
// SegmentTree.__setitem__ does (segment_tree.py:77-87), so after a batch of
// leaf writes the bottom-up recompute of the touched paths leaves the same
// float64 values the reference's one-at-a-time loop leaves; the prefix-sum
// descent and the range sum use the reference's comparison / subtraction /
// nesting order, so sampled indices are bit-identical for the same uniforms.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "../../include/dtreplay.h"
#include "dtrender.h"   // dr::kPalGray (palette-index frames)

struct dt_per {
  int device = 0;
  int64_t size = 0, cap = 0, len = 0, next = 0;
  int log2cap = 0;
  double alpha = 0.0;
  double* sum = nullptr;   // [2*cap]
  double* mn = nullptr;    // [2*cap]
  double* maxp = nullptr;  // [1]
  int32_t* winner = nullptr;  // [cap], -1 when idle
  int32_t* err = nullptr;     // [2] bits (0: bad priority, 1: bad index), rejected entries
  void* buf = nullptr;
  std::string msg;
};

namespace {

constexpr int kTreeThreads = 1024;
constexpr int kSampleThreads = 256;
constexpr int kMaxDepth = 40;

// Python's min(a, b): the first argument unless the second is smaller.
__device__ __forceinline__ double py_min(double a, double b) { return b < a ? b : a; }

__device__ __forceinline__ void recompute(double* sum, double* mn, int64_t node) {
  sum[node] = sum[2 * node] + sum[2 * node + 1];
  mn[node] = py_min(mn[2 * node], mn[2 * node + 1]);
}

__global__ void fill_kernel(double* sum, double* mn, double* maxp, int32_t* winner, int64_t cap) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 2 * cap;
       i += (int64_t)gridDim.x * blockDim.x) {
    sum[i] = 0.0;
    mn[i] = INFINITY;
    if (i < cap) winner[i] = -1;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *maxp = 1.0;
}

// n adds starting at slot `next`; one workgroup.  Every new leaf gets the same
// value v, so a touched node whose leaf span lies inside the written range
// [L, H) holds exactly v * 2^level (sum: sums of equal halves double exactly)
// and v (min): those are written in parallel, with no level-by-level
// dependency.  The <= 2 nodes a level whose spans cross L or H are recomputed
// by one lane from their children -- closed-form, the previous level's
// crossing node, or an untouched node, all untouched ones loaded into LDS at
// once first -- so the walk to the root is one load latency, not one a level.
// The same values as recomputing every touched node level by level.  A batch
// that wraps at `size` (two ranges) takes the level-by-level walk.
constexpr int kAddMaxLevels = 40;

__global__ void __launch_bounds__(kTreeThreads)
add_kernel(double* sum, double* mn, const double* maxp, int64_t cap, int log2cap, int64_t size,
           int64_t next, int64_t n, double alpha, int64_t* slots) {
  __shared__ double pre_s[kAddMaxLevels * 4], pre_m[kAddMaxLevels * 4];
  const double v = pow(*maxp, alpha);  // buffers.py:173-174
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
    const int64_t s = (next + k) % size;
    if (slots) slots[k] = s;
  }
  const int64_t m = n < size ? n : size;  // distinct slots written
  const int64_t end = next + m;
  if (end <= size) {
    const int64_t L = cap + next, H = cap + end;   // leaf-node range [L, H)
    auto interior = [&](int64_t p, int l) { return (p << l) >= L && ((p + 1) << l) <= H; };
    auto untouched = [&](int64_t p, int l) { return ((p + 1) << l) <= L || (p << l) >= H; };
    // the untouched children of the crossing nodes, every level at once
    for (int it = threadIdx.x; it < 4 * log2cap; it += blockDim.x) {
      const int l = it / 4 + 1, side = (it >> 1) & 1, ch = it & 1;
      const int64_t p = side ? (H - 1) >> l : L >> l;
      const int64_t c = 2 * p + ch;
      if (!interior(p, l) && untouched(c, l - 1)) {
        pre_s[it] = sum[c];
        pre_m[it] = mn[c];
      }
    }
    // the interior nodes (leaves included)
    for (int l = 0; l <= log2cap; ++l) {
      const int64_t first = ((L + (int64_t(1) << l) - 1) >> l), last = (H >> l) - 1;
      const double sv = ldexp(v, l);
      for (int64_t p = first + threadIdx.x; p <= last; p += blockDim.x) {
        sum[p] = sv;
        mn[p] = v;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t prev_p[2] = {-1, -1};
      double prev_s[2] = {0.0, 0.0}, prev_m[2] = {0.0, 0.0};
      for (int l = 1; l <= log2cap; ++l) {
        int64_t cur_p[2] = {-1, -1};
        double cur_s[2] = {0.0, 0.0}, cur_m[2] = {0.0, 0.0};
        for (int side = 0; side < 2; ++side) {
          const int64_t p = side ? (H - 1) >> l : L >> l;
          if (interior(p, l) || (side == 1 && p == cur_p[0])) continue;
          double cs[2], cm[2];
          for (int ch = 0; ch < 2; ++ch) {
            const int64_t c = 2 * p + ch;
            if (interior(c, l - 1)) {
              cs[ch] = ldexp(v, l - 1);
              cm[ch] = v;
            } else if (c == prev_p[0]) {
              cs[ch] = prev_s[0];
              cm[ch] = prev_m[0];
            } else if (c == prev_p[1]) {
              cs[ch] = prev_s[1];
              cm[ch] = prev_m[1];
            } else {   // untouched: prefetched
              const int it = 4 * (l - 1) + 2 * side + ch;
              cs[ch] = pre_s[it];
              cm[ch] = pre_m[it];
            }
          }
          cur_p[side] = p;
          cur_s[side] = cs[0] + cs[1];
          cur_m[side] = py_min(cm[0], cm[1]);
          sum[p] = cur_s[side];
          mn[p] = cur_m[side];
        }
        for (int q = 0; q < 2; ++q) {
          prev_p[q] = cur_p[q];
          prev_s[q] = cur_s[q];
          prev_m[q] = cur_m[q];
        }
      }
    }
    return;
  }
  int64_t lo[2], hi[2];
  lo[0] = cap + next;
  hi[0] = cap + (end < size ? end : size);
  lo[1] = cap;
  hi[1] = cap + (end > size ? end - size : 0);
  for (int r = 0; r < 2; ++r)
    for (int64_t i = lo[r] + threadIdx.x; i < hi[r]; i += blockDim.x) {
      sum[i] = v;
      mn[i] = v;
    }
  for (int l = 0; l < log2cap; ++l) {
    __syncthreads();
    for (int r = 0; r < 2; ++r) {
      if (hi[r] <= lo[r]) continue;
      lo[r] >>= 1;
      hi[r] = ((hi[r] - 1) >> 1) + 1;
      for (int64_t i = lo[r] + threadIdx.x; i < hi[r]; i += blockDim.x) recompute(sum, mn, i);
    }
  }
}

__device__ double block_max(double v, double* scratch) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  const int w = threadIdx.x / 64, nw = blockDim.x / 64;
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = scratch[0];
    for (int i = 1; i < nw; ++i) r = fmax(r, scratch[i]);
    scratch[0] = r;
  }
  __syncthreads();
  return scratch[0];
}

// the priorities of an update: given (dt_per_update), or |td| + eps from the
// trainer's float32 TD errors (dt_per_update_td: the loop's abs -> float64 ->
// + eps in one pass, the same values)
struct PrioD {
  const double* p;
  __device__ double operator[](int i) const { return p[i]; }
};
struct PrioTd {
  const float* td;
  double eps;
  __device__ double operator[](int i) const { return (double)fabsf(td[i]) + eps; }
};

constexpr int kUpdMax = 128;        // entries of the LDS ancestor walk
constexpr int kUpdMaxLevels = 24;   // tree levels of the LDS ancestor walk

template <class P>
__global__ void __launch_bounds__(kTreeThreads)
update_kernel(double* sum, double* mn, double* maxp, int32_t* winner, int32_t* err, int64_t cap,
              int log2cap, int64_t len, int32_t n, const int64_t* idx, P prio, double alpha) {
  __shared__ double scratch[kTreeThreads / 64];
  double pmax = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t j = idx[i];
    const double p = prio[i];
    const bool ok_p = p > 0.0;  // false for NaN too
    const bool ok_i = j >= 0 && j < len;
    if (!ok_p) atomicOr(err, 1);
    if (!ok_i) atomicOr(err, 2);
    if (!ok_p || !ok_i) atomicAdd(err + 1, 1);   // counted, reported by dt_per_check
    if (ok_p && ok_i) {
      atomicMax(&winner[j], i);  // the sequential loop's last write wins
      pmax = fmax(pmax, p);
    }
  }
  pmax = block_max(pmax, scratch);  // also the barrier after the atomics
  if (threadIdx.x == 0 && pmax > *maxp) *maxp = pmax;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t j = idx[i];
    if (j >= 0 && j < len && prio[i] > 0.0 && winner[j] == i) {
      const double v = pow(prio[i], alpha);
      sum[cap + j] = v;
      mn[cap + j] = v;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t j = idx[i];
    if (j >= 0 && j < len) winner[j] = -1;
  }
  if (n <= kUpdMax && log2cap <= kUpdMaxLevels) {
    // Every written leaf's ancestors as one chain per entry, computed in LDS:
    // at level l, entry i's node has one child on its own chain and a
    // sibling that is either on some entry's chain (its value from LDS) or
    // untouched by this call -- those are loaded for every level at once
    // first, so the walk to the root is LDS-speed instead of a memory
    // round trip a level.  The same operands as recomputing level by level.
    __shared__ double pre_s[kUpdMaxLevels][kUpdMax], pre_m[kUpdMaxLevels][kUpdMax];
    __shared__ int16_t from[kUpdMaxLevels][kUpdMax];
    __shared__ double vs[2][kUpdMax], vm[2][kUpdMax];
    __shared__ int64_t leaf[kUpdMax];   // cap + j, or -1 for a rejected entry
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int64_t j = idx[i];
      leaf[i] = (j >= 0 && j < len && prio[i] > 0.0) ? cap + j : -1;
    }
    __syncthreads();
    for (int it = threadIdx.x; it < n * log2cap; it += blockDim.x) {
      const int i = it % n, l = it / n + 1;
      if (leaf[i] < 0) continue;
      const int64_t sib = (leaf[i] >> (l - 1)) ^ 1;
      int k = -1;
      for (int q = 0; q < n; ++q)
        if (leaf[q] >= 0 && (leaf[q] >> (l - 1)) == sib) {
          k = q;
          break;
        }
      from[l - 1][i] = (int16_t)k;
      if (k < 0) {
        pre_s[l - 1][i] = sum[sib];
        pre_m[l - 1][i] = mn[sib];
      }
    }
    for (int i = threadIdx.x; i < n; i += blockDim.x)
      if (leaf[i] >= 0) {
        vs[0][i] = sum[leaf[i]];   // the winner's leaf (written above)
        vm[0][i] = mn[leaf[i]];
      }
    __syncthreads();
    for (int l = 1; l <= log2cap; ++l) {
      const int a = (l - 1) & 1, b = l & 1;
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (leaf[i] < 0) continue;
        const int k = from[l - 1][i];
        const double os = vs[a][i], om = vm[a][i];
        const double ss = k >= 0 ? vs[a][k] : pre_s[l - 1][i];
        const double sm = k >= 0 ? vm[a][k] : pre_m[l - 1][i];
        const bool left = ((leaf[i] >> (l - 1)) & 1) == 0;
        const double ns = left ? os + ss : ss + os;
        const double nm = left ? py_min(om, sm) : py_min(sm, om);
        vs[b][i] = ns;
        vm[b][i] = nm;
        const int64_t node = leaf[i] >> l;
        sum[node] = ns;
        mn[node] = nm;
      }
      __syncthreads();
    }
    return;
  }
  // the ancestors of every written leaf, level by level; a node shared by
  // several leaves is recomputed redundantly to the same value
  for (int l = 1; l <= log2cap; ++l) {
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int64_t j = idx[i];
      if (j >= 0 && j < len && prio[i] > 0.0) recompute(sum, mn, (cap + j) >> l);
    }
  }
}

// reduce(0, len - 1) of segment_tree.py:37-74 for the sum tree: the recursion
// with start == node_start peels exact left children, combined right-nested:
// a1 + (a2 + (... + ak)).
// The node addresses depend only on `end` (cap a power of two: at depth d the
// path's node covers 2^(lg - d) leaves; `end` is its last leaf -> take it and
// stop; `end` in its right half -> take its left child), so every load is
// issued before the first is used: one memory latency, not one a level, and
// the same values summed in the same order.
__device__ double prefix_range_sum(const double* sum, int64_t cap, int64_t end) {
  const int lg = 63 - __builtin_clzll((unsigned long long)cap);
  double vals[kMaxDepth];
  bool on[kMaxDepth];
  bool done = false;
#pragma unroll
  for (int d = 0; d < kMaxDepth; ++d) {
    const int rem = lg - d;
    bool take = false;
    int64_t at = 0;
    if (!done && rem >= 0) {
      const int64_t node = (cap + end) >> rem;
      const int64_t ones = (int64_t(1) << rem) - 1;
      if ((end & ones) == ones) {
        take = true;
        at = node;
        done = true;
      } else if ((end >> (rem - 1)) & 1) {
        take = true;
        at = 2 * node;
      }
    }
    on[d] = take;
    vals[d] = take ? sum[at] : 0.0;
  }
  double acc = 0.0;
  bool first = true;
#pragma unroll
  for (int d = kMaxDepth - 1; d >= 0; --d)
    if (on[d]) {
      acc = first ? vals[d] : vals[d] + acc;
      first = false;
    }
  return acc;
}

// The top levels of the sum tree (nodes [1, kTopNodes)) are staged in LDS by
// the whole workgroup, all loads in flight at once, while thread 0 forms the
// range sum; the descent then walks those levels in LDS and only the deeper
// ones in global memory (segment_tree.py:125-131's comparisons and order).
constexpr int kTopNodes = 2048;

__global__ void __launch_bounds__(kSampleThreads)
sample_kernel(const double* sum, const double* mn, int64_t cap, int64_t len, int32_t batch,
              const double* u, double beta, int64_t* idx_out, double* w_out) {
  __shared__ double s_range, s_total, s_maxw;
  __shared__ double s_top[kTopNodes];
  const int64_t top = 2 * cap < kTopNodes ? 2 * cap : kTopNodes;
  {
    constexpr int kPer = kTopNodes / kSampleThreads;
    double v[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int64_t nd = threadIdx.x + q * kSampleThreads;
      v[q] = nd >= 1 && nd < top ? sum[nd] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) s_top[threadIdx.x + q * kSampleThreads] = v[q];
  }
  if (threadIdx.x == 0) {
    const double total = sum[1], mn1 = mn[1];
    s_range = prefix_range_sum(sum, cap, len - 2);
    s_total = total;
    const double p_min = mn1 / total;                               // buffers.py:226
    s_maxw = pow(p_min * (double)len, -beta);                      // :227
  }
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  double mass = u[i] * s_range;                                    // :180
  int64_t node = 1;
  while (node < cap) {                                             // segment_tree.py:125-131
    const double l = 2 * node < top ? s_top[2 * node] : sum[2 * node];
    if (l > mass) {
      node = 2 * node;
    } else {
      mass -= l;
      node = 2 * node + 1;
    }
  }
  const int64_t j = node - cap;
  idx_out[i] = j;
  const double p_sample = sum[node] / s_total;                     // :230
  w_out[i] = pow(p_sample * (double)len, -beta) / s_maxw;          // :231-232
}

// Frame store (aido1_amd/replay.py, ReplayBuffer frame_envs): one workgroup
// per env copies the env's newest frame (`frame4` float4s at src + e *
// src_stride4, the rollout ring's newest slot) into frame row base_row + e,
// and its lane 0 advances the env's stack of frame rows: the transition's obs
// is the stack before, its next_obs the stack after -- the older rows shifted
// left and the new row appended, or every entry the new row where `done`
// marks a respawned env (the renderer refilled every slot of its stack).
constexpr int kFrameThreads = 256;

// dt_frame_gather: block (x, b) covers pixels [x * threads, ...) of sample b;
// a thread reads its pixel from the k frames of obs and of next_obs (each
// plane read coalesced) and writes the k-float NHWC pixel of each
template <typename F>
__device__ __forceinline__ float frame_px(const F* frames, int64_t i) {
  if constexpr (sizeof(F) == 1)
    return dr::kPalGray[frames[i] & 7u];
  else
    return frames[i];
}

template <typename F>
__global__ void __launch_bounds__(kFrameThreads)
frame_gather_kernel(const int64_t* __restrict__ idx, const F* __restrict__ frames, int64_t hw,
                    int k, const int32_t* __restrict__ obs_ptr,
                    const int32_t* __restrict__ next_ptr, const float* __restrict__ action,
                    const double* __restrict__ reward, const uint8_t* __restrict__ done,
                    float* __restrict__ obs, float* __restrict__ nxt, float* __restrict__ act,
                    float* __restrict__ rew, float* __restrict__ notdone) {
  const int b = blockIdx.y;
  const int64_t i = idx[b];
  const int64_t px = (int64_t)blockIdx.x * kFrameThreads + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x < 2) act[2 * b + threadIdx.x] = action[2 * i + threadIdx.x];
  if (blockIdx.x == 0 && threadIdx.x == 2) rew[b] = (float)reward[i];
  if (blockIdx.x == 0 && threadIdx.x == 3) notdone[b] = done[i] ? 0.0f : 1.0f;
  if (px >= hw) return;
  float* o = obs + ((int64_t)b * hw + px) * k;
  float* q = nxt + ((int64_t)b * hw + px) * k;
  for (int c = 0; c < k; ++c) {
    o[c] = frame_px(frames, (int64_t)obs_ptr[i * k + c] * hw + px);
    q[c] = frame_px(frames, (int64_t)next_ptr[i * k + c] * hw + px);
  }
}

__global__ void __launch_bounds__(kFrameThreads)
frame_add_kernel(int64_t frame4, const float4* __restrict__ src, int64_t src_stride4,
                 float4* __restrict__ dst, int k, int32_t* __restrict__ stack,
                 const uint8_t* __restrict__ done, int32_t base_row, int32_t* __restrict__ obs_ptr,
                 int32_t* __restrict__ next_ptr) {
  const int e = blockIdx.x;
  const float4* s = src + (size_t)e * src_stride4;
  float4* d = dst + (size_t)e * frame4;
#pragma unroll 4
  for (int64_t i = threadIdx.x; i < frame4; i += kFrameThreads) d[i] = s[i];
  if (threadIdx.x == 0) {
    const int32_t row = base_row + e;
    const bool fresh = done != nullptr && done[e] != 0;
    int32_t* st = stack + (size_t)e * k;
    int32_t* op = obs_ptr + (size_t)e * k;
    int32_t* np = next_ptr + (size_t)e * k;
    for (int j = 0; j < k; ++j) op[j] = st[j];
    for (int j = 0; j + 1 < k; ++j) {
      const int32_t v = fresh ? row : st[j + 1];
      np[j] = v;
      st[j] = v;
    }
    np[k - 1] = row;
    st[k - 1] = row;
  }
}

#define PER_HIP(h, expr)                                                       \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      (h)->msg = std::string(#expr) + ": " + hipGetErrorString(_e);             \
      return DT_E_HIP;                                                         \
    }                                                                          \
  } while (0)

std::string g_per_create_err;

}  // namespace

extern "C" {

int dt_per_create(int64_t size, double alpha, int32_t device, dt_per** out) {
  g_per_create_err.clear();
  if (!out || size < 1 || !(alpha > 0.0) || size > (int64_t(1) << 31)) {
    g_per_create_err = "dt_per_create: need 1 <= size <= 2^31 and alpha > 0";
    return DT_E_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    g_per_create_err = "dt_per_create: no HIP device " + std::to_string(device);
    return DT_E_NODEV;
  }
  dt_per* h = new dt_per();
  h->device = device;
  h->size = size;
  h->alpha = alpha;
  h->cap = 1;
  while (h->cap < size) {
    h->cap *= 2;
    ++h->log2cap;
  }
  const size_t tb = (size_t)(2 * h->cap) * sizeof(double);
  const size_t wb = (((size_t)h->cap * 4) + 255) & ~size_t(255);
  if (hipSetDevice(device) != hipSuccess || hipMalloc(&h->buf, 2 * tb + wb + 256) != hipSuccess) {
    g_per_create_err = "dt_per_create: hipMalloc failed";
    delete h;
    return DT_E_HIP;
  }
  char* b = (char*)h->buf;
  h->sum = (double*)b;
  h->mn = (double*)(b + tb);
  h->winner = (int32_t*)(b + 2 * tb);
  h->maxp = (double*)(b + 2 * tb + wb);
  h->err = (int32_t*)(b + 2 * tb + wb + 64);
  const int grid = (int)std::min<int64_t>((2 * h->cap + 255) / 256, 4096);
  fill_kernel<<<grid, 256>>>(h->sum, h->mn, h->maxp, h->winner, h->cap);
  if (hipMemset(h->err, 0, 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    g_per_create_err = "dt_per_create: init failed";
    (void)hipFree(h->buf);
    delete h;
    return DT_E_HIP;
  }
  *out = h;
  return DT_OK;
}

void dt_per_destroy(dt_per* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipFree(h->buf);
  delete h;
}

const char* dt_per_last_error(const dt_per* h) { return h ? h->msg.c_str() : g_per_create_err.c_str(); }
int64_t dt_per_capacity(const dt_per* h) { return h ? h->cap : -1; }
int64_t dt_per_len(const dt_per* h) { return h ? h->len : -1; }
int64_t dt_per_next_idx(const dt_per* h) { return h ? h->next : -1; }

int dt_per_add(dt_per* h, int64_t n, int64_t* slots_dev, void* stream) {
  if (!h || n < 0) return DT_E_ARG;
  if (n == 0) return DT_OK;
  PER_HIP(h, hipSetDevice(h->device));
  add_kernel<<<1, kTreeThreads, 0, (hipStream_t)stream>>>(h->sum, h->mn, h->maxp, h->cap, h->log2cap,
                                                          h->size, h->next, n, h->alpha, slots_dev);
  PER_HIP(h, hipGetLastError());
  h->next = (h->next + n) % h->size;
  h->len = std::min(h->len + n, h->size);
  return DT_OK;
}

int dt_per_sample(dt_per* h, int32_t batch, const double* u_dev, double beta, int64_t* idx_dev,
                  double* weights_dev, void* stream) {
  if (!h || batch < 0 || !(beta > 0.0) || (batch > 0 && (!u_dev || !idx_dev || !weights_dev))) {
    if (h) h->msg = "dt_per_sample: bad argument (beta must be > 0)";
    return DT_E_ARG;
  }
  if (h->len < 2) {
    h->msg = "dt_per_sample: need at least 2 stored transitions";
    return DT_E_ARG;
  }
  if (batch == 0) return DT_OK;
  PER_HIP(h, hipSetDevice(h->device));
  const int grid = (batch + kSampleThreads - 1) / kSampleThreads;
  sample_kernel<<<grid, kSampleThreads, 0, (hipStream_t)stream>>>(h->sum, h->mn, h->cap, h->len,
                                                                  batch, u_dev, beta, idx_dev,
                                                                  weights_dev);
  PER_HIP(h, hipGetLastError());
  return DT_OK;
}

int dt_per_update(dt_per* h, int32_t n, const int64_t* idx_dev, const double* priorities_dev,
                  void* stream) {
  if (!h || n < 0 || (n > 0 && (!idx_dev || !priorities_dev))) return DT_E_ARG;
  if (n == 0) return DT_OK;
  PER_HIP(h, hipSetDevice(h->device));
  update_kernel<<<1, kTreeThreads, 0, (hipStream_t)stream>>>(
      h->sum, h->mn, h->maxp, h->winner, h->err, h->cap, h->log2cap, h->len, n, idx_dev,
      PrioD{priorities_dev}, h->alpha);
  PER_HIP(h, hipGetLastError());
  return DT_OK;
}

int dt_per_update_td(dt_per* h, int32_t n, const int64_t* idx_dev, const float* td_dev,
                     double eps, void* stream) {
  if (!h || n < 0 || (n > 0 && (!idx_dev || !td_dev))) return DT_E_ARG;
  if (n == 0) return DT_OK;
  PER_HIP(h, hipSetDevice(h->device));
  update_kernel<<<1, kTreeThreads, 0, (hipStream_t)stream>>>(
      h->sum, h->mn, h->maxp, h->winner, h->err, h->cap, h->log2cap, h->len, n, idx_dev,
      PrioTd{td_dev, eps}, h->alpha);
  PER_HIP(h, hipGetLastError());
  return DT_OK;
}

int dt_per_read(dt_per* h, double* sum_dev, double* min_dev, double* max_priority_dev,
                void* stream) {
  if (!h) return DT_E_ARG;
  PER_HIP(h, hipSetDevice(h->device));
  const size_t tb = (size_t)(2 * h->cap) * sizeof(double);
  hipStream_t s = (hipStream_t)stream;
  if (sum_dev) PER_HIP(h, hipMemcpyAsync(sum_dev, h->sum, tb, hipMemcpyDeviceToDevice, s));
  if (min_dev) PER_HIP(h, hipMemcpyAsync(min_dev, h->mn, tb, hipMemcpyDeviceToDevice, s));
  if (max_priority_dev)
    PER_HIP(h, hipMemcpyAsync(max_priority_dev, h->maxp, 8, hipMemcpyDeviceToDevice, s));
  return DT_OK;
}

int dt_frame_add(int32_t n, int64_t frame_elems, const void* src, int64_t src_env_stride,
                 void* dst, int32_t k, int32_t* stack, const uint8_t* done, int32_t base_row,
                 int32_t* obs_ptr, int32_t* next_ptr, void* stream) {
  if (n < 0 || k < 1 || frame_elems < 4 || frame_elems % 4 || src_env_stride % 4) return DT_E_ARG;
  if (n == 0) return DT_OK;
  if (!src || !dst || !stack || !obs_ptr || !next_ptr || base_row < 0) return DT_E_ARG;
  if (((uintptr_t)src | (uintptr_t)dst) & 15) return DT_E_ARG;
  frame_add_kernel<<<n, kFrameThreads, 0, (hipStream_t)stream>>>(
      frame_elems / 4, reinterpret_cast<const float4*>(src), src_env_stride / 4,
      reinterpret_cast<float4*>(dst), k, stack, done, base_row, obs_ptr, next_ptr);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_frame_gather(int32_t batch, const int64_t* idx, const void* frames, int32_t frame_kind,
                    int64_t hw, int32_t k, const int32_t* obs_ptr, const int32_t* next_ptr,
                    const float* action, const double* reward, const uint8_t* done, float* obs,
                    float* nxt, float* act, float* rew, float* notdone, void* stream) {
  if (batch < 0 || hw < 1 || k < 1 || k > 4 || frame_kind < 0 || frame_kind > 1) return DT_E_ARG;
  if (batch == 0) return DT_OK;
  if (!idx || !frames || !obs_ptr || !next_ptr || !action || !reward || !done || !obs || !nxt ||
      !act || !rew || !notdone)
    return DT_E_ARG;
  const int64_t per = (hw + kFrameThreads - 1) / kFrameThreads;
  if (per > 65535) return DT_E_ARG;
  const dim3 grid((unsigned)per, (unsigned)batch);
  if (frame_kind == 1)
    frame_gather_kernel<<<grid, kFrameThreads, 0, (hipStream_t)stream>>>(
        idx, static_cast<const uint8_t*>(frames), hw, k, obs_ptr, next_ptr, action, reward, done,
        obs, nxt, act, rew, notdone);
  else
    frame_gather_kernel<<<grid, kFrameThreads, 0, (hipStream_t)stream>>>(
        idx, static_cast<const float*>(frames), hw, k, obs_ptr, next_ptr, action, reward, done,
        obs, nxt, act, rew, notdone);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_per_check(dt_per* h) {
  if (!h) return DT_E_ARG;
  PER_HIP(h, hipSetDevice(h->device));
  PER_HIP(h, hipDeviceSynchronize());
  int32_t e[2] = {0, 0};
  PER_HIP(h, hipMemcpy(e, h->err, 8, hipMemcpyDeviceToHost));
  if (!e[0]) return DT_OK;
  PER_HIP(h, hipMemset(h->err, 0, 8));
  h->msg = "update_priorities: ";
  if (e[0] & 1) h->msg += "priority must be > 0 (NaN included); ";
  if (e[0] & 2) h->msg += "index outside [0, len); ";
  h->msg += std::to_string(e[1]) + " offending entries were skipped";
  return DT_E_ARG;
}

}  // extern "C"
