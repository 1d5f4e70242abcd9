// The DDPG update's convolutions (include/dtupd.h): config.json's conv_2d
// layers of the actor and critic in f32, forward (x3: f32 operands as fp16
// hi / lo pairs on v_mfma_f32_32x32x16_f16, DTUPD_X3 below), weight gradient
// and input gradient (v_mfma_f32_32x32x2_f32), replacing MIOpen in the
// train-mode networks of training/trainers.py:143-237.
//
// Every layer is C_out = 32 and NHWC, so each pass is a GEMM whose N or M is
// the 32 channels:
//   forward  D[pixel][co]   = sum_k  X[pixel][k]   W[co][k]     (A = im2col row, B = W)
//   wgrad    D[co][k]       = sum_p  dZ[p][co]     X[p][k]      (A = dZ, B = im2col)
//   dgrad    D[pixel][ci]   = sum_t  dZ[o(t)][co]  W[co][ci]    (A = dZ, B = W^T)
// A 32x32x2 MFMA takes ONE f32 per lane for each operand (A[i = l & 31][k =
// l >> 5], B[k = l >> 5][j = l & 31]).  A lane loads a float4 of four
// consecutive k instead and feeds four MFMAs, element e to the e-th: the
// k-slot kk of MFMA e is the reduction index 8s + 4kk + e, the same for A
// and B, so the sum is the convolution's, in a different order.  Loads are
// then 16-B pieces of one pixel's channels (32 consecutive floats a pixel per
// half-wave: whole 128-B lines), and the weights sit in LDS.
//
// Geometry is compile-time (the four config.json layers at 120 x 160
// observations); the host entry points dispatch on (C_in, KS, ST, IH, IW).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/dttrain.h"
#include "../../include/dtupd.h"
#include "dtsync.h"

// tools/upd_micro.py builds variants that skip parts of the forward to time
// them (1: the A loads, 2: W's staging, 4: the statistics' merge, 8: the
// K-split sum, 16: the chain's partial loads, 32: the chain's merge); 0 in
// the library
#ifndef DTUPD_SKIP
#define DTUPD_SKIP 0
#endif
// input-gradient waves a workgroup per layer (tools/upd_micro.py variants)
// weight gradient: double-buffered row staging for conv2-4 (the x3 MFMAs
// left the row loads exposed: conv2 32.5 -> 27.9 us at batch 64) and conv1
// (tools/upd_micro.py variants)
#ifndef DTUPD_WG_DB
#define DTUPD_WG_DB 1
#endif
#ifndef DTUPD_WG_DB1
#define DTUPD_WG_DB1 0
#endif
// the forward's K slices (waves a tile) per layer (tools/upd_micro.py variants)
#ifndef DTUPD_KS1
#define DTUPD_KS1 2
#endif
#ifndef DTUPD_KS2
#define DTUPD_KS2 2
#endif
#ifndef DTUPD_KS3
#define DTUPD_KS3 8
#endif
#ifndef DTUPD_KS4
#define DTUPD_KS4 16
#endif
#ifndef DTUPD_DG2_NW
#define DTUPD_DG2_NW 8
#endif
#ifndef DTUPD_DG3_NW
#define DTUPD_DG3_NW 4
#endif
#ifndef DTUPD_DG4_NW
#define DTUPD_DG4_NW 4
#endif

namespace {

using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int CIN_, int KS_, int ST_, int IH_, int IW_>
struct Geom {
  static constexpr int CIN = CIN_, KS = KS_, ST = ST_, IH = IH_, IW = IW_;
  static constexpr int OH = (IH - KS) / ST + 1, OW = (IW - KS) / ST + 1;
  static constexpr int OPIX = OH * OW;
  static constexpr int K = KS * KS * CIN;          // reduction length (im2col row)
  static constexpr int KROW = KS * CIN;            // contiguous floats of one kernel row
  static constexpr int KSTEPS = K / 8;             // 8 k a float4 step (4 MFMAs)
  static constexpr int TPS = (OPIX + 31) / 32;     // 32-pixel tiles a sample
  static_assert(K % 8 == 0 && KROW % 4 == 0, "float4 steps stay inside a kernel row");
  // offset (floats) of reduction index k inside a pixel's patch
  __host__ __device__ static constexpr int koff(int k) { return (k / KROW) * IW * CIN + k % KROW; }
  // first float of output pixel p's patch in sample s
  __device__ static int xbase(int s, int p) {
    const int oy = p / OW, ox = p - oy * OW;
    return ((s * IH + oy * ST) * IW + ox * ST) * CIN;
  }
};

using L1 = Geom<3, 8, 2, 120, 160>;
using L2 = Geom<32, 4, 2, 57, 77>;
using L3 = Geom<32, 4, 2, 27, 37>;
using L4 = Geom<32, 4, 1, 12, 17>;

// four consecutive floats of a patch row (16-B aligned for C_in 32, 8-B for
// C_in 3: the row starts at 6 * ox floats)
template <int CIN>
__device__ __forceinline__ float4 ld4(const float* p) {
  if constexpr (CIN % 4 == 0) {
    return *reinterpret_cast<const float4*>(p);
  } else {
    const float2 a = *reinterpret_cast<const float2*>(p);
    const float2 b = *reinterpret_cast<const float2*>(p + 2);
    return make_float4(a.x, a.y, b.x, b.y);
  }
}

// The forward's x3 form (DTUPD_X3, the library default): each f32 operand
// as an fp16 pair hi = fp16(v), lo = fp16((v - hi) * 2^11), and a 16-k unit
// as three v_mfma_f32_32x32x16_f16 into two f32 accumulators,
//   acc0 += Xh Wh,   acc1 += Xh Wl + Xl Wh,   z = acc0 + acc1 / 2^11
// (the dropped Xl Wl and the split's rounding: ~2^-21 of each product, the
// actor's conv chain, csrc/dtconvx.hip), 3/16 of the f32 MFMA cycles.
// Operands past fp16's range (|v| >= 65520) become inf: the guard reports
// them.  0 keeps the f32 MFMA chain (tools/upd_micro.py variants).
#ifndef DTUPD_X3
#define DTUPD_X3 1
#endif
using half8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x2 = __attribute__((ext_vector_type(2))) float;
using f16x2 = __attribute__((ext_vector_type(2))) _Float16;
using u32x4v = __attribute__((ext_vector_type(4))) uint32_t;
constexpr float kLo = 2048.0f, kLoInv = 1.0f / 2048.0f;

__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  const f32x2 x = {a, b};
  const f16x2 h = __builtin_convertvector(x, f16x2);
  const f32x2 r = (x - __builtin_convertvector(h, f32x2)) * kLo;
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, f16x2));
}
// eight consecutive k (two float4s) -> their hi and lo fragments
__device__ __forceinline__ void split8(float4 a, float4 b, half8& h, half8& l) {
  uint32_t uh[4], ul[4];
  split2(a.x, a.y, uh[0], ul[0]);
  split2(a.z, a.w, uh[1], ul[1]);
  split2(b.x, b.y, uh[2], ul[2]);
  split2(b.z, b.w, uh[3], ul[3]);
  h = __builtin_bit_cast(half8, u32x4v{uh[0], uh[1], uh[2], uh[3]});
  l = __builtin_bit_cast(half8, u32x4v{ul[0], ul[1], ul[2], ul[3]});
}

// four values as (hi, lo) words: hi in the low half
__device__ __forceinline__ uint4 hl4(float4 v) {
  uint32_t h0, l0, h1, l1;
  split2(v.x, v.y, h0, l0);
  split2(v.z, v.w, h1, l1);
  return make_uint4((h0 & 0xffffu) | (l0 << 16), (h0 >> 16) | (l0 & 0xffff0000u),
                    (h1 & 0xffffu) | (l1 << 16), (h1 >> 16) | (l1 & 0xffff0000u));
}
// eight (hi, lo) words -> the hi and lo fragments
__device__ __forceinline__ void hl_frag(const uint32_t (&w)[8], half8& h, half8& l) {
  u32x4v uh, ul;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t a = w[2 * i], b = w[2 * i + 1];
    uh[i] = (a & 0xffffu) | (b << 16);
    ul[i] = (a >> 16) | (b & 0xffff0000u);
  }
  h = __builtin_bit_cast(half8, uh);
  l = __builtin_bit_cast(half8, ul);
}

__device__ __forceinline__ f32x16 mfma4(float4 a, float4 b, f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, c, 0, 0, 0);
  return c;
}

// row of the 32x32 accumulator register r holds for lane half h
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }


// The train-mode BatchNorm after a block's conv -> LeakyReLU, fused into the
// forward's epilogue (STATS): the batch statistics of a = leaky(z + bias).
// A lane's accumulator column is one output channel for every tile, so each
// lane keeps a Welford (count, mean, M2) of its channel across its tiles
// (each tile two-pass over its <= 16 rows, Chan-merged in); at the end the
// lane pairs and the waves merge, each workgroup writes its partial through
// to memory, and the last to arrive merges them all (dtsync.h), writes
// mean / invstd and moves the running statistics `updates` times, as
// dt_bn_leaky_fwd does.
struct FwdBn {
  const float* bias;
  float slope, eps, momentum;
  float* running_mean;
  float* running_var;
  int64_t* nbt;
  int updates;
  float* mean_invstd;
  float* work;     // [kMaxGrid][32][3] partials, then the counters (dt_upd_bn_work_floats)
  int32_t* guard;
};
constexpr int kMaxGrid = 256;   // workgroups (= partials) of a STATS launch

// ---- cross-workgroup statistics ----------------------------------------------------------
// A launch's BatchNorm statistics travel as per-workgroup partials laid out
// [workgroup][3][32] (count, mean, M2 of the 32 channels), merged with Chan's
// rule (dtsync.h) in trees of cross-lane shuffles rather than long serial
// chains, always in the same order: every merger of the same partials (the
// last workgroup of dt_upd_conv_fwd_bn, or each workgroup of the chain's
// next kernel) gets the same bits.  All for 1024-thread workgroups.
struct Welford {
  float n, mean, m2;
};
__device__ __forceinline__ void chan(Welford& a, const Welford& b) { chan(a.n, a.mean, a.m2, b.n, b.mean, b.m2); }
__device__ __forceinline__ Welford shfl_xor_w(const Welford& a, int m) {
  return Welford{__shfl_xor(a.n, m), __shfl_xor(a.mean, m), __shfl_xor(a.m2, m)};
}

// red[16][32]: 16 ways a channel -> the channel's merge in the threads t < 512
// with (t & 15) == 0 (channel t >> 4); no barrier after
__device__ __forceinline__ Welford merge16(const Welford (*red)[32]) {
  const int t = threadIdx.x;
  Welford w{0.0f, 0.0f, 0.0f};
  if (t < 512) {   // waves 0-7 whole
    w = red[t & 15][t >> 4];
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) chan(w, shfl_xor_w(w, m));
  }
  return w;
}
__device__ __forceinline__ bool merge16_owner() { return threadIdx.x < 512 && (threadIdx.x & 15) == 0; }

// the workgroup's partial of its lanes' channels (lane & 31) -> part[blockIdx.x]:
// written through (WT) for a last-arrival merge inside this launch, plainly
// for the next kernel (the chain of include/dtupd.h) to merge
template <int NT, bool WT>
__device__ void wg_partial(float* part, float cnt, float mean, float m2) {
  static_assert(NT == 1024, "16 waves");
  __shared__ Welford red[16][32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  Welford own{cnt, mean, m2};
  chan(own, shfl_xor_w(own, 32));            // lane pairs (l, l ^ 32) hold the same channel
  if (lane < 32) red[wave][lane] = own;
  __syncthreads();
  const Welford w = merge16(red);
  if (merge16_owner()) {
    const int ch = tid >> 4;
    float* p = part + (size_t)blockIdx.x * 96 + ch;
    if constexpr (WT) {
      st_wt(p, w.n);
      st_wt(p + 32, w.mean);
      st_wt(p + 64, w.m2);
    } else {
      p[0] = w.n;
      p[32] = w.mean;
      p[64] = w.m2;
    }
  }
}

// Merging `parts` partials: thread t takes channels 4 (t & 7) .. + 3 of
// partials (t >> 3) and (t >> 3) + 128 (loaded as float4s: PartLoads),
// then the lanes of a wave merge by shuffles, the waves through LDS (merge16).
constexpr int kPartHalf = 128;
static_assert(kMaxGrid <= 2 * kPartHalf, "two partials a thread");
struct PartLoads {
  float4 n[2], mean[2], m2[2];
};

template <bool WT>
__device__ __forceinline__ PartLoads part_loads(const float* part, int parts) {
  PartLoads r;
  const int t = threadIdx.x, qd = t & 7, gi = t >> 3;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int g = gi + kPartHalf * h;
    const float* p = part + (size_t)(g < parts ? g : 0) * 96 + 4 * qd;
    if constexpr (WT) {
      r.n[h] = make_float4(ld_wt(p), ld_wt(p + 1), ld_wt(p + 2), ld_wt(p + 3));
      r.mean[h] = make_float4(ld_wt(p + 32), ld_wt(p + 33), ld_wt(p + 34), ld_wt(p + 35));
      r.m2[h] = make_float4(ld_wt(p + 64), ld_wt(p + 65), ld_wt(p + 66), ld_wt(p + 67));
    } else {
      r.n[h] = *reinterpret_cast<const float4*>(p);
      r.mean[h] = *reinterpret_cast<const float4*>(p + 32);
      r.m2[h] = *reinterpret_cast<const float4*>(p + 64);
    }
    if (g >= parts) r.n[h] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // merges as nothing
  }
  return r;
}

// -> the merge of every partial, valid in merge16_owner() threads (channel t >> 4)
__device__ __forceinline__ Welford merge_parts(const PartLoads& r) {
  __shared__ Welford red[16][32];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, qd = t & 7;
  Welford s[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float n4[4] = {r.n[h].x, r.n[h].y, r.n[h].z, r.n[h].w};
    const float m4[4] = {r.mean[h].x, r.mean[h].y, r.mean[h].z, r.mean[h].w};
    const float q4[4] = {r.m2[h].x, r.m2[h].y, r.m2[h].z, r.m2[h].w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (h == 0) s[c] = Welford{n4[c], m4[c], q4[c]};
      else chan(s[c], Welford{n4[c], m4[c], q4[c]});
    }
  }
#pragma unroll
  for (int m = 8; m < 64; m <<= 1)          // the wave's eight partial pairs a quad
#pragma unroll
    for (int c = 0; c < 4; ++c) chan(s[c], shfl_xor_w(s[c], m));
  if (lane < 8)
#pragma unroll
    for (int c = 0; c < 4; ++c) red[wave][4 * qd + c] = s[c];
  __syncthreads();
  return merge16(red);
}

template <int NT>
__device__ void merge_partials_last(const FwdBn& fb, float cnt, float mean, float m2, int64_t m) {
  static_assert(NT == 1024, "16 waves");
  const int tid = threadIdx.x;
  float* part = fb.work;
  wg_partial<NT, true>(part, cnt, mean, m2);
  unsigned int* counters = reinterpret_cast<unsigned int*>(part + (size_t)kMaxGrid * 96);
  if (!last_arrival(&counters[0])) return;
  acquire_partials();
  const PartLoads r = part_loads<true>(part, gridDim.x);
  {   // counts back to zero (dtsync.h): a partial read stale shows as a lost count
    const int qd = tid & 7, gi = tid >> 3;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int g = gi + kPartHalf * h;
      if (g < (int)gridDim.x)
#pragma unroll
        for (int c = 0; c < 4; ++c) st_wt(part + (size_t)g * 96 + 4 * qd + c, 0.0f);
    }
  }
  float rm = 0.0f, rv = 0.0f;
  if (merge16_owner()) {
    rm = fb.running_mean[tid >> 4];
    rv = fb.running_var[tid >> 4];
  }
  const Welford w = merge_parts(r);
  if (merge16_owner()) {
    const int ch = tid >> 4;
    const float var = w.m2 / w.n;
    const float invstd = 1.0f / sqrtf(var + fb.eps);
    fb.mean_invstd[ch] = w.mean;
    fb.mean_invstd[32 + ch] = invstd;
    const float cn = w.n;
    const bool lost = m < (int64_t(1) << 24) ? cn != (float)m : fabsf(cn - (float)m) > 1e-6f * (float)m;
    guard_raise(fb.guard, DT_GUARD_BN_COUNT, lost);
    guard_raise(fb.guard, DT_GUARD_BN_FWD, !finitef(w.mean) || !finitef(invstd));
    const float unbiased = cn > 1.0f ? w.m2 / (cn - 1.0f) : var;
    for (int u = 0; u < fb.updates; ++u) {
      rm = (1.0f - fb.momentum) * rm + fb.momentum * w.mean;
      rv = (1.0f - fb.momentum) * rv + fb.momentum * unbiased;
    }
    fb.running_mean[ch] = rm;
    fb.running_var[ch] = rv;
    if (ch == 0 && fb.nbt) fb.nbt[0] += fb.updates;
  }
}

// ---- the chain's hand-off (include/dtupd.h DtUpdBn) -------------------------------------
// y = bn(leaky(z + bias)) exactly as dt_bn_leaky_apply computes it
__device__ __forceinline__ float norm1(float z, float b, float mu, float sc, float bt, float slope) {
  float v = z + b;
  v = v > 0.0f ? v : v * slope;
  return (v - mu) * sc + bt;
}
__device__ __forceinline__ float4 norm4(float4 z, float4 b, float4 mu, float4 sc, float4 bt,
                                        float slope) {
  return make_float4(norm1(z.x, b.x, mu.x, sc.x, bt.x, slope), norm1(z.y, b.y, mu.y, sc.y, bt.y, slope),
                     norm1(z.z, b.z, mu.z, sc.z, bt.z, slope), norm1(z.w, b.w, mu.w, sc.w, bt.w, slope));
}

// Every workgroup of a chain kernel merges the producer's partials itself
// (merge_parts: the same order as dt_upd_conv_fwd_bn's last workgroup), so
// all agree bit for bit, and builds tab = {bias, mean, invstd * gamma, beta}
// per channel in LDS.  The first workgroup (`finalize`) also writes
// mean_invstd, moves the running statistics and reports to the guard, as the
// merging workgroup of dt_upd_conv_fwd_bn does.  Two halves: norm_loads
// issues every load (partials, parameters, running statistics) so the caller
// can start its own loads behind them; norm_build merges and fills tab.
struct NormRegs {
  PartLoads p;
  float bias, gamma, beta, rm, rv;
};

template <int NT>
__device__ __forceinline__ NormRegs norm_loads(const DtUpdBn& b, bool finalize) {
  static_assert(NT == 1024, "16 waves");
  NormRegs r;
  if (DTUPD_SKIP & 16) {
    r.p.n[0] = r.p.n[1] = r.p.mean[0] = r.p.mean[1] = r.p.m2[0] = r.p.m2[1] =
        make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  } else {
    r.p = part_loads<false>(b.part, b.parts);
  }
  r.bias = r.gamma = r.beta = r.rm = r.rv = 0.0f;
  if (merge16_owner()) {
    const int ch = threadIdx.x >> 4;
    r.bias = b.bias[ch];
    r.gamma = b.gamma[ch];
    r.beta = b.beta[ch];
    if (finalize) {
      r.rm = b.running_mean[ch];
      r.rv = b.running_var[ch];
    }
  }
  return r;
}

template <int NT>
__device__ void norm_build(const DtUpdBn& b, const NormRegs& r, float (*tab)[32], bool finalize) {
  const int tid = threadIdx.x;
  if (DTUPD_SKIP & 32) {
    if (tid < 32) {
      tab[0][tid] = 0.1f;
      tab[1][tid] = 0.5f;
      tab[2][tid] = 1.5f;
      tab[3][tid] = 0.2f;
    }
    __syncthreads();
    return;
  }
  const Welford w = merge_parts(r.p);
  if (merge16_owner()) {
    const int ch = tid >> 4;
    const float cn = w.n, cm = w.mean, cq = w.m2;
    const float var = cq / cn;
    const float invstd = 1.0f / sqrtf(var + b.eps);
    tab[0][ch] = r.bias;
    tab[1][ch] = cm;
    tab[2][ch] = invstd * r.gamma;
    tab[3][ch] = r.beta;
    if (finalize) {
      b.mean_invstd[ch] = cm;
      b.mean_invstd[32 + ch] = invstd;
      const int64_t m = b.m;
      const bool lost = m < (int64_t(1) << 24) ? cn != (float)m : fabsf(cn - (float)m) > 1e-6f * (float)m;
      guard_raise(b.guard, DT_GUARD_BN_COUNT, lost);
      guard_raise(b.guard, DT_GUARD_BN_FWD, !finitef(cm) || !finitef(invstd));
      const float unbiased = cn > 1.0f ? cq / (cn - 1.0f) : var;
      float rm = r.rm, rv = r.rv;
      for (int u = 0; u < b.updates; ++u) {
        rm = (1.0f - b.momentum) * rm + b.momentum * cm;
        rv = (1.0f - b.momentum) * rv + b.momentum * unbiased;
      }
      b.running_mean[ch] = rm;
      b.running_var[ch] = rv;
      if (ch == 0 && b.num_batches_tracked) b.num_batches_tracked[0] += b.updates;
    }
  }
  __syncthreads();
}

// y = bn(leaky(z + bias)) of the chain's last block: every workgroup merges the
// partials (norm_loads / norm_build) and normalises its share of z
constexpr int kFinishPer = 4;       // float4s a thread
constexpr int kFinishMaxGrid = 1024;

__global__ void __launch_bounds__(1024)
bn_finish_kernel(int64_t m, int hw, const float* __restrict__ z, DtUpdBn b, float* __restrict__ y) {
  __shared__ __attribute__((aligned(16))) float tab[4][32];
  const bool fin = blockIdx.x == 0;
  const NormRegs r = norm_loads<1024>(b, fin);
  // this thread's z (at most kFinishPer float4s: the grid covers m) loaded
  // while the partials merge
  const int64_t items = m * 8, stride = (int64_t)gridDim.x * 1024;
  const int64_t q0 = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  float4 v[kFinishPer];
#pragma unroll
  for (int k = 0; k < kFinishPer; ++k) {
    const int64_t q = q0 + k * stride;
    v[k] = q < items ? reinterpret_cast<const float4*>(z)[q] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  norm_build<1024>(b, r, tab, fin);
  const int cg = threadIdx.x & 7;               // the grid stride is a multiple of 8
  const float4 tb = reinterpret_cast<const float4*>(tab[0])[cg];
  const float4 tm = reinterpret_cast<const float4*>(tab[1])[cg];
  const float4 ts = reinterpret_cast<const float4*>(tab[2])[cg];
  const float4 tt = reinterpret_cast<const float4*>(tab[3])[cg];
  // y as z (hw == 0) or NCHW with hw pixels a sample (the flatten that
  // follows the trunk is then a view)
  auto put = [&](int64_t q, float4 o) __attribute__((always_inline)) {
    if (hw == 0) {
      reinterpret_cast<float4*>(y)[q] = o;
    } else {
      const int64_t pix = q >> 3, smp = pix / hw;
      float* d = y + (smp * 32 + 4 * cg) * hw + (pix - smp * hw);
      d[0] = o.x;
      d[hw] = o.y;
      d[2 * hw] = o.z;
      d[3 * hw] = o.w;
    }
  };
#pragma unroll
  for (int k = 0; k < kFinishPer; ++k) {
    const int64_t q = q0 + k * stride;
    if (q < items) put(q, norm4(v[k], tb, tm, ts, tt, b.slope));
  }
  for (int64_t q = q0 + kFinishPer * stride; q < items; q += stride)   // past the grid's cover
    put(q, norm4(reinterpret_cast<const float4*>(z)[q], tb, tm, ts, tt, b.slope));
}

// ---- forward ---------------------------------------------------------------------------
// A workgroup of kFwdThreads (16 waves: W is staged once for all of them, and
// a STATS launch, capped at kMaxGrid workgroups, still has four waves a SIMD
// to hide its loads' latency) holds W in LDS ([32][K + 4]: row stride 4
// floats past K, so the 32 output-channel lanes of a B read fall on distinct
// banks) and walks 32-pixel tiles of one sample each; KSPLIT waves share a
// tile, each a slice of K, summed through LDS (the small layers: more waves
// than tiles).
constexpr int kFwdThreads = 1024;
#ifndef DTUPD_ALL_LOADS
#define DTUPD_ALL_LOADS 8
#endif
constexpr int kFwdAllLoads = DTUPD_ALL_LOADS;   // slices of up to this many k-steps load all A first


// STATS: 0 none, 1 merged by the last workgroup (dt_upd_conv_fwd_bn), 2
// partials for the next kernel (dt_upd_conv_fwd_part).  NORM: x is the
// previous block's z, normalised on load (norm_loads / norm_build from `in`).
template <class G, int KSPLIT, int STATS, bool NORM>
__global__ void __launch_bounds__(kFwdThreads)
fwd_kernel(int n, const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ z,
           FwdBn fb, DtUpdBn in) {
  constexpr bool X3 = DTUPD_X3 != 0;
  constexpr int WST = G::K + 4;
  constexpr int NW = kFwdThreads / 64;
  constexpr int GP = NW / KSPLIT;                // tiles a workgroup round
  constexpr int SPW = G::KSTEPS / KSPLIT;        // k-steps a wave (f32)
  constexpr int KU = G::K / 16;                  // 16-k units (x3)
  constexpr int UPW = KU / KSPLIT;               // units a wave (x3)
  static_assert(G::KSTEPS % KSPLIT == 0 && NW % KSPLIT == 0, "even K slices");
  static_assert(!X3 || (G::K % 16 == 0 && KU % KSPLIT == 0 && G::KROW % 8 == 0),
                "x3: whole 16-k units a slice, 8 k inside a kernel row");
  // W: f32 rows [32][K + 4], or (x3) its B fragments, unit u lane l at u * 64 + l
  __shared__ __attribute__((aligned(16))) float ws[X3 ? 1 : 32 * WST];
  __shared__ half8 wsh[X3 ? KU * 64 : 1], wsl[X3 ? KU * 64 : 1];
  __shared__ float red[KSPLIT > 1 ? GP * (KSPLIT - 1) * 16 * 64 : 1];
  __shared__ __attribute__((aligned(16))) float tab[NORM ? 4 : 1][32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kk = lane >> 5;
  NormRegs nr;
  if constexpr (NORM) {   // the partials' loads first, W's behind them
    static_assert(G::CIN == 32, "the chain's inputs are 32-channel activations");
    nr = norm_loads<kFwdThreads>(in, blockIdx.x == 0);
  }
  if constexpr (X3) {
    // B fragment of unit u, lane l: W[co = l & 31][16 u + 8 (l >> 5) + 0 .. 7]
    for (int q = tid; q < ((DTUPD_SKIP & 2) ? 0 : KU * 64); q += kFwdThreads) {
      const int u = q >> 6, l = q & 63;
      const float4* src = reinterpret_cast<const float4*>(w + (l & 31) * G::K + 16 * u + 8 * (l >> 5));
      split8(src[0], src[1], wsh[q], wsl[q]);
    }
  } else {
    for (int q = tid; q < ((DTUPD_SKIP & 2) ? 0 : 32 * G::K / 4); q += kFwdThreads) {
      const int co = q / (G::K / 4), k4 = q - co * (G::K / 4);
      *reinterpret_cast<float4*>(ws + co * WST + 4 * k4) = reinterpret_cast<const float4*>(w)[q];
    }
  }
  if constexpr (NORM) norm_build<kFwdThreads>(in, nr, tab, blockIdx.x == 0);   // ends in a barrier
  else __syncthreads();
  const int g = wave / KSPLIT, ks = wave - g * KSPLIT;
  const int tiles = n * G::TPS;
  const float* wrow = ws + col * WST + 4 * kk;
  float w_n = 0.0f, w_mean = 0.0f, w_m2 = 0.0f;    // STATS: this lane's channel
  const float bc = STATS ? fb.bias[col] : 0.0f;
  for (int base = blockIdx.x * GP; base < tiles; base += gridDim.x * GP) {
    const int tile = base + g;
    const bool tvalid = tile < tiles;
    const int tc = tvalid ? tile : 0;
    const int s = tc / G::TPS, tb = tc - s * G::TPS;
    const int p = tb * 32 + col;
    const int pc = p < G::OPIX ? p : 0;          // an invalid row reads pixel 0, unused
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    if constexpr (X3) {
      // unit u: A = this lane's pixel, k = 16 u + 8 kk + 0 .. 7 (two float4s
      // of one kernel row), normalised for NORM, split; B from LDS
      const float* xp = x + G::xbase(s, pc);
      const int u0 = ks * UPW;
      f32x16 acc1;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[r] = 0.0f;
      struct A8 { float4 a, b; };
      auto load = [&](int uu) -> A8 {
        const int kc = 16 * (u0 + uu) + 8 * kk;
        if (DTUPD_SKIP & 1) return A8{make_float4(xp[0], kc, uu, 1.0f), make_float4(1.0f, kc, 0.5f, 2.0f)};
        const float* q = xp + G::koff(kc);
        return A8{ld4<G::CIN>(q), ld4<G::CIN>(q + 4)};
      };
      auto unit = [&](int uu, A8 v) {
        const int u = u0 + uu;
        if constexpr (NORM) {
          asm volatile("" ::: "memory");
          const int c0 = (16 * u + 8 * kk) & 31;
          const float4* t0 = reinterpret_cast<const float4*>(&tab[0][c0]);
          const float4* t1 = reinterpret_cast<const float4*>(&tab[1][c0]);
          const float4* t2 = reinterpret_cast<const float4*>(&tab[2][c0]);
          const float4* t3 = reinterpret_cast<const float4*>(&tab[3][c0]);
          v.a = norm4(v.a, t0[0], t1[0], t2[0], t3[0], in.slope);
          v.b = norm4(v.b, t0[1], t1[1], t2[1], t3[1], in.slope);
        }
        half8 xh, xl;
        split8(v.a, v.b, xh, xl);
        const half8 bh = wsh[u * 64 + lane], bl = wsl[u * 64 + lane];
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bh, acc, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bl, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, bh, acc1, 0, 0, 0);
      };
      if constexpr (UPW <= kFwdAllLoads / 2) {
        A8 av[UPW];
#pragma unroll
        for (int uu = 0; uu < UPW; ++uu) av[uu] = load(uu);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int uu = 0; uu < UPW; ++uu) unit(uu, av[uu]);
      } else {
#pragma unroll 2
        for (int uu = 0; uu < UPW; ++uu) unit(uu, load(uu));
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += acc1[r] * kLoInv;
    } else {
    const float* xl = x + G::xbase(s, pc) + 4 * kk;
    const int s0 = ks * SPW;
    // one step: A (normalised for NORM: channels c0 .. c0 + 3 of the previous
    // block) times W's float4 from LDS, four MFMAs
    auto step = [&](int st, float4 a) {
      const int kc = 8 * (s0 + st);
      if constexpr (NORM) {
        // its table reads stay here (hoisted over the slice they need a
        // slice's worth of registers)
        asm volatile("" ::: "memory");
        const int c0 = (kc + 4 * kk) & 31;
        a = norm4(a, *reinterpret_cast<const float4*>(&tab[0][c0]),
                  *reinterpret_cast<const float4*>(&tab[1][c0]),
                  *reinterpret_cast<const float4*>(&tab[2][c0]),
                  *reinterpret_cast<const float4*>(&tab[3][c0]), in.slope);
      }
      const float4 b = *reinterpret_cast<const float4*>(wrow + kc);
      acc = mfma4(a, b, acc);
    };
    auto load = [&](int st) -> float4 {
      const int kc = 8 * (s0 + st);
      return (DTUPD_SKIP & 1) ? make_float4(xl[0], kc, st, 1.0f) : ld4<G::CIN>(xl + G::koff(kc));
    };
    if constexpr (SPW <= kFwdAllLoads) {
      // every A load of the slice in flight before the first MFMA: one
      // latency a tile, the SIMD's other waves' MFMAs covering it
      float4 av[SPW];
#pragma unroll
      for (int st = 0; st < SPW; ++st) av[st] = load(st);
      asm volatile("" ::: "memory");   // keeps the scheduler from sinking loads into the MFMAs
#pragma unroll
      for (int st = 0; st < SPW; ++st) step(st, av[st]);
    } else {
      constexpr int kUnroll = NORM ? 2 : 4;   // NORM: its table reads need the registers
#pragma unroll kUnroll
      for (int st = 0; st < SPW; ++st) step(st, load(st));
    }
    }
    if constexpr (KSPLIT > 1 && !(DTUPD_SKIP & 8)) {   // slice ks > 0 of tile g at slot g * (KSPLIT - 1) + ks - 1
      float* rs = red + (size_t)g * (KSPLIT - 1) * 16 * 64 + lane;
      if (ks > 0)
#pragma unroll
        for (int r = 0; r < 16; ++r) rs[((ks - 1) * 16 + r) * 64] = acc[r];
      __syncthreads();
      if (ks == 0)
#pragma unroll 1
        for (int o = 0; o < KSPLIT - 1; ++o)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] += rs[(o * 16 + r) * 64];
      __syncthreads();
    }
    if (ks == 0 && tvalid) {
      float* zs = z + (size_t)s * G::OPIX * 32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pr = tb * 32 + acc_row(r, kk);
        if (pr < G::OPIX) zs[pr * 32 + col] = acc[r];
      }
      if constexpr (STATS) {   // a = leaky(z + bias), as dt_bn_leaky_fwd computes it
        float a[16], tn = 0.0f, ts = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool ok = tb * 32 + acc_row(r, kk) < G::OPIX;
          const float v = acc[r] + bc;
          a[r] = v > 0.0f ? v : v * fb.slope;
          tn += ok ? 1.0f : 0.0f;
          ts += ok ? a[r] : 0.0f;
        }
        const float tm = ts / tn;
        float tq = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = a[r] - tm;
          tq += tb * 32 + acc_row(r, kk) < G::OPIX ? d * d : 0.0f;
        }
        chan(w_n, w_mean, w_m2, tn, tm, tq);
      }
    }
  }
  if constexpr (STATS == 1 && !(DTUPD_SKIP & 4))
    merge_partials_last<kFwdThreads>(fb, w_n, w_mean, w_m2, (int64_t)n * G::OPIX);
  if constexpr (STATS == 2) wg_partial<kFwdThreads, false>(fb.work, w_n, w_mean, w_m2);
}

// ---- weight gradient -------------------------------------------------------------------
// A workgroup takes whole output rows (sample s, row oy): it stages the KS
// input rows that row reads (KS * IW * C_in contiguous floats of NHWC) and
// the row's dZ (OW * 32) in LDS with float4 loads, then every wave runs its
// NBW 32-wide blocks of k over the row's pixels two at a time (the MFMA's two
// k-slots): A = dZ[pixel][co] (lane co), B = the pixel's patch value k (lane
// k), both LDS reads.  An input pixel is read from HBM once per output row
// that needs it, not once per (pixel, tap).  The workgroup's partial dW goes
// to part[blockIdx.x]; wgrad_reduce_kernel sums them in index order.
// workgroups (= partials) of a launch at most: enough to fill the chip, few
// enough that the partials stay small next to the layer's own traffic
template <class G>
constexpr int wgrad_max_grid() { return G::CIN == 3 ? 512 : (G::OH > 20 ? 256 : 128); }

// NORM: x is the previous block's z, staged as bn(leaky(z + bias)) with
// in.mean_invstd (the chain's forward wrote it)
template <class G, int NBW, int WAVES, bool NORM, bool DB>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(1, 4)))
wgrad_kernel(int n, const float* __restrict__ x, const float* __restrict__ dz,
             float* __restrict__ part, DtUpdBn in) {
  static_assert(WAVES * NBW * 32 == G::K, "the waves cover K");
  constexpr int XROW = G::IW * G::CIN;       // floats of one input row
  constexpr int XT = G::KS * XROW;           // the rows one output row reads
  constexpr int DT = G::OW * 32;
  static_assert(XROW % 4 == 0 && DT % 4 == 0, "float4 staging");
  constexpr int NT = 64 * WAVES;
  constexpr int NB = DB ? 2 : 1;             // staging buffers
  __shared__ __attribute__((aligned(16))) float xs[NB][XT];
  __shared__ __attribute__((aligned(16))) float ds[NB][DT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kk = lane >> 5;
  // NORM: a thread's float4s are always channels 4 (tid & 7) .. + 3 (NT and a
  // row's floats are multiples of 32)
  float4 nb, nm, ns, nt;
  if constexpr (NORM) {
    static_assert(G::CIN == 32 && NT % 8 == 0, "32-channel rows");
    const int c0 = 4 * (tid & 7);
    nb = *reinterpret_cast<const float4*>(in.bias + c0);
    nm = *reinterpret_cast<const float4*>(in.mean_invstd + c0);
    const float4 is = *reinterpret_cast<const float4*>(in.mean_invstd + 32 + c0);
    const float4 g = *reinterpret_cast<const float4*>(in.gamma + c0);
    ns = make_float4(is.x * g.x, is.y * g.y, is.z * g.z, is.w * g.w);
    nt = *reinterpret_cast<const float4*>(in.beta + c0);
  }
  int kr[NBW];   // k's offset inside the staged rows
#pragma unroll
  for (int b = 0; b < NBW; ++b) {
    const int k = (wave * NBW + b) * 32 + col;
    kr[b] = (k / G::KROW) * XROW + k % G::KROW;
  }
  // x3 where a row fills >= 60 % of its 16-pixel units: conv3's 17-pixel
  // rows would leave 47 % of the slots empty (measured at batch 64: 18.8 us
  // f32 against 20.2 x3)
  constexpr bool X3 = DTUPD_X3 != 0 && 10 * G::OW >= 6 * 16 * ((G::OW + 15) / 16);
  f32x16 acc[NBW], acc1[X3 ? NBW : 1];
#pragma unroll
  for (int b = 0; b < NBW; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.0f;
  if constexpr (X3)
#pragma unroll
    for (int b = 0; b < NBW; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[b][r] = 0.0f;
  const int rows = n * G::OH;
  // a row's staging as loads into registers (fetch) and LDS stores (commit):
  // DB fetches row i + 1 before row i's MFMAs and commits it after them
  constexpr int PX = (XT / 4 + NT - 1) / NT, PD = (DT / 4 + NT - 1) / NT;
  float4 rx0, rx1, rx2, rx3, rx4, rx5, rd0, rd1;   // PX <= 6, PD <= 2 (asserted)
  static_assert(PX <= 6 && PD <= 2, "staging registers");
#define DTUPD_FETCH(ROW)                                                                          \
  do {                                                                                           \
    const int sm_ = (ROW) / G::OH, oy_ = (ROW) - sm_ * G::OH;                                    \
    const float4* xsrc_ =                                                                        \
        reinterpret_cast<const float4*>(x + (size_t)(sm_ * G::IH + G::ST * oy_) * XROW) + tid;   \
    const float4* dsrc_ = reinterpret_cast<const float4*>(dz + (size_t)(ROW) * DT) + tid;        \
    if (0 < PX && tid + 0 * NT < XT / 4) rx0 = xsrc_[0 * NT];                                     \
    if (1 < PX && tid + 1 * NT < XT / 4) rx1 = xsrc_[1 * NT];                                     \
    if (2 < PX && tid + 2 * NT < XT / 4) rx2 = xsrc_[2 * NT];                                     \
    if (3 < PX && tid + 3 * NT < XT / 4) rx3 = xsrc_[3 * NT];                                     \
    if (4 < PX && tid + 4 * NT < XT / 4) rx4 = xsrc_[4 * NT];                                     \
    if (5 < PX && tid + 5 * NT < XT / 4) rx5 = xsrc_[5 * NT];                                     \
    if (0 < PD && tid + 0 * NT < DT / 4) rd0 = dsrc_[0 * NT];                                     \
    if (1 < PD && tid + 1 * NT < DT / 4) rd1 = dsrc_[1 * NT];                                     \
  } while (0)
  // x3: the staged values as (hi, lo) fp16 words (hl4), split once a stage
  // instead of once a use
  auto put = [&](int buf, int i, float4 v) __attribute__((always_inline)) {
    if constexpr (NORM) v = norm4(v, nb, nm, ns, nt, in.slope);
    if constexpr (X3) reinterpret_cast<uint4*>(xs[buf])[tid + i * NT] = hl4(v);
    else reinterpret_cast<float4*>(xs[buf])[tid + i * NT] = v;
  };
  auto putd = [&](int buf, int i, float4 v) __attribute__((always_inline)) {
    if constexpr (X3) reinterpret_cast<uint4*>(ds[buf])[tid + i * NT] = hl4(v);
    else reinterpret_cast<float4*>(ds[buf])[tid + i * NT] = v;
  };
  auto commit = [&](int buf) __attribute__((always_inline)) {
    if (0 < PX && tid + 0 * NT < XT / 4) put(buf, 0, rx0);
    if (1 < PX && tid + 1 * NT < XT / 4) put(buf, 1, rx1);
    if (2 < PX && tid + 2 * NT < XT / 4) put(buf, 2, rx2);
    if (3 < PX && tid + 3 * NT < XT / 4) put(buf, 3, rx3);
    if (4 < PX && tid + 4 * NT < XT / 4) put(buf, 4, rx4);
    if (5 < PX && tid + 5 * NT < XT / 4) put(buf, 5, rx5);
    if (0 < PD && tid + 0 * NT < DT / 4) putd(buf, 0, rd0);
    if (1 < PD && tid + 1 * NT < DT / 4) putd(buf, 1, rd1);
  };
  auto compute = [&](int buf) __attribute__((always_inline)) {
    if constexpr (X3) {
      // 16 pixels a unit: A = dZ[ox0 + 8 kk + j][co], B = X[ox0 + 8 kk + j][k]
      // (pixels past the row: A zero, B pixel 0's)
      const uint32_t* xb = reinterpret_cast<const uint32_t*>(xs[buf]);
      const uint32_t* db = reinterpret_cast<const uint32_t*>(ds[buf]);
#pragma unroll 1
      for (int ox0 = 0; ox0 < G::OW; ox0 += 16) {
        uint32_t aw[8], xw[NBW][8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ox = ox0 + 8 * kk + j;
          const bool ok = ox < G::OW;
          aw[j] = ok ? db[ox * 32 + col] : 0u;
          const int xo = (ok ? ox : 0) * G::ST * G::CIN;
#pragma unroll
          for (int b = 0; b < NBW; ++b) xw[b][j] = xb[xo + kr[b]];
        }
        half8 ah, al;
        hl_frag(aw, ah, al);
#pragma unroll
        for (int b = 0; b < NBW; ++b) {
          half8 xh, xl;
          hl_frag(xw[b], xh, xl);
          acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xh, acc[b], 0, 0, 0);
          acc1[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xl, acc1[b], 0, 0, 0);
          acc1[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, xh, acc1[b], 0, 0, 0);
        }
      }
      return;
    }
    const float* xb = xs[buf];
    const float* db = ds[buf];
#pragma unroll 2
    for (int ox0 = 0; ox0 < G::OW; ox0 += 2) {
      const int ox = ox0 + kk;
      const bool ok = ox < G::OW;
      const float a = ok ? db[ox * 32 + col] : 0.0f;
      const int xo = (ok ? ox : 0) * G::ST * G::CIN;
#pragma unroll
      for (int b = 0; b < NBW; ++b)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, xb[xo + kr[b]], acc[b], 0, 0, 0);
    }
  };
  if constexpr (DB) {
    int buf = 0;
    if ((int)blockIdx.x < rows) {
      DTUPD_FETCH((int)blockIdx.x);
      commit(0);
    }
    __syncthreads();
    for (int row = blockIdx.x; row < rows; row += gridDim.x) {
      const int next = row + gridDim.x;
      if (next < rows) DTUPD_FETCH(next);     // in flight during this row's MFMAs
      compute(buf);
      if (next < rows) commit(buf ^ 1);       // the other buffer: its readers passed the barrier
      __syncthreads();
      buf ^= 1;
    }
  } else {
    for (int row = blockIdx.x; row < rows; row += gridDim.x) {
      __syncthreads();                        // the previous row's reads
      DTUPD_FETCH(row);
      commit(0);
      __syncthreads();
      compute(0);
    }
  }
#undef DTUPD_FETCH
  if constexpr (X3)
#pragma unroll
    for (int b = 0; b < NBW; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[b][r] += acc1[b][r] * kLoInv;
  // D[co][k]: lane (k = block * 32 + col), rows co
  float* pp = part + (size_t)blockIdx.x * 32 * G::K;
#pragma unroll
  for (int b = 0; b < NBW; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      pp[acc_row(r, kk) * G::K + (wave * NBW + b) * 32 + col] = acc[b][r];
}

// dw[i] = sum of the chunks' partials: a workgroup takes kRedCols float4
// columns (4 outputs each), kRedWays threads a column each summing every
// kRedWays-th chunk (two accumulators), then the ways in a fixed two-level
// order (deterministic).  Few loads a thread, all of a column's chunks in
// flight at once: the reduce is one memory round trip (round 6; the former
// 8-way scalar form ran the conv1 partials at 1 TB/s).
constexpr int kRedCols = 16, kRedWays = 64, kRedThreads = kRedCols * kRedWays;
__global__ void __launch_bounds__(kRedThreads)
wgrad_reduce_kernel(int chunks, int len, const float* __restrict__ part, float* __restrict__ dw) {
  __shared__ float4 red[kRedWays][kRedCols];
  __shared__ float4 red2[8][kRedCols];
  const int o = threadIdx.x & (kRedCols - 1), w = threadIdx.x / kRedCols;
  const int len4 = len >> 2;
  const int i4 = blockIdx.x * kRedCols + o;
  float4 s0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), s1 = s0;
  if (i4 < len4) {
    const float4* p = reinterpret_cast<const float4*>(part) + i4;
    int c = w;
    for (; c + kRedWays < chunks; c += 2 * kRedWays) {
      const float4 a = p[(size_t)c * len4], b = p[(size_t)(c + kRedWays) * len4];
      s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
      s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
    }
    if (c < chunks) {
      const float4 a = p[(size_t)c * len4];
      s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
    }
  }
  red[w][o] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
  __syncthreads();
  if (w < 8) {
    float4 t = red[8 * w][o];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const float4 v = red[8 * w + k][o];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    red2[w][o] = t;
  }
  __syncthreads();
  if (w == 0 && i4 < len4) {
    float4 t = red2[0][o];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const float4 v = red2[k][o];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    reinterpret_cast<float4*>(dw)[i4] = t;
  }
}

// ---- input gradient (C_in = 32) ----------------------------------------------------------
// Input pixels split into ST x ST parity classes (ph, pw): in one class the
// kernel taps that reach a pixel are the same, kh = ph + ST th, kw = pw + ST tw
// (th, tw < KS / ST), from output pixel (a - th, b - tw) where (ih, iw) =
// (ST a + ph, ST b + pw).  A tile is 32 consecutive (a, b) of one class, so
// B = W^T of a tap is uniform across the tile; taps falling outside the
// output contribute zero.  W^T sits in LDS as [tap][ci][co + 4].
template <class G>
struct DGeom {
  static constexpr int ST = G::ST, T1 = G::KS / G::ST, TAPS = T1 * T1;
  static constexpr int NCLS = ST * ST;
  __host__ __device__ static constexpr int ac(int c) { return (G::IH - c / ST + ST - 1) / ST; }
  __host__ __device__ static constexpr int bc(int c) { return (G::IW - c % ST + ST - 1) / ST; }
  __host__ __device__ static constexpr int tiles(int c) { return (ac(c) * bc(c) + 31) / 32; }
  __host__ __device__ static constexpr int first(int c) {   // first tile of class c in a sample
    int t = 0;
    for (int i = 0; i < c; ++i) t += tiles(i);
    return t;
  }
  static constexpr int TPS = first(NCLS);
};

// NW waves a workgroup: many for the layer with the most tiles a sample,
// few where a sample has only a handful (more workgroups, each staging W^T)
template <class G, int NW>
__global__ void __launch_bounds__(64 * NW)
dgrad_kernel(int n, const float* __restrict__ dz, const float* __restrict__ w,
             float* __restrict__ dx) {
  using D = DGeom<G>;
  static_assert(G::CIN == 32, "dgrad for 32-channel inputs");
  constexpr bool X3 = DTUPD_X3 != 0;
  constexpr int KK = G::KS * G::KS;               // taps of W
  constexpr int CST = 36;                         // co stride of a W^T row
  // f32: W^T as [tap][ci][co + 4]; x3: its B fragments, tap t, unit u (co
  // 16 u ..), lane l at (t * 2 + u) * 64 + l, hi and lo
  __shared__ __attribute__((aligned(16))) float wt[X3 ? 1 : KK * 32 * CST];
  __shared__ half8 wth[X3 ? KK * 128 : 1], wtl[X3 ? KK * 128 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kk = lane >> 5;
  if constexpr (X3) {
    // fragment (t, u, l): W[co = 16 u + 8 (l >> 5) + j][t][ci = l & 31], j < 8
    for (int q = tid; q < KK * 128; q += 64 * NW) {
      const int t = q >> 7, u = (q >> 6) & 1, l = q & 63;
      const float* src = w + (size_t)(16 * u + 8 * (l >> 5)) * G::K + t * 32 + (l & 31);
      const float4 a = make_float4(src[0], src[G::K], src[2 * G::K], src[3 * G::K]);
      const float4 b = make_float4(src[4 * G::K], src[5 * G::K], src[6 * G::K], src[7 * G::K]);
      split8(a, b, wth[q], wtl[q]);
    }
  } else {
    // W [co][kh][kw][ci] -> wt[kh * KS + kw][ci][co]
    for (int i = tid; i < 32 * G::K; i += 64 * NW) {
      const int co = i / G::K, r = i - co * G::K;
      const int tap = r / 32, ci = r - tap * 32;
      wt[(tap * 32 + ci) * CST + co] = w[i];
    }
  }
  __syncthreads();
  const int tiles = n * D::TPS;
  for (int tile = blockIdx.x * NW + wave; tile < tiles; tile += gridDim.x * NW) {
    const int s = tile / D::TPS;
    int t = tile - s * D::TPS, cls = 0;
#pragma unroll
    for (int c = 1; c < D::NCLS; ++c)
      if (t >= D::first(c)) cls = c;
    t -= D::first(cls);
    const int ph = cls / D::ST, pw = cls - ph * D::ST;
    const int bcn = D::bc(cls), np = D::ac(cls) * bcn;
    const int idx = t * 32 + col;
    const int ic = idx < np ? idx : 0;
    const int a = ic / bcn, b = ic - a * bcn;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    if constexpr (X3) {
      // unit u of a tap: A = dZ[o][16 u + 8 kk + 0 .. 7] (zero off the output)
      const float* dzs = dz + (size_t)s * G::OPIX * 32 + 8 * kk;
      f32x16 acc1;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[r] = 0.0f;
#pragma unroll 2
      for (int tap = 0; tap < D::TAPS; ++tap) {
        const int th = tap / D::T1, tw = tap - th * D::T1;
        const int oy = a - th, ox = b - tw;
        const bool ok = idx < np && oy >= 0 && oy < G::OH && ox >= 0 && ox < G::OW;
        const float4* src = reinterpret_cast<const float4*>(dzs + (ok ? (oy * G::OW + ox) * 32 : 0));
        const int wtap = (ph + D::ST * th) * G::KS + pw + D::ST * tw;
        float4 av[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          av[i] = src[(i >> 1) * 4 + (i & 1)];
          if (!ok) av[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          half8 xh, xl;
          split8(av[2 * u], av[2 * u + 1], xh, xl);
          const half8 bh = wth[(wtap * 2 + u) * 64 + lane], bl = wtl[(wtap * 2 + u) * 64 + lane];
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bh, acc, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, bl, acc1, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, bh, acc1, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += acc1[r] * kLoInv;
    } else {
      const float* dzs = dz + (size_t)s * G::OPIX * 32 + 4 * kk;
#pragma unroll 4
      for (int tap = 0; tap < D::TAPS; ++tap) {
        const int th = tap / D::T1, tw = tap - th * D::T1;
        const int oy = a - th, ox = b - tw;
        const bool ok = idx < np && oy >= 0 && oy < G::OH && ox >= 0 && ox < G::OW;
        const float* src = dzs + (ok ? (oy * G::OW + ox) * 32 : 0);
        const int kh = ph + D::ST * th, kw = pw + D::ST * tw;
        const float* wrow = wt + ((kh * G::KS + kw) * 32 + col) * CST + 4 * kk;
#pragma unroll
        for (int c8 = 0; c8 < 4; ++c8) {
          float4 av = *reinterpret_cast<const float4*>(src + 8 * c8);
          if (!ok) av = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          const float4 bv = *reinterpret_cast<const float4*>(wrow + 8 * c8);
          acc = mfma4(av, bv, acc);
        }
      }
    }
    float* dxs = dx + (size_t)s * G::IH * G::IW * 32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ir = t * 32 + acc_row(r, kk);
      if (ir < np) {
        const int ar = ir / bcn, br = ir - ar * bcn;
        dxs[((D::ST * ar + ph) * G::IW + D::ST * br + pw) * 32 + col] = acc[r];
      }
    }
  }
}

// ---- the linear layer after the trunk (flatten -> dropout -> linear 4032 -> 256 / 512) ----
// y[m][n] = b[n] + sum_k x[m][k] W[n][k] with M (the batch) small and K long:
// library GEMMs pick one tile a workgroup over all of K (latency-bound, 20 us
// at batch 64).  Here K is split: each wave takes a slice of k-steps of a
// 32 x 32 output tile (float4 loads of x and W rows, the K-permutation trick),
// the four waves of a workgroup sum through LDS into one partial, and
// lin_reduce_kernel adds the partials in index order plus the bias.
constexpr int kLinWaves = 4;

// The dropout before the linear (flatten -> dropout -> linear, config.json),
// folded into its three kernels: u [m, k] uniforms in [0, 1) (or null: no
// dropout), an element kept where u >= p and then scaled by 1 / (1 - p), as
// F.dropout's bernoulli(1 - p) mask; the same u in the forward (on x's
// loads), the input gradient (on its stores) and the weight gradient (on x's
// loads).
struct Drop {
  const float* u;
  float p, scale;
  float* xd;   // forward: the dropped input written out (the n0 = 0 tiles), or null
};
__device__ __forceinline__ float4 drop4(float4 v, const float* u, float p, float scale) {
  const float4 q = *reinterpret_cast<const float4*>(u);
  return make_float4(q.x >= p ? v.x * scale : 0.0f, q.y >= p ? v.y * scale : 0.0f,
                     q.z >= p ? v.z * scale : 0.0f, q.w >= p ? v.w * scale : 0.0f);
}

// torch's leaky_relu backward on the output (same sign as the input for slope > 0)
__device__ __forceinline__ float4 leaky_grad4(float4 g, float4 y, float slope) {
  return make_float4(y.x > 0.0f ? g.x : g.x * slope, y.y > 0.0f ? g.y : g.y * slope,
                     y.z > 0.0f ? g.z : g.z * slope, y.w > 0.0f ? g.w : g.w * slope);
}

__global__ void __launch_bounds__(64 * kLinWaves)
lin_fwd_kernel(int m, int n, int k, int chunk, const float* __restrict__ x,
               const float* __restrict__ w, float* __restrict__ part, Drop dr) {
  __shared__ float red[kLinWaves - 1][16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kk = lane >> 5;
  const int ntile = n / 32, tile = blockIdx.x % (ntile * ((m + 31) / 32));
  const int split = blockIdx.x / (ntile * ((m + 31) / 32));
  const int m0 = (tile / ntile) * 32, n0 = (tile % ntile) * 32;
  const int steps = k / 8;
  const int s0 = (split * kLinWaves + wave) * chunk;
  const int s1 = s0 + chunk < steps ? s0 + chunk : steps;
  const bool mok = m0 + col < m;
  const float* xr = x + (size_t)(mok ? m0 + col : 0) * k + 4 * kk;
  const float* wr = w + (size_t)(n0 + col) * k + 4 * kk;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll 4
  for (int st = s0; st < s1; ++st) {
    float4 a = *reinterpret_cast<const float4*>(xr + 8 * st);
    if (dr.u) {
      a = drop4(a, dr.u + (xr - x) + 8 * st, dr.p, dr.scale);
      if (dr.xd && n0 == 0 && mok) *reinterpret_cast<float4*>(dr.xd + (xr - x) + 8 * st) = a;
    }
    if (!mok) a = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float4 b = *reinterpret_cast<const float4*>(wr + 8 * st);
    acc = mfma4(a, b, acc);
  }
  if (wave > 0)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave - 1][r][lane] = acc[r];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int o = 0; o < kLinWaves - 1; ++o)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += red[o][r][lane];
    float* pp = part + (size_t)split * m * n;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = m0 + acc_row(r, kk);
      if (mm < m) pp[(size_t)mm * n + n0 + col] = acc[r];
    }
  }
}

__global__ void __launch_bounds__(256)
lin_reduce_kernel(int mn, int n, int splits, const float* __restrict__ part,
                  const float* __restrict__ bias, int act, float slope, float* __restrict__ y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= mn) return;
  float s = 0.0f;
  int p = 0;
  for (; p + 8 <= splits; p += 8) {   // eight loads in flight, summed in index order
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = part[(size_t)(p + j) * mn + i];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
  }
  for (; p < splits; ++p) s += part[(size_t)p * mn + i];
  float v = bias ? s + bias[i % n] : s;
  if (act) v = v > 0.0f ? v : v * slope;        // a following LeakyReLU, as torch computes it
  y[i] = v;
}

// dx[m][k] = sum_n dy[m][n] W[n][k]: a workgroup a 32 x 32 tile of dx, its
// four waves a quarter of n each, summed through LDS
__global__ void __launch_bounds__(64 * kLinWaves)
lin_dgrad_kernel(int m, int n, int k, const float* __restrict__ dy, const float* __restrict__ w,
                 const float* __restrict__ yact, float slope, float* __restrict__ dx, Drop dr) {
  __shared__ float red[kLinWaves - 1][16][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kk = lane >> 5;
  const int ktile = k / 32;
  const int m0 = (blockIdx.x / ktile) * 32, k0 = (blockIdx.x % ktile) * 32;
  const int steps = n / 8, chunk = (steps + kLinWaves - 1) / kLinWaves;
  const int s0 = wave * chunk, s1 = s0 + chunk < steps ? s0 + chunk : steps;
  const bool mok = m0 + col < m;
  const float* dyr = dy + (size_t)(mok ? m0 + col : 0) * n + 4 * kk;
  const float* wc = w + (size_t)(4 * kk) * k + k0 + col;   // W[n][k0 + col], n = 8 st + 4 kk + e
  float um[16];   // the dropout uniforms of this lane's dx elements, loaded up front
  if (dr.u)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = m0 + acc_row(r, kk);
      um[r] = mm < m ? dr.u[(size_t)mm * k + k0 + col] : 0.0f;
    }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
#pragma unroll 2
  for (int st = s0; st < s1; ++st) {
    float4 a = *reinterpret_cast<const float4*>(dyr + 8 * st);
    if (yact) a = leaky_grad4(a, *reinterpret_cast<const float4*>(yact + (dyr - dy) + 8 * st), slope);
    if (!mok) a = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float* wp = wc + (size_t)(8 * st) * k;
    const float4 b = make_float4(wp[0], wp[k], wp[2 * (size_t)k], wp[3 * (size_t)k]);
    acc = mfma4(a, b, acc);
  }
  if (wave > 0)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave - 1][r][lane] = acc[r];
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int o = 0; o < kLinWaves - 1; ++o)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += red[o][r][lane];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = m0 + acc_row(r, kk);
      if (mm < m) {
        const size_t at = (size_t)mm * k + k0 + col;
        dx[at] = dr.u ? (um[r] >= dr.p ? acc[r] * dr.scale : 0.0f) : acc[r];
      }
    }
  }
}

// dW[n][k] = sum_m dy[m][n] x[m][k] (a wave a 32 x 32 tile, all m) and
// db[n] = sum_m dy[m][n] (the k0 = 0 tiles, from the same loads)
__global__ void __launch_bounds__(64 * kLinWaves)
lin_wgrad_kernel(int m, int n, int k, const float* __restrict__ dy, const float* __restrict__ x,
                 const float* __restrict__ yact, float slope, float* __restrict__ dw,
                 float* __restrict__ db) {
  // dy through a fused LeakyReLU (yact: its output, the same sign as its input)
  auto gy = [&](size_t i) __attribute__((always_inline)) {
    const float g = dy[i];
    return yact ? (yact[i] > 0.0f ? g : g * slope) : g;
  };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, kk = lane >> 5;
  const int ktile = k / 32, tiles = (n / 32) * ktile;
  const int tile = blockIdx.x * kLinWaves + wave;
  if (tile >= tiles) return;
  const int n0 = (tile / ktile) * 32, k0 = (tile % ktile) * 32;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  const int steps = (m + 7) / 8;
  float sb = 0.0f;
  constexpr int kBatch = 8;                 // steps whose loads go out together (m <= 64: all)
  for (int s0 = 0; s0 < steps; s0 += kBatch) {
    float av[kBatch][4], bv[kBatch][4];
#pragma unroll
    for (int j = 0; j < kBatch; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int mm = 8 * (s0 + j) + 4 * kk + e;
        const bool ok = s0 + j < steps && mm < m;
        av[j][e] = ok ? gy((size_t)mm * n + n0 + col) : 0.0f;
        bv[j][e] = ok ? x[(size_t)mm * k + k0 + col] : 0.0f;
      }
#pragma unroll
    for (int j = 0; j < kBatch; ++j)
      if (s0 + j < steps)
        acc = mfma4(make_float4(av[j][0], av[j][1], av[j][2], av[j][3]),
                    make_float4(bv[j][0], bv[j][1], bv[j][2], bv[j][3]), acc);
    if (k0 == 0)   // db from the same loads: this lane's half of m, in order
#pragma unroll
      for (int j = 0; j < kBatch; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) sb += av[j][e];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) dw[(size_t)(n0 + acc_row(r, kk)) * k + k0 + col] = acc[r];
  if (k0 == 0) {                          // the two halves of m (lane pairs l, l ^ 32)
    const float other = __shfl_xor(sb, 32);
    if (db && kk == 0) db[n0 + col] = sb + other;
  }
}

// splits of K a forward launch uses (about a wave a SIMD over the tiles)
int lin_splits(int m, int n, int k) {
  const int tiles = (n / 32) * ((m + 31) / 32), steps = k / 8;
  int sw = 256 / (tiles > 0 ? tiles : 1);                 // workgroups a tile
  sw = sw < 1 ? 1 : sw;
  const int maxw = (steps + kLinWaves - 1) / kLinWaves;   // at least one step a wave
  return sw < maxw ? sw : maxw;
}

// ---- host ------------------------------------------------------------------------------
int resident(const void* kern, int threads, int cap) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  int per = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, threads, 0) != hipSuccess || per < 1)
    per = 1;
  const int g = per * cus;
  return g < cap ? g : cap;
}

template <class G, int KSPLIT, int STATS, bool NORM>
int launch_fwd(int n, const float* x, const float* w, float* z, const FwdBn& fb, const DtUpdBn& in,
               hipStream_t s, int32_t* grid_out) {
  constexpr int GP = kFwdThreads / 64 / KSPLIT;
  const int tiles = n * G::TPS;
  int grid = (tiles + GP - 1) / GP;
  // STATS: at most kMaxGrid partials
  static const int res =
      resident(reinterpret_cast<const void*>(fwd_kernel<G, KSPLIT, STATS, NORM>), kFwdThreads,
               STATS ? kMaxGrid : 1 << 20);
  grid = grid < res ? grid : res;
  hipLaunchKernelGGL((fwd_kernel<G, KSPLIT, STATS, NORM>), dim3(grid), dim3(kFwdThreads), 0, s, n,
                     x, w, z, fb, in);
  if (grid_out) *grid_out = grid;
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

template <int STATS, bool NORM>
int dispatch_fwd(int l, int n, const float* x, const float* w, float* z, const FwdBn& fb,
                 const DtUpdBn& in, hipStream_t s, int32_t* grid_out = nullptr) {
  switch (l) {
    case 1:
      if constexpr (NORM) return DT_E_ARG;
      else return launch_fwd<L1, DTUPD_KS1, STATS, false>(n, x, w, z, fb, in, s, grid_out);
    case 2: return launch_fwd<L2, DTUPD_KS2, STATS, NORM>(n, x, w, z, fb, in, s, grid_out);
    case 3: return launch_fwd<L3, DTUPD_KS3, STATS, NORM>(n, x, w, z, fb, in, s, grid_out);
    default: return launch_fwd<L4, DTUPD_KS4, STATS, NORM>(n, x, w, z, fb, in, s, grid_out);
  }
}

// workgroups (= partials) of a weight-gradient launch
template <class G>
int wgrad_chunks(int n) {
  const int rows = n * G::OH;
  return rows < wgrad_max_grid<G>() ? rows : wgrad_max_grid<G>();
}

template <class G, int NBW, int WAVES, bool NORM, bool DB = (DTUPD_WG_DB != 0)>
int launch_wgrad(int n, const float* x, const DtUpdBn& in, const float* dz, float* dw, float* work,
                 hipStream_t s) {
  const int chunks = wgrad_chunks<G>(n);
  hipLaunchKernelGGL((wgrad_kernel<G, NBW, WAVES, NORM, DB>), dim3(chunks), dim3(64 * WAVES), 0, s,
                     n, x, dz, work, in);
  constexpr int len = 32 * G::K;
  static_assert(len % 4 == 0, "float4 columns");
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((len / 4 + kRedCols - 1) / kRedCols),
                     dim3(kRedThreads), 0, s, chunks, len, work, dw);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

template <class G, int NW>
int launch_dgrad(int n, const float* dz, const float* w, float* dx, hipStream_t s) {
  const int tiles = n * DGeom<G>::TPS;
  int grid = (tiles + NW - 1) / NW;
  static const int res =
      resident(reinterpret_cast<const void*>(dgrad_kernel<G, NW>), 64 * NW, 1 << 20);
  grid = grid < res ? grid : res;
  hipLaunchKernelGGL((dgrad_kernel<G, NW>), dim3(grid), dim3(64 * NW), 0, s, n, dz, w, dx);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// a chain hand-off's required pointers
bool valid_in(const DtUpdBn& b) {
  return b.part && b.parts >= 1 && b.parts <= kMaxGrid && b.m >= 1 && b.bias && b.gamma &&
         b.beta && b.running_mean && b.running_var && b.mean_invstd && b.updates >= 1;
}

// which of the four layers (0: none)
int layer_of(int cin, int ks, int st, int ih, int iw) {
  if (cin == 3 && ks == 8 && st == 2 && ih == 120 && iw == 160) return 1;
  if (cin == 32 && ks == 4 && st == 2 && ih == 57 && iw == 77) return 2;
  if (cin == 32 && ks == 4 && st == 2 && ih == 27 && iw == 37) return 3;
  if (cin == 32 && ks == 4 && st == 1 && ih == 12 && iw == 17) return 4;
  return 0;
}

}  // namespace

extern "C" {

int dt_upd_conv_fwd(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                    const float* x, const float* w, float* z, void* stream) {
  const int l = layer_of(cin, ks, st, ih, iw);
  if (!l || n < 0 || (n > 0 && (!x || !w || !z))) return DT_E_ARG;
  if (n == 0) return DT_OK;
  return dispatch_fwd<0, false>(l, n, x, w, z, FwdBn{}, DtUpdBn{}, (hipStream_t)stream);
}

int dt_upd_conv_fwd_bn(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                       const float* x, const float* w, const float* bias, float slope, float eps,
                       float momentum, float* running_mean, float* running_var,
                       int64_t* num_batches_tracked, int32_t updates, float* z,
                       float* mean_invstd, float* work, int32_t* guard, void* stream) {
  const int l = layer_of(cin, ks, st, ih, iw);
  if (!l || n < 1 || updates < 1 || !x || !w || !z || !bias || !running_mean || !running_var ||
      !mean_invstd || !work)
    return DT_E_ARG;
  const FwdBn fb{bias, slope, eps, momentum, running_mean, running_var, num_batches_tracked,
                 (int)updates, mean_invstd, work, guard};
  return dispatch_fwd<1, false>(l, n, x, w, z, fb, DtUpdBn{}, (hipStream_t)stream);
}

int64_t dt_upd_bn_work_floats(void) { return (int64_t)kMaxGrid * 32 * 3 + 16; }

int64_t dt_upd_wgrad_work_floats(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih,
                                 int32_t iw) {
  if (n < 1) return -1;
  switch (layer_of(cin, ks, st, ih, iw)) {
    case 1: return (int64_t)wgrad_chunks<L1>(n) * 32 * L1::K;
    case 2: return (int64_t)wgrad_chunks<L2>(n) * 32 * L2::K;
    case 3: return (int64_t)wgrad_chunks<L3>(n) * 32 * L3::K;
    case 4: return (int64_t)wgrad_chunks<L4>(n) * 32 * L4::K;
    default: return -1;
  }
}

int dt_upd_conv_wgrad_bn(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                         const float* x, const DtUpdBn* in, const float* dz, float* dw,
                         float* work, void* stream) {
  const int l = layer_of(cin, ks, st, ih, iw);
  if (!l || n < 1 || !x || !dz || !dw || !work || !aligned16(dw) || !aligned16(work)) return DT_E_ARG;
  if (in && (l == 1 || !in->mean_invstd || !in->bias || !in->gamma || !in->beta ||
             !aligned16(in->mean_invstd) || !aligned16(in->bias) || !aligned16(in->gamma) ||
             !aligned16(in->beta)))
    return DT_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  const DtUpdBn b = in ? *in : DtUpdBn{};
  switch (l) {
    case 1: return launch_wgrad<L1, 1, 6, false, DTUPD_WG_DB1 != 0>(n, x, b, dz, dw, work, s);
    case 2:
      return in ? launch_wgrad<L2, 2, 8, true>(n, x, b, dz, dw, work, s)
                : launch_wgrad<L2, 2, 8, false>(n, x, b, dz, dw, work, s);
    case 3:
      return in ? launch_wgrad<L3, 2, 8, true>(n, x, b, dz, dw, work, s)
                : launch_wgrad<L3, 2, 8, false>(n, x, b, dz, dw, work, s);
    default:
      return in ? launch_wgrad<L4, 2, 8, true>(n, x, b, dz, dw, work, s)
                : launch_wgrad<L4, 2, 8, false>(n, x, b, dz, dw, work, s);
  }
}

int dt_upd_conv_wgrad(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                      const float* x, const float* dz, float* dw, float* work, void* stream) {
  return dt_upd_conv_wgrad_bn(cin, ks, st, n, ih, iw, x, nullptr, dz, dw, work, stream);
}

int64_t dt_upd_part_floats(void) { return (int64_t)kMaxGrid * 32 * 3; }

static bool lin_shape_ok(int32_t m, int32_t n, int32_t k) {
  return m >= 1 && n >= 32 && n % 32 == 0 && k >= 8 && k % 32 == 0;
}

int64_t dt_upd_linear_work_floats(int32_t m, int32_t n, int32_t k) {
  if (!lin_shape_ok(m, n, k)) return -1;
  return (int64_t)lin_splits(m, n, k) * m * n;
}

static bool drop_ok(const float* u, float p) {
  return !u || (aligned16(u) && p >= 0.0f && p < 1.0f);
}
static Drop drop_of(const float* u, float p, float* xd = nullptr) {
  return Drop{u, p, u ? 1.0f / (1.0f - p) : 1.0f, u ? xd : nullptr};
}

int dt_upd_linear_fwd_drop(int32_t m, int32_t n, int32_t k, const float* x, const float* u,
                           float p, float* xd, const float* w, const float* b, int32_t leaky,
                           float slope, float* y, float* work, void* stream) {
  if (!lin_shape_ok(m, n, k) || !x || !w || !y || !work || !aligned16(x) || !aligned16(w) ||
      !drop_ok(u, p) || (xd && !aligned16(xd)))
    return DT_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int splits = lin_splits(m, n, k);
  const int tiles = (n / 32) * ((m + 31) / 32);
  const int steps = k / 8, chunk = (steps + splits * kLinWaves - 1) / (splits * kLinWaves);
  hipLaunchKernelGGL(lin_fwd_kernel, dim3(tiles * splits), dim3(64 * kLinWaves), 0, s, m, n, k,
                     chunk, x, w, work, drop_of(u, p, xd));
  const int mn = m * n;
  hipLaunchKernelGGL(lin_reduce_kernel, dim3((mn + 255) / 256), dim3(256), 0, s, mn, n, splits,
                     work, b, (int)(leaky != 0), slope, y);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_upd_linear_fwd(int32_t m, int32_t n, int32_t k, const float* x, const float* w,
                      const float* b, int32_t leaky, float slope, float* y, float* work,
                      void* stream) {
  return dt_upd_linear_fwd_drop(m, n, k, x, nullptr, 0.0f, nullptr, w, b, leaky, slope, y, work,
                                stream);
}

int dt_upd_linear_dgrad_drop(int32_t m, int32_t n, int32_t k, const float* dy, const float* w,
                             const float* yact, float slope, const float* u, float p, float* dx,
                             void* stream) {
  if (!lin_shape_ok(m, n, k) || !dy || !w || !dx || !aligned16(dy) || (yact && !aligned16(yact)) ||
      !drop_ok(u, p))
    return DT_E_ARG;
  const int grid = ((m + 31) / 32) * (k / 32);
  hipLaunchKernelGGL(lin_dgrad_kernel, dim3(grid), dim3(64 * kLinWaves), 0, (hipStream_t)stream,
                     m, n, k, dy, w, yact, slope, dx, drop_of(u, p));
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_upd_linear_dgrad(int32_t m, int32_t n, int32_t k, const float* dy, const float* w,
                        const float* yact, float slope, float* dx, void* stream) {
  return dt_upd_linear_dgrad_drop(m, n, k, dy, w, yact, slope, nullptr, 0.0f, dx, stream);
}

int dt_upd_linear_wgrad(int32_t m, int32_t n, int32_t k, const float* dy, const float* x,
                        const float* yact, float slope, float* dw, float* db, void* stream) {
  if (!lin_shape_ok(m, n, k) || !dy || !x || !dw) return DT_E_ARG;
  const int tiles = (n / 32) * (k / 32);
  hipLaunchKernelGGL(lin_wgrad_kernel, dim3((tiles + kLinWaves - 1) / kLinWaves),
                     dim3(64 * kLinWaves), 0, (hipStream_t)stream, m, n, k, dy, x, yact, slope,
                     dw, db);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_upd_conv_fwd_part(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                         const float* x, const DtUpdBn* in, const float* w, const float* bias,
                         float slope, float* z, float* part, int32_t* parts, void* stream) {
  const int l = layer_of(cin, ks, st, ih, iw);
  if (!l || n < 1 || !x || !w || !bias || !z || !part || !parts) return DT_E_ARG;
  if (in && (l == 1 || !valid_in(*in))) return DT_E_ARG;
  FwdBn fb{};
  fb.bias = bias;
  fb.slope = slope;
  fb.work = part;
  hipStream_t s = (hipStream_t)stream;
  return in ? dispatch_fwd<2, true>(l, n, x, w, z, fb, *in, s, parts)
            : dispatch_fwd<2, false>(l, n, x, w, z, fb, DtUpdBn{}, s, parts);
}

int dt_upd_bn_finish(int64_t m, int32_t hw, const float* z, const DtUpdBn* bn, float* y,
                     void* stream) {
  if (m < 1 || hw < 0 || (hw > 0 && m % hw != 0) || !z || !y || !bn || !valid_in(*bn) ||
      !aligned16(z) || !aligned16(y))
    return DT_E_ARG;
  const int64_t items = m * 8;
  const int64_t per = 1024 * kFinishPer;
  int64_t grid = (items + per - 1) / per;
  grid = grid < kFinishMaxGrid ? grid : kFinishMaxGrid;
  hipLaunchKernelGGL(bn_finish_kernel, dim3((unsigned)grid), dim3(1024), 0, (hipStream_t)stream, m,
                     (int)hw, z, *bn, y);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_upd_conv_dgrad(int32_t cin, int32_t ks, int32_t st, int32_t n, int32_t ih, int32_t iw,
                      const float* dz, const float* w, float* dx, void* stream) {
  const int l = layer_of(cin, ks, st, ih, iw);
  if (l < 2 || n < 0 || (n > 0 && (!dz || !w || !dx))) return DT_E_ARG;
  if (n == 0) return DT_OK;
  hipStream_t s = (hipStream_t)stream;
  switch (l) {
    case 2: return launch_dgrad<L2, DTUPD_DG2_NW>(n, dz, w, dx, s);
    case 3: return launch_dgrad<L3, DTUPD_DG3_NW>(n, dz, w, dx, s);
    default: return launch_dgrad<L4, DTUPD_DG4_NW>(n, dz, w, dx, s);
  }
}

}  // extern "C"
