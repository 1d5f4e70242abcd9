// The actor's four convolutions at float32 accuracy on fp16 MFMA: the
// reference-precision acting path (the reference acts in float32:
// models/ddpg/model.py:79-88, duckietown_rl/ddpg.py:44-62) -- see
// include/dtactor.h (dt_conv1x_split, dt_conv32x_split).
//
// "x3": every f32 operand x is carried as an fp16 pair (hi, lo),
//   hi = fp16(x),  lo = fp16((x - hi) * 2^11),  x = hi + 2^-11 lo  (|error| <= 2^-24 |x|),
// and a product as three fp16 MFMA products accumulated in f32,
//   a * b ~ ah*bh + 2^-11 (ah*bl + al*bh)        (the dropped al*bl is ~2^-24 |a b|),
// the ah*bh products in one accumulator and the cross products in a second, so
// every operand is a normal fp16 number (an unscaled low part, ~2^-12 |w| for a
// typical weight, would sit in fp16's subnormal range).  fp16 x fp16 products
// are exact in f32, so the operands carry f32's rounding and the sums are f32
// sums: the same accuracy class as the reference's float32 convolutions, at
// 3/16 of the MFMA cycles an f32-input MFMA (v_mfma_f32_32x32x2_f32) needs.
//
// Activations between the layers are stored as such pairs in the "HLB"
// layout (struct Hlb below: per image row, 4 blocks of 8 channels x {hi, lo}
// segments, each segment the row's pixels as 16-B chunks in the CONSUMER's
// read order -- even then odd columns for a stride-2 consumer), 4 B an
// element like f32, centred on the sample's pixel 0 as in the fp16 chain
// (dtconv_common.h centre_px32).  A consumer's B-operand load is then 32
// lanes reading 512 contiguous bytes, not 32 pixels 256 B apart: the L1 tag
// lookups a load costs fell 4x (measured on the pixel-major form first).
//
// conv1x_kernel: conv1s_kernel's row stream (dtconv.hip) with a hi ring and a
//   lo ring in LDS, both weight halves in registers, three MFMAs a k step.
// conv32x_kernel: conv2..conv4.  The previous layer's per-sample BatchNorm is
//   folded into the weights once per sample (w' = w * sc[c], bias' = bias +
//   sum_k w * sh[c]) and split into hi / lo fragments in LDS (64 KB); the B
//   operand (the input's HL pairs) is read straight from global memory
//   (L2-served im2col, no LDS ring: an f32-sized ring of conv2's 77-pixel rows
//   would leave one workgroup a CU).  Four waves, one 32-pixel tile each a
//   round; the next (round, kernel row) unit's 16 loads in flight while a
//   unit's 24 MFMAs run.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "../../include/dtactor.h"
#include "dtconv_common.h"
#include "dtrender.h"   // dr::kPalGray: the grey levels of palette-index frames

// conv2 / conv3 workgroup shape: waves a workgroup (4: two workgroups a CU;
// 8: one) and units of B-operand loads in flight a wave (1: two waves a
// SIMD; 3: one wave a SIMD, 512 registers)
#ifndef DTCONVX_NW
#define DTCONVX_NW 4
#endif
#ifndef DTCONVX_DEPTH
#define DTCONVX_DEPTH 1
#endif

namespace {

using namespace dtconv;
using namespace dtconv::c1;

constexpr float kLo = 2048.0f, kLoInv = 1.0f / 2048.0f;

// x as an (hi, lo) fp16 pair in one word: hi in the low half
__device__ __forceinline__ uint32_t hl16(float x) {
  const _Float16 h = (_Float16)x;
  const _Float16 l = (_Float16)((x - (float)h) * kLo);
  return (uint32_t)__builtin_bit_cast(uint16_t, h) |
         ((uint32_t)__builtin_bit_cast(uint16_t, l) << 16);
}
// two (hi, lo) words -> their hi halves / their lo halves as fp16 pairs
__device__ __forceinline__ uint32_t hi_pair(uint32_t a, uint32_t b) {
  return (a & 0xffffu) | (b << 16);
}
__device__ __forceinline__ uint32_t lo_pair(uint32_t a, uint32_t b) {
  return (a >> 16) | (b & 0xffff0000u);
}
// (a, b) -> the fp16 pairs (hi(a), hi(b)) and (lo(a), lo(b)): packed
// conversions (v_cvt_pk_f16_f32, round to nearest even), 3 VALU a value
using f32x2 = __attribute__((ext_vector_type(2))) float;
using f16x2 = __attribute__((ext_vector_type(2))) _Float16;
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  const f32x2 x = {a, b};
  const f16x2 h = __builtin_convertvector(x, f16x2);
  const f32x2 r = (x - __builtin_convertvector(h, f32x2)) * kLo;
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, f16x2));
}

// The HLB layout of a W-wide image whose consumer reads it at stride S: a
// row is 4 channel blocks x {hi, lo} segments of kSegPx 16-B chunks (8
// channels' fp16 values); pixel x sits at chunk pos(x) of each segment, the
// even columns first, then the odd ones, when S = 2.  Row y, block cb, half
// hl (0 hi, 1 lo), pixel x: byte off(y, cb, hl, x).
template <int W_, int S>
struct Hlb {
  static constexpr int kHalf = (W_ + 1) / 2;
  static constexpr int kSegPx = S == 2 ? 2 * kHalf : W_;
  static constexpr int kSeg = kSegPx * 16;
  static constexpr int kRow = 8 * kSeg;
  __host__ __device__ static constexpr int pos(int x) {
    return S == 2 ? ((x & 1) ? kHalf + (x >> 1) : (x >> 1)) : x;
  }
  __host__ __device__ static constexpr int off(int y, int cb, int hl, int x) {
    return y * kRow + (2 * cb + hl) * kSeg + 16 * pos(x);
  }
};

// One output pixel's 32 channels into an HLB image (OW_ wide, its consumer's
// stride SN) from a 32x32 MFMA tile (lane = pixel column, register r =
// channel (r&3) + 8*(r>>2) + 4h): v_permlane32_swap pairs the two half-waves'
// 4-channel groups, so a lane holds channels 16m + 8h .. +7 = block 2m + h
// and stores it as one 16-B chunk of hi and one of lo.  Branch-free: an
// invalid lane's offset lies past the sample and the buffer store is dropped.
template <int OH_, int OW_, int SN>
__device__ __forceinline__ void store_hlb(unsigned char* sample, int oy, int ox,
                                          const float (&v)[16], int h, bool valid) {
  using L = Hlb<OW_, SN>;
  constexpr int kBytes = OH_ * L::kRow;
  uint32_t uh[4][2], ul[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 2; ++e) split2(v[4 * q + 2 * e], v[4 * q + 2 * e + 1], uh[q][e], ul[q][e]);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      auto r = __builtin_amdgcn_permlane32_swap(uh[2 * m][e], uh[2 * m + 1][e], false, false);
      uh[2 * m][e] = r[0];
      uh[2 * m + 1][e] = r[1];
      r = __builtin_amdgcn_permlane32_swap(ul[2 * m][e], ul[2 * m + 1][e], false, false);
      ul[2 * m][e] = r[0];
      ul[2 * m + 1][e] = r[1];
    }
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(sample, 0, kBytes, 0x00020000);
  const int base = valid ? L::off(oy, h, 0, ox) : kBytes;
#pragma unroll
  for (int m = 0; m < 2; ++m) {   // block 2m + h: base + 2m segments-pairs on
    const u32x4 dh = {uh[2 * m][0], uh[2 * m][1], uh[2 * m + 1][0], uh[2 * m + 1][1]};
    const u32x4 dl = {ul[2 * m][0], ul[2 * m][1], ul[2 * m + 1][0], ul[2 * m + 1][1]};
    __builtin_amdgcn_raw_buffer_store_b128(dh, rsrc, base + 4 * m * L::kSeg, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(dl, rsrc, base + (4 * m + 1) * L::kSeg, 0, 0);
  }
}

// Per-lane Welford statistics of a 32x32 tile's 16 channels merged over the
// sample: the lanes of each half (shuffles), then the waves (red, one
// barrier), written as (mean, M2, c) per channel by threads < CO.
template <int NW>
__device__ __forceinline__ void stats_flush(float& w_cnt, float (&w_mean)[16], float (&w_m2)[16],
                                            float (*red)[CO][3], const float* s_c, float* out,
                                            int tid, int wave, int col, int h) {
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) {
    const float nb = __shfl_xor(w_cnt, o, 32);
    const float tot = w_cnt + nb;
    const float fa = tot > 0.0f ? nb / tot : 0.0f, fb = tot > 0.0f ? w_cnt * nb / tot : 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float mb = __shfl_xor(w_mean[r], o, 32), m2b = __shfl_xor(w_m2[r], o, 32);
      const float d = mb - w_mean[r];
      w_mean[r] += d * fa;
      w_m2[r] += m2b + d * d * fb;
    }
    w_cnt = tot;
  }
  if (col == 0)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int c = (r & 3) + 8 * (r >> 2) + 4 * h;
      red[wave][c][0] = w_cnt;
      red[wave][c][1] = w_mean[r];
      red[wave][c][2] = w_m2[r];
    }
  __syncthreads();
  if (tid < CO) {
    float cnt = 0.0f, mean = 0.0f, m2 = 0.0f;
    for (int w = 0; w < NW; ++w) {
      const float nb = red[w][tid][0];
      if (nb <= 0.0f) continue;
      const float tot = cnt + nb, d = red[w][tid][1] - mean;
      mean += d * (nb / tot);
      m2 += red[w][tid][2] + d * d * (cnt * nb / tot);
      cnt = tot;
    }
    float* pp = out + tid * 3;
    pp[0] = mean;
    pp[1] = m2;
    pp[2] = s_c[tid];
  }
  w_cnt = 0.0f;
#pragma unroll
  for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;
}

// ---- conv1 -------------------------------------------------------------------------
constexpr int kXPxB = 6;                  // bytes a ring pixel: 3 fp16 channels (hi or lo)
constexpr int kXRowB = IW * kXPxB;        // 960 B a ring row
constexpr int kXMfma = 12, kXGrp = 3;     // k steps a tile (K 192), a B-fragment group

// kIdx: palette-index frames (u8), decoded through an 8-entry (hi, lo) table
template <bool kIdx>
__global__ void __launch_bounds__(kSThreads, 2)   // 2 waves / SIMD: <= 256 registers
conv1x_kernel(int n, const void* __restrict__ ring, int slots, int s0, int s1, int s2,
              const half8* __restrict__ wfrag, const float* __restrict__ bias,
              unsigned char* __restrict__ y, float* __restrict__ partials, float slope,
              WeightSplit ws) {
  using Elem = typename std::conditional<kIdx, uint8_t, float>::type;
  using Item = typename std::conditional<kIdx, uint32_t, float4>::type;
  const Elem* __restrict__ ringT = static_cast<const Elem*>(ring);
  __shared__ __attribute__((aligned(16))) unsigned char rbh[kSRing * kXRowB];
  __shared__ __attribute__((aligned(16))) unsigned char rbl[kSRing * kXRowB];
  __shared__ uint32_t s_hl[8];
  __shared__ float red[kSW][CO][3];
  __shared__ float s_bias[CO];
  __shared__ float s_c[CO];   // the sample's centre: its pixel-0 outputs
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, h = lane >> 5;
  const SplitPart sp = split_part(ws, n);
  if (sp.set2) {
    wfrag = static_cast<const half8*>(ws.wfrag);
    bias = ws.bias;
  }
  const int send = sp.send;
  const int total = sp.my * kSSteps;
  if (total == 0) return;
  auto sample = [&](int k) __attribute__((always_inline)) { return sp.sbeg + sp.bid + k * sp.gdim; };
  const size_t plane = (size_t)IH * IW;

  int it_r[kSPre], it_off[kSPre], it_lds[kSPre];
#pragma unroll
  for (int i = 0; i < kSPre; ++i) {
    const int q = tid + i * kSThreads;
    it_r[i] = q / kSQuads;
    it_off[i] = it_r[i] * IW + 4 * (q - it_r[i] * kSQuads);
    it_lds[i] = 4 * kXPxB * (q - it_r[i] * kSQuads);
  }
  // rows r0..r1 of the k-th sample into registers (conv1s_kernel's issue:
  // every load on every path, sample clamped, row-free steps read row 0)
  auto issue = [&](Item (&pre)[kSPre][3], int k, int r0, int r1) __attribute__((always_inline)) {
    const int rows = r1 - r0 + 1;
    const int ns = sample(k) < send ? sample(k) : send - 1;
    const Elem* base = ringT + (size_t)ns * slots * plane + (size_t)(rows > 0 ? r0 : 0) * IW;
    const Elem* p0 = base + (size_t)s0 * plane;
    const Elem* p1 = base + (size_t)s1 * plane;
    const Elem* p2 = base + (size_t)s2 * plane;
#pragma unroll
    for (int i = 0; i < kSPre; ++i) {
      const int off = it_r[i] < rows ? it_off[i] : 0;
      pre[i][0] = *reinterpret_cast<const Item*>(p0 + off);
      pre[i][1] = *reinterpret_cast<const Item*>(p1 + off);
      pre[i][2] = *reinterpret_cast<const Item*>(p2 + off);
    }
  };
  // a load item's 4 pixels of one frame as (hi, lo) words
  auto px4 = [&](const Item& it, uint32_t (&o)[4]) __attribute__((always_inline)) {
    if constexpr (kIdx) {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = s_hl[(it >> (8 * e)) & 7u];
    } else {
      o[0] = hl16(it.x);
      o[1] = hl16(it.y);
      o[2] = hl16(it.z);
      o[3] = hl16(it.w);
    }
  };
  // the rows into the hi and lo rings: 4 pixels x 3 channels pixel-major a
  // ring, row R of the stream (k * IH + r) in slot R % kSRing
  auto commit = [&](const Item (&pre)[kSPre][3], int k, int r0, int r1) __attribute__((always_inline)) {
    const int rows = r1 - r0 + 1;
#pragma unroll
    for (int i = 0; i < kSPre; ++i) {
      if (it_r[i] >= rows) continue;
      const int slot = (k * IH + r0 + it_r[i]) & (kSRing - 1);
      uint32_t av[4], bv[4], cv[4];
      px4(pre[i][0], av);
      px4(pre[i][1], bv);
      px4(pre[i][2], cv);
      const uint32_t f[12] = {av[0], bv[0], cv[0], av[1], bv[1], cv[1],
                              av[2], bv[2], cv[2], av[3], bv[3], cv[3]};
      uint2* dh = reinterpret_cast<uint2*>(rbh + slot * kXRowB + it_lds[i]);   // 8-B aligned
      uint2* dl = reinterpret_cast<uint2*>(rbl + slot * kXRowB + it_lds[i]);
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        dh[e] = make_uint2(hi_pair(f[4 * e], f[4 * e + 1]), hi_pair(f[4 * e + 2], f[4 * e + 3]));
        dl[e] = make_uint2(lo_pair(f[4 * e], f[4 * e + 1]), lo_pair(f[4 * e + 2], f[4 * e + 3]));
      }
    }
  };

  // A fragments, hi and lo halves (K 192 as conv1s_kernel: step s covers
  // kernel row 2(s/3) + h and 8 of its 24 (kx, c) values, t = 8(s%3) + j),
  // gathered once from dt_conv1's fragment layout
  half8 wah[kXMfma], wal[kXMfma];
  {
    const _Float16* wh = reinterpret_cast<const _Float16*>(wfrag);
    const _Float16* wl = wh + 16 * 64 * 8;
    const int co = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int s = 0; s < kXMfma; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ky = 2 * (s / 3) + hh, t = 8 * (s % 3) + e, kx = t / 3, c = t % 3;
        const int s1 = 2 * ky + kx / 4, l1 = co + 32 * ((kx & 3) >> 1), j1 = 4 * (kx & 1) + c;
        wah[s][e] = wh[(s1 * 64 + l1) * 8 + j1];
        wal[s][e] = wl[(s1 * 64 + l1) * 8 + j1];
      }
  }
  if (tid < CO) s_bias[tid] = bias[tid];
  if (kIdx && tid < 8) s_hl[tid] = hl16(dr::kPalGray[tid]);
  float w_cnt = 0.0f, w_mean[16], w_m2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;

  auto step = [&](int g, int k, int j, Item (&nxt)[kSPre][3], const Item (&cur)[kSPre][3]) __attribute__((always_inline)) {
    const int ns = sample(k);
    const bool last_j = j + 1 == kSSteps;
    const int k1 = last_j ? k + 1 : k, j1 = last_j ? 0 : j + 1;   // step g+1
    const int k2 = (j1 + 1 == kSSteps) ? k1 + 1 : k1;             // step g+2
    issue(nxt, k2, s_first_new(j1), s_last_new(j1));

    const int t = kSW * j + wave;
    const int p = 32 * t + col;
    const bool valid = p < kSPix;
    const int pc = valid ? p : 0;
    const int oy = pc / OW, ox = pc - oy * OW;
    const int rbase = k * IH + 2 * oy;
    const int cx = 12 * ox;
    f32x16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc0[r] = s_bias[(r & 3) + 8 * (r >> 2) + 4 * h];
      acc1[r] = 0.0f;
    }
    half8 bqh[2][kXGrp], bql[2][kXGrp];
    auto ld = [&](half8 (&bh)[kXGrp], half8 (&bl)[kXGrp], int gy) __attribute__((always_inline)) {
      using u32x4a = __attribute__((ext_vector_type(4), aligned(4))) uint32_t;
#pragma unroll
      for (int i = 0; i < kXGrp; ++i) {   // row 2gy + h, bytes 12 ox + 16 i: 4-B aligned
        const int off = ((rbase + 2 * gy + h) & (kSRing - 1)) * kXRowB + cx + 16 * i;
        bh[i] = __builtin_bit_cast(half8, *reinterpret_cast<const u32x4a*>(rbh + off));
        bl[i] = __builtin_bit_cast(half8, *reinterpret_cast<const u32x4a*>(rbl + off));
      }
    };
    ld(bqh[0], bql[0], 0);
#pragma unroll
    for (int gy = 0; gy < 4; ++gy) {
      if (gy < 3) ld(bqh[(gy + 1) & 1], bql[(gy + 1) & 1], gy + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < kXGrp; ++i) {
        const int s = kXGrp * gy + i;
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wah[s], bqh[gy & 1][i], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wah[s], bql[gy & 1][i], acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(wal[s], bqh[gy & 1][i], acc1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = lrelu2(acc0[r] + acc1[r] * kLoInv, slope);
    centre_px32(v, s_c, j == 0 && wave == 0 && col == 0, j == 0, h);
    store_hlb<OH, OW, 2>(y + (size_t)ns * OH * Hlb<OW, 2>::kRow, oy, ox, v, h, valid);
    if (valid) {   // Welford over this lane's pixels
      w_cnt += 1.0f;
      const float inv = 1.0f / w_cnt;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = v[r] - w_mean[r];
        w_mean[r] += d * inv;
        w_m2[r] += d * (v[r] - w_mean[r]);
      }
    }
    if (last_j)
      stats_flush<kSW>(w_cnt, w_mean, w_m2, red, s_c, partials + (size_t)ns * CO * 3, tid, wave,
                       col, h);
    // step g+1's rows into the rings (slots no wave reads in this step); the
    // barrier publishes them
    if (g + 1 < total) commit(cur, k1, s_first_new(j), s_last_new(j));
    __syncthreads();
  };

  Item pa[kSPre][3], pb[kSPre][3];
  issue(pa, 0, 0, s_hi(0));
  if (kIdx) __syncthreads();   // s_hl
  commit(pa, 0, 0, s_hi(0));
  if (total > 1) issue(pb, kSSteps == 1 ? 1 : 0, s_first_new(0), s_last_new(0));
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0);   // see conv1s_kernel: keeps the loop's vmcnt waits exact
  int k = 0, j = 0;
  for (int g = 0; g < total; g += 2) {
    step(g, k, j, pa, pb);
    if (++j == kSSteps) { j = 0; ++k; }
    if (g + 1 < total) {
      step(g + 1, k, j, pb, pa);
      if (++j == kSSteps) { j = 0; ++k; }
    }
  }
}

// ---- conv2..conv4 --------------------------------------------------------------------
// conv_2d(32 -> 32, 4x4, stride ST) on an HL input [IH, IW] a sample.  k step
// s (0..31) of a tile covers input pixel (ky, kx) = (s / 8, (s / 2) % 4),
// channels 16 (s % 2) + 8 h .. +7 (dt_conv32's order); a unit is one kernel
// row (8 steps, 24 MFMAs) of one round's tile.  kLast (conv4): the round holds
// the whole sample; its own BatchNorm in-kernel (exact two-pass statistics),
// written f32 flattened in NCHW order for the first linear.
template <int IH_, int IW_, int OH_, int OW_, int ST, int SN, int NW, int DEPTH, bool kLast>
__global__ void __launch_bounds__(64 * NW, (NW == 8 || DEPTH == 1) ? 2 : 1)
conv32x_kernel(int n, const unsigned char* __restrict__ x, const float* __restrict__ wsrc,
               const float* __restrict__ bias, const float* __restrict__ prev_part,
               const float* __restrict__ in_gamma, const float* __restrict__ in_beta,
               float in_eps, void* __restrict__ y, float* __restrict__ part,
               const float* __restrict__ out_gamma, const float* __restrict__ out_beta,
               float out_eps, float slope, WeightSplit ws) {
  constexpr int kPix = OH_ * OW_, kTiles = (kPix + 31) / 32, kRounds = (kTiles + NW - 1) / NW;
  constexpr int kThreads = 64 * NW;
  constexpr int kSets = DEPTH + 1;   // B-operand register sets: DEPTH units of loads in flight
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(kSets == 2 || kSets == 4, "the sets cycle within a round's 4 units");
  static_assert(NW == 4 || DEPTH == 1, "8 waves share a SIMD by two: <= 256 registers");
  using In = Hlb<IW_, ST>;           // the input as this layer reads it
  constexpr int kInBytes = IH_ * In::kRow;
  static_assert(!kLast || kRounds == 1, "the in-kernel norm needs the sample in one round");
  __shared__ half8 s_wh[32 * 64], s_wl[32 * 64];   // folded weights, hi / lo fragments
  __shared__ float s_sc[CO], s_sh[CO], s_b2[CO], s_c[CO], s_bred[kThreads / 32][CO];
  __shared__ float red[NW][CO][3];
  __shared__ float s_omean[CO], s_osc[CO], s_obeta[CO];
  __shared__ float s_wexp[2];   // 2^-e (the folded weights' scale), 2^e
  __shared__ unsigned int s_wmax;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, h = lane >> 5;
  const SplitPart sp = split_part(ws, n);
  if (sp.set2) {
    wsrc = static_cast<const float*>(ws.wfrag);
    bias = ws.bias;
    in_gamma = ws.in_gamma;
    in_beta = ws.in_beta;
    out_gamma = ws.out_gamma;
    out_beta = ws.out_beta;
  }
  if (sp.my == 0) return;
  const int send = sp.send;
  auto sample = [&](int k) __attribute__((always_inline)) {
    const int s = sp.sbeg + sp.bid + k * sp.gdim;
    return s < send ? s : send - 1;
  };

  // max |w| of the set, once a launch: with the largest |sc| of a sample it
  // bounds the folded weights, scaled by 2^-e into fp16's range when needed
  if (tid == 0) s_wmax = 0u;
  __syncthreads();
  {
    float m = 0.0f;
    const float4* w4 = reinterpret_cast<const float4*>(wsrc);
#pragma unroll 4
    for (int i = 0; i < 4096 / kThreads; ++i) {   // the 4096 float4 of the set
      const float4 q = w4[tid + kThreads * i];
      m = fmaxf(m, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fmaxf(fabsf(q.z), fabsf(q.w))));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) atomicMax(&s_wmax, __float_as_uint(m));
  }
  __syncthreads();

  // a unit's B operand: 8 k steps x (hi, lo) 16-B chunks of the lane's pixel
  // (ST ox + kx, row ST oy + ky), block 2 hf + h: In::off, its lane part in
  // the VGPR offset and the step's constant part in the SGPR offset.  Every
  // load issued, pixel and sample clamped, so every offset lies inside the
  // sample (the raw-buffer range check, which does not cover the SGPR
  // offset, is never relied on) and the vmcnt waits stay exact.
  auto unit_load = [&](u32x4 (&bh)[8], u32x4 (&bl)[8], int k, int u) __attribute__((always_inline)) {
    const int r = u >> 2, gy = u & 3;
    const int t = NW * r + wave;
    const int p = 32 * (t < kTiles ? t : 0) + col;
    const int pc = p < kPix ? p : 0;
    const int oy = pc / OW_, ox = pc - oy * OW_;
    const int vb = In::off(ST * oy + gy, h, 0, 0) + 16 * ox;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(x + (size_t)sample(k) * kInBytes), 0, kInBytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int kx = i >> 1, hf = i & 1;
      const int c = 4 * hf * In::kSeg + 16 * (ST == 2 ? In::pos(kx) : kx);
      bh[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vb, c, 0);
      bl[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vb, c + In::kSeg, 0);
    }
  };

  float w_cnt = 0.0f, w_mean[16], w_m2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;
  f32x16 acc0, acc1;
  u32x4 bh[kSets][8], bl[kSets][8];   // the B operands of kSets units (hi, lo)
  constexpr int kUnits = 4 * kRounds;

  // one unit: issue unit u + DEPTH's loads into its set, run this one's MFMAs
  // on set u % kSets; the tile's epilogue after its last kernel row.  `cur`
  // and `nxt` are compile-time set indices (the rounds are unrolled by 4).
  auto unit = [&](int k, int u, u32x4 (&ch)[8], u32x4 (&cl)[8], u32x4 (&nh)[8],
                  u32x4 (&nl)[8]) __attribute__((always_inline)) {
    const int un = u + DEPTH;
    unit_load(nh, nl, un >= kUnits ? k + 1 : k, un >= kUnits ? un - kUnits : un);
    const int r = u >> 2, gy = u & 3;
    const int t = NW * r + wave;
    if (gy == 0) {
#pragma unroll
      for (int q = 0; q < 16; ++q) acc0[q] = acc1[q] = 0.0f;
    }
    if (t < kTiles) {   // wave-uniform
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int s = 8 * gy + i;
        const half8 ah = s_wh[s * 64 + lane], al = s_wl[s * 64 + lane];
        const half8 xh = __builtin_bit_cast(half8, ch[i]), xl = __builtin_bit_cast(half8, cl[i]);
        acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xh, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xl, acc1, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, xh, acc1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (gy != 3) return;
    // epilogue of round r's tile
    const int ns = sample(k);
    if (r == 0) __syncthreads();   // s_b2 (threads < CO, after the weight barrier)
    const float isc = s_wexp[1];
    const int p = 32 * t + col;
    const bool valid = t < kTiles && p < kPix;
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q)
      v[q] = lrelu2((acc0[q] + acc1[q] * kLoInv) * isc + s_b2[(q & 3) + 8 * (q >> 2) + 4 * h],
                    slope);
    if constexpr (!kLast) {
      centre_px32(v, s_c, r == 0 && wave == 0 && col == 0, r == 0, h);
      const int pc = valid ? p : 0, oy = pc / OW_;
      store_hlb<OH_, OW_, SN>(static_cast<unsigned char*>(y) + (size_t)ns * OH_ * Hlb<OW_, SN>::kRow,
                              oy, pc - oy * OW_, v, h, valid);
      if (valid) {
        w_cnt += 1.0f;
        const float inv = 1.0f / w_cnt;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const float d = v[q] - w_mean[q];
          w_mean[q] += d * inv;
          w_m2[q] += d * (v[q] - w_mean[q]);
        }
      }
      if (r + 1 == kRounds)
        stats_flush<NW>(w_cnt, w_mean, w_m2, red, s_c, part + (size_t)ns * CO * 3, tid, wave, col,
                       h);
    } else {
      // exact two-pass statistics: per wave over its 32 pixels (shuffles),
      // the waves merged with Chan's formula by threads < CO
      float nw = valid ? 1.0f : 0.0f;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) nw += __shfl_xor(nw, o, 32);
      const float inw = nw > 0.0f ? 1.0f / nw : 0.0f;
      float sum[16], m2[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) sum[q] = valid ? v[q] : 0.0f;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1)
#pragma unroll
        for (int q = 0; q < 16; ++q) sum[q] += __shfl_xor(sum[q], o, 32);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const float d = valid ? v[q] - sum[q] * inw : 0.0f;
        m2[q] = d * d;
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1)
#pragma unroll
        for (int q = 0; q < 16; ++q) m2[q] += __shfl_xor(m2[q], o, 32);
      if (col == 0)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int c = (q & 3) + 8 * (q >> 2) + 4 * h;
          red[wave][c][0] = nw;
          red[wave][c][1] = sum[q] * inw;
          red[wave][c][2] = m2[q];
        }
      __syncthreads();
      if (tid < CO) {
        float cnt = 0.0f, mean = 0.0f, mm = 0.0f;
        for (int w = 0; w < NW; ++w) {
          const float nb = red[w][tid][0];
          if (nb <= 0.0f) continue;
          const float tot = cnt + nb, d = red[w][tid][1] - mean;
          mean += d * (nb / tot);
          mm += red[w][tid][2] + d * d * (cnt * nb / tot);
          cnt = tot;
        }
        s_omean[tid] = mean;
        s_osc[tid] = out_gamma[tid] / sqrtf(mm / (float)kPix + out_eps);
        s_obeta[tid] = out_beta[tid];
      }
      __syncthreads();
      constexpr int kBytes = kPix * CO * 4;
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
          static_cast<float*>(y) + (size_t)ns * CO * kPix, 0, kBytes, 0x00020000);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int c = (q & 3) + 8 * (q >> 2) + 4 * h;
        const float o = (v[q] - s_omean[c]) * s_osc[c] + s_obeta[c];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), rsrc,
                                              valid ? (c * kPix + p) * 4 : kBytes, 0, 0);
      }
    }
  };

#pragma unroll
  for (int d = 0; d < DEPTH; ++d) unit_load(bh[d], bl[d], d >= kUnits ? 1 : 0, d % kUnits);
  for (int k = 0; k < sp.my; ++k) {
    const int ns = sample(k);
    // (a) the input's BatchNorm (per sample, batch of one) and the weight scale
    if (tid < CO) {
      const float* pp = prev_part + ((size_t)ns * CO + tid) * 3;
      const float mean = pp[0], m2 = pp[1];
      const float sc = in_gamma[tid] / sqrtf(m2 / (float)(IH_ * IW_) + in_eps);
      s_sc[tid] = sc;
      s_sh[tid] = in_beta[tid] - mean * sc;
      float a = fabsf(sc);
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 32));
      if (tid == 0) {
        const float bound = a * __uint_as_float(s_wmax);
        int e = 0;
        if (bound > 16384.0f && bound < __builtin_inff()) (void)frexpf(bound * (1.0f / 16384.0f), &e);
        s_wexp[0] = ldexpf(1.0f, -e);
        s_wexp[1] = ldexpf(1.0f, e);
      }
    }
    __syncthreads();
    // (b) the folded weights: A fragment (s, l) holds w[l % 32][16 (s % 2) +
    // 8 (l / 32) + j][(s / 2) / 4][(s / 2) % 4]; thread tid folds fragments
    // tid + kThreads i, all of output channel tid % 32, and sums its share of
    // sum_k w * sh for bias'
    {
      const float wsc = s_wexp[0];
      float bacc = 0.0f;
#pragma unroll 2
      for (int i = 0; i < 2048 / kThreads; ++i) {
        const int pidx = tid + kThreads * i, s = pidx >> 6, l = pidx & 63;
        const float4* src = reinterpret_cast<const float4*>(wsrc) + 2 * pidx;
        const float4 q0 = src[0], q1 = src[1];
        const float wv[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        const int ci0 = 16 * (s & 1) + 8 * (l >> 5);
        half8 hh, ll;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float t = wv[j] * s_sc[ci0 + j] * wsc;
          const _Float16 th = (_Float16)t;
          hh[j] = th;
          ll[j] = (_Float16)((t - (float)th) * kLo);
          bacc += wv[j] * s_sh[ci0 + j];
        }
        s_wh[pidx] = hh;
        s_wl[pidx] = ll;
      }
      s_bred[tid >> 5][tid & 31] = bacc;
    }
    __syncthreads();
    if (tid < CO) {
      float b2 = bias[tid];
#pragma unroll
      for (int m = 0; m < kThreads / 32; ++m) b2 += s_bred[m][tid];
      s_b2[tid] = b2;
    }
    // (c) the rounds: units alternate between the two register sets
#pragma unroll 1
    for (int r = 0; r < kRounds; ++r) {
#pragma unroll
      for (int gy = 0; gy < 4; ++gy)
        unit(k, 4 * r + gy, bh[gy % kSets], bl[gy % kSets], bh[(gy + DEPTH) % kSets],
             bl[(gy + DEPTH) % kSets]);
    }
  }
}

template <int IH_, int IW_, int OH_, int OW_, int ST, int SN, int NW, int DEPTH, bool kLast>
int launch_conv32x(int n, const void* x, const float* w, const float* bias, const float* pp,
                   const float* ig, const float* ib, float ieps, void* y, float* part,
                   const float* og, const float* ob, float oeps, float slope, hipStream_t s,
                   WeightSplit ws, int n0) {
  auto kern = conv32x_kernel<IH_, IW_, OH_, OW_, ST, SN, NW, DEPTH, kLast>;
  static int grid = 0;   // resident workgroups, persistent
  if (!grid) grid = resident_grid(kern, 64 * NW, 0);
  const int g = split_grid(ws, n, n0, grid);
  hipLaunchKernelGGL(kern, dim3(g), dim3(64 * NW), 0, s, n, (const unsigned char*)x, w, bias, pp, ig,
                     ib, ieps, y, part, og, ob, oeps, slope, ws);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// ---- the output branch: lin1 (4032 -> 512) + LeakyReLU + lin2 (512 -> 2) + head --------
// x3 like the convolutions: C[feature][sample] = W1 . x^T on fp16 MFMA with
// A = lin1's weights as pre-split (hi, lo) fragments (feature rows), B = the
// samples' flattened activations (f32, split as they are loaded).
// head_lin1_kernel: a workgroup owns 64 samples, all 512 features and a
//   quarter of K (8 waves, 2 feature tiles x 2 sample tiles each), so lin1's
//   8 MB of fragments are streamed once per 64 samples rather than per 32
//   (a one-pass form with 32 samples a workgroup took 213 us at 4096
//   samples, streaming them); it writes its partial sums [part][feature][row].
// head_finish_kernel: the four partials + bias, LeakyReLU, lin2, the head;
//   four lanes a sample, 128 features each.  Summation order is fixed:
//   deterministic.
constexpr int kHFeat = 512, kHK = 4032, kHSteps = kHK / 16;   // 252 k steps
constexpr int kHWaves = 8, kHParts = 4, kHPartSteps = kHSteps / kHParts;   // 63
constexpr int kHRows = 64;                                                 // samples a workgroup
static_assert(kHSteps % kHParts == 0, "K split");

__device__ __forceinline__ float head_act(float v, int head) {
  if (head == 1) return tanhf(v);
  if (head == 2) return 1.0f / (1.0f + expf(-v));
  return v;
}

// the workgroup's rows: tiles of kHRows, the first set's [0, n0) then the second's
struct HeadTile {
  bool set2;
  int rbeg, rend;
};
__device__ __forceinline__ HeadTile head_tile(int b, int n, int n0) {
  const int t1 = (n0 + kHRows - 1) / kHRows;
  HeadTile t;
  t.set2 = b >= t1;
  t.rbeg = t.set2 ? n0 + kHRows * (b - t1) : kHRows * b;
  t.rend = t.set2 ? n : n0;
  return t;
}

// The head's dropout (reference mode: F.dropout(flatten, p) before lin1),
// folded into lin1's staging: element (row, k) is kept where u >= p, u a
// 16-bit uniform in [0, 1) from a counter-based hash of (seed, row * K + k)
// (lowbias32, two rounds keyed by the seed; one hash a pair of elements),
// then scaled by 1 / (1 - p) -- F.dropout's bernoulli(1 - p) mask and scale
// with its own generator instead of torch's stream.
__device__ __forceinline__ uint32_t drop_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
struct HeadDrop {
  float p, scale;   // p == 0: no dropout
  uint32_t seed;
};

// XCD-aware order (blocks are dealt round-robin over the 8 XCDs, so b and
// b + 8 share one): block b works K quarter (b % 8) / 2, so each XCD's L2
// holds one quarter of lin1's fragments (2 MB) for all its workgroups; the
// grid is padded to a multiple of 8, the spare blocks exit.
// The workgroup's 64 x-rows are staged through LDS a stage of kHStage k steps
// at a time -- loaded from HBM once, dropped out and split into (hi, lo) once,
// instead of by each of the 8 waves (which read the same rows: 8x the L1
// traffic and the split VALU) -- double-buffered, one barrier a stage.
constexpr int kHStage = 3;                         // k steps a stage (63 = 21 x 3)
constexpr int kHStages = kHPartSteps / kHStage;
constexpr int kHStageK = 16 * kHStage;             // 48 k
constexpr int kHRowH = kHStageK + 8;               // halves a staged row (112 B: conflict-free b128 reads)
constexpr int kHChunks = kHStageK / 8;             // 8-k chunks a row
static_assert(kHPartSteps % kHStage == 0, "whole stages");
static_assert(kHRows * kHChunks <= 64 * kHWaves, "a chunk a thread");
// lin1's weight fragments are loaded kNB - 1 k steps ahead of their MFMAs
// into kNB register buffers, step s in buffer s % kNB; the stage loop runs
// kU stages an iteration so that index is a compile-time constant.  x3 holds
// hi and lo fragments (16 registers a buffer): 4 buffers fit its 256.
#ifndef DTHEAD_NB
#define DTHEAD_NB 4
#endif
#ifndef DTHEAD_NB16
#define DTHEAD_NB16 6
#endif
__host__ __device__ constexpr int head_gcd(int a, int b) { return b ? head_gcd(b, a % b) : a; }
template <bool kX3> struct HeadPf {
  static constexpr int kNB = kX3 ? DTHEAD_NB : DTHEAD_NB16;
  static constexpr int kWpf = kNB - 1;
  static constexpr int kU = kNB / head_gcd(kNB, kHStage);   // stages an iteration
  static_assert(kNB >= 2 && kNB <= 12, "register buffers");
};
template <typename F, int... J>
__device__ __forceinline__ void head_stages(F&& f, int g, std::integer_sequence<int, J...>) {
  (f(g + J, std::integral_constant<int, J>{}), ...);
}

// kX3: x f32, its products as three fp16 MFMAs on (hi, lo) pairs; else the
// fp16 fast mode: x fp16, one MFMA a product (the fragments' hi half only)
template <bool kX3>
__global__ void __launch_bounds__(64 * kHWaves, 2)
head_lin1_kernel(int n, int n0, int ldp, int tiles, const void* __restrict__ xv,
                 const half8* __restrict__ w1a, const half8* __restrict__ w1b,
                 float* __restrict__ part, HeadDrop dr) {
  __shared__ __attribute__((aligned(16))) _Float16 xs[2][2][kHRows * kHRowH];   // [buf][hi, lo]
  const int b = blockIdx.x, xcd = b & 7;
  const int kp = xcd >> 1;                        // the K quarter
  const int tile = (b >> 3) * 2 + (xcd & 1);
  if (tile >= tiles) return;
  const HeadTile ht = head_tile(tile, n, n0);
  const half8* __restrict__ w1 = ht.set2 ? w1b : w1a;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, h = lane >> 5;
  // staging: thread tid < 64 * 6 owns row tid / 6, chunk tid % 6 of a stage
  const bool stager = tid < kHRows * kHChunks;
  const int srow = tid / kHChunks, schunk = tid - srow * kHChunks;
  const int grow = ht.rbeg + srow;                 // the global sample row
  const bool rvalid = stager && grow < ht.rend;
  const size_t xoff = (size_t)(rvalid ? grow : ht.rbeg) * kHK + 16 * kHPartSteps * kp + 8 * schunk;
  float4 xq[2];   // kX3: 8 floats; fp16: 8 halves in xq[0]
  auto stage_load = [&](int g) __attribute__((always_inline)) {
    if (!stager) return;
    if constexpr (kX3) {
      const float4* xsrc = reinterpret_cast<const float4*>(static_cast<const float*>(xv) + xoff);
      xq[0] = xsrc[(kHStageK / 4) * g];
      xq[1] = xsrc[(kHStageK / 4) * g + 1];
    } else {
      const float4* xsrc =
          reinterpret_cast<const float4*>(static_cast<const _Float16*>(xv) + xoff);
      xq[0] = xsrc[(kHStageK / 8) * g];
    }
  };
  auto stage_store = [&](int g, int buf) __attribute__((always_inline)) {
    if (!stager) return;
    float v[8];
    if constexpr (kX3) {
      v[0] = xq[0].x, v[1] = xq[0].y, v[2] = xq[0].z, v[3] = xq[0].w;
      v[4] = xq[1].x, v[5] = xq[1].y, v[6] = xq[1].z, v[7] = xq[1].w;
    } else {
      const half8 hv = __builtin_bit_cast(half8, xq[0]);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)hv[j];
    }
    if (dr.p > 0.0f) {
      // one hash a pair of elements, 16 bits each: u = h16 / 2^16
      const uint32_t k0 = 16 * kHPartSteps * kp + kHStageK * g + 8 * schunk;
      const uint32_t base = (uint32_t)grow * (uint32_t)kHK + k0;
      const uint32_t mix = drop_hash(dr.seed ^ 0x9e3779b9u);
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        const uint32_t hh = drop_hash(drop_hash((base + j) ^ mix) + dr.seed);
        const float u0 = (float)(hh & 0xffffu) * (1.0f / 65536.0f);
        const float u1 = (float)(hh >> 16) * (1.0f / 65536.0f);
        v[j] = u0 >= dr.p ? v[j] * dr.scale : 0.0f;
        v[j + 1] = u1 >= dr.p ? v[j + 1] * dr.scale : 0.0f;
      }
    }
    const int at = srow * kHRowH + 8 * schunk;
    if constexpr (kX3) {
      uint32_t hi[4], lo[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) split2(v[2 * e], v[2 * e + 1], hi[e], lo[e]);
      *reinterpret_cast<u32x4*>(&xs[buf][0][at]) = u32x4{hi[0], hi[1], hi[2], hi[3]};
      *reinterpret_cast<u32x4*>(&xs[buf][1][at]) = u32x4{lo[0], lo[1], lo[2], lo[3]};
    } else {
      half8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) hv[j] = (_Float16)v[j];
      *reinterpret_cast<half8*>(&xs[buf][0][at]) = hv;
    }
  };
  // w1 fragments: [2 (hi, lo)][16 feature tiles][252 k steps][64 lanes]
  constexpr int kHalfFrag = 16 * kHSteps * 64;
  const half8* wt[2];
#pragma unroll
  for (int c = 0; c < 2; ++c)
    wt[c] = w1 + ((size_t)(2 * wave + c) * kHSteps + kHPartSteps * kp) * 64 + lane;
  f32x16 acc0[2][2], acc1[2][2];   // [feature tile][sample tile]
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc0[c][st][r] = acc1[c][st][r] = 0.0f;
  constexpr int kNB = HeadPf<kX3>::kNB, kWpf = HeadPf<kX3>::kWpf;
  half8 ah[kNB][2], al[kX3 ? kNB : 1][2];   // [buffer = step % kNB][feature tile]
  auto wload = [&](int bb, int s) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      ah[bb][c] = wt[c][s * 64];
      if constexpr (kX3) al[kX3 ? bb : 0][c] = wt[c][kHalfFrag + s * 64];
    }
  };
  // step ss of stage buffer `buf` on weight buffer bb: B = the staged rows
  // (lane: sample col of each tile, k 16 ss + 8 h .. + 7)
  auto step = [&](int buf, int ss, int bb) __attribute__((always_inline)) {
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int at = (32 * st + col) * kHRowH + 16 * ss + 8 * h;
      const half8 xh = *reinterpret_cast<const half8*>(&xs[buf][0][at]);
#pragma unroll
      for (int c = 0; c < 2; ++c)
        acc0[c][st] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[bb][c], xh, acc0[c][st], 0, 0, 0);
      if constexpr (kX3) {
        const half8 xl = *reinterpret_cast<const half8*>(&xs[buf][1][at]);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          acc1[c][st] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[bb][c], xl, acc1[c][st], 0, 0, 0);
          acc1[c][st] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[kX3 ? bb : 0][c], xh, acc1[c][st], 0, 0, 0);
        }
      }
    }
  };
  stage_load(0);
#pragma unroll
  for (int s = 0; s < kWpf; ++s) wload(s % kNB, s);
  stage_store(0, 0);
  __syncthreads();
  // stage g = kU i + PAR: step s = 3 g + ss sits in register buffer
  // (3 PAR + ss) % kNB (kU stages are a multiple of kNB steps), its rows in
  // LDS buffer g & 1
  constexpr int kU = HeadPf<kX3>::kU;
  auto stage = [&](int g, auto par) __attribute__((always_inline)) {
    constexpr int PAR = decltype(par)::value;
    if (g + 1 < kHStages) stage_load(g + 1);      // in flight during this stage's MFMAs
#pragma unroll
    for (int ss = 0; ss < kHStage; ++ss) {
      const int s = kHStage * g + ss;              // the quarter's k step
      if (s + kWpf < kHPartSteps) wload((kHStage * PAR + ss + kWpf) % kNB, s + kWpf);
      step(g & 1, ss, (kHStage * PAR + ss) % kNB);
    }
    if (g + 1 < kHStages) stage_store(g + 1, (g & 1) ^ 1);
    __syncthreads();
  };
  int g = 0;
  for (; g + kU <= kHStages; g += kU) head_stages(stage, g, std::make_integer_sequence<int, kU>{});
  head_stages(stage, g, std::make_integer_sequence<int, kHStages % kU>{});
  // partial sums [part][feature][row]: lanes of a half-wave are 32 consecutive rows
  float* pp = part + (size_t)kp * kHFeat * ldp;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int row = ht.rbeg + 32 * st + col;
      if (row < ht.rend)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int f = 32 * (2 * wave + c) + (r & 3) + 8 * (r >> 2) + 4 * h;
          pp[(size_t)f * ldp + row] = kX3 ? acc0[c][st][r] + acc1[c][st][r] * kLoInv : acc0[c][st][r];
        }
    }
}

// 16 rows a workgroup, 16 lanes a row (consecutive lanes: consecutive rows,
// so a load is 16 consecutive floats of one feature); lane g of a row sums
// features g, g + 16, ... (32), the 16 partial dot products of a row reduced
// in LDS in a fixed order
// T: the head's parameters as the actor keeps them (f32, or fp16 in fast mode)
template <typename T>
__global__ void __launch_bounds__(256)
head_finish_kernel(int n, int n0, int ldp, const float* __restrict__ part,
                   const T* __restrict__ b1a, const T* __restrict__ w2a,
                   const T* __restrict__ b2a, const T* __restrict__ b1b,
                   const T* __restrict__ w2b, const T* __restrict__ b2b, int head,
                   float slope, float* __restrict__ out) {
  __shared__ float red[16][16][2];
  const int tid = threadIdx.x, g = tid >> 4, rr = tid & 15;
  const int row = 16 * blockIdx.x + rr;
  const bool valid = row < n;
  const int rc = valid ? row : 0;
  const bool set2 = rc >= n0;
  const T* __restrict__ b1 = set2 ? b1b : b1a;
  const T* __restrict__ w2 = set2 ? w2b : w2a;
  float p0 = 0.0f, p1 = 0.0f;
#pragma unroll 4
  for (int f = g; f < kHFeat; f += 16) {
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < kHParts; ++k) a += part[((size_t)k * kHFeat + f) * ldp + rc];
    const float v = lrelu2(a + (float)b1[f], slope);
    p0 = fmaf(v, (float)w2[f], p0);
    p1 = fmaf(v, (float)w2[kHFeat + f], p1);
  }
  red[rr][g][0] = p0;
  red[rr][g][1] = p1;
  __syncthreads();
  if (tid < 32) {
    const int r2 = tid >> 1, j = tid & 1;
    const int orow = 16 * blockIdx.x + r2;
    if (orow < n) {
      const T* __restrict__ b2 = orow >= n0 ? b2b : b2a;
      float a = (float)b2[j];
#pragma unroll
      for (int q = 0; q < 16; ++q) a += red[r2][q][j];
      out[(size_t)orow * 2 + j] = head_act(a, head);
    }
  }
}

template <bool kIdx>
int conv1x_launch(const void* ring, int32_t n, int32_t slots, const int32_t* order,
                  const void* wfrag, const float* bias, const dt_conv_set* set2, void* y,
                  float* partials, float slope, void* stream) {
  if (!ring || !wfrag || !bias || !y || !partials || !order || n < 0 || slots < 3) return DT_E_ARG;
  for (int i = 0; i < 3; ++i)
    if (order[i] < 0 || order[i] >= slots) return DT_E_ARG;
  if (set2 && (set2->n0 < 0 || set2->n0 > n || !set2->wfrag || !set2->bias)) return DT_E_ARG;
  if (n == 0) return DT_OK;
  static int grid = 0;
  if (!grid) grid = resident_grid(conv1x_kernel<kIdx>, kSThreads, 0);
  WeightSplit ws{};
  if (set2) {
    ws.wfrag = set2->wfrag;
    ws.bias = set2->bias;
  }
  const int g = split_grid(ws, n, set2 ? set2->n0 : n, grid);
  hipLaunchKernelGGL((conv1x_kernel<kIdx>), dim3(g), dim3(kSThreads), 0, (hipStream_t)stream, n,
                     ring, slots, order[0], order[1], order[2], (const half8*)wfrag, bias,
                     (unsigned char*)y, partials, slope, ws);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

}  // namespace

extern "C" int dt_conv1x_split(const void* ring, int32_t index, int32_t n, int32_t slots,
                               const int32_t* order, const void* wfrag, const float* bias,
                               const dt_conv_set* set2, void* y, float* partials, float slope,
                               void* stream) {
  return index ? conv1x_launch<true>(ring, n, slots, order, wfrag, bias, set2, y, partials, slope,
                                     stream)
               : conv1x_launch<false>(ring, n, slots, order, wfrag, bias, set2, y, partials,
                                      slope, stream);
}

extern "C" int64_t dt_actor_head_x3_work_floats(int32_t n) {
  return n < 0 ? -1 : (int64_t)kHParts * kHFeat * n;
}

namespace {
template <bool kX3, typename T>
int head_launch(int32_t n, int32_t n0, int32_t k, const void* x, float p, uint32_t seed,
                const void* w1a, const T* b1a, const T* w2a, const T* b2a, const void* w1b,
                const T* b1b, const T* w2b, const T* b2b, int32_t head, float slope, float* work,
                float* out, void* stream) {
  if (!x || !w1a || !b1a || !w2a || !b2a || !work || !out || n < 0 || n0 < 0 || n0 > n ||
      k != kHK || head < 0 || head > 2 || !(p >= 0.0f && p < 1.0f))
    return DT_E_ARG;
  if (n0 < n && (!w1b || !b1b || !w2b || !b2b)) return DT_E_ARG;
  if (n == 0) return DT_OK;
  hipStream_t s = (hipStream_t)stream;
  const int tiles = (n0 + kHRows - 1) / kHRows + (n - n0 + kHRows - 1) / kHRows;
  const int blocks = 8 * ((tiles + 1) / 2);   // two tiles of each quarter an 8-block round
  const HeadDrop dr{p, p > 0.0f ? 1.0f / (1.0f - p) : 1.0f, seed};
  hipLaunchKernelGGL(head_lin1_kernel<kX3>, dim3(blocks), dim3(64 * kHWaves), 0, s, n, n0, n,
                     tiles, x, (const half8*)w1a, (const half8*)(w1b ? w1b : w1a), work, dr);
  hipLaunchKernelGGL(head_finish_kernel<T>, dim3((n + 15) / 16), dim3(256), 0, s, n, n0, n,
                     work, b1a, w2a, b2a, b1b ? b1b : b1a, w2b ? w2b : w2a, b2b ? b2b : b2a,
                     head, slope, out);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}
}  // namespace

extern "C" int dt_actor_head_x3_drop(int32_t n, int32_t n0, int32_t k, const float* x,
                                     float p, uint32_t seed, const void* w1a, const float* b1a,
                                     const float* w2a, const float* b2a, const void* w1b,
                                     const float* b1b, const float* w2b, const float* b2b,
                                     int32_t head, float slope, float* work, float* out,
                                     void* stream) {
  return head_launch<true, float>(n, n0, k, x, p, seed, w1a, b1a, w2a, b2a, w1b, b1b, w2b, b2b,
                                  head, slope, work, out, stream);
}

extern "C" int dt_actor_head_f16_drop(int32_t n, int32_t n0, int32_t k, const void* x, float p,
                                      uint32_t seed, const void* w1a, const void* b1a,
                                      const void* w2a, const void* b2a, const void* w1b,
                                      const void* b1b, const void* w2b, const void* b2b,
                                      int32_t head, float slope, float* work, float* out,
                                      void* stream) {
  using H = _Float16;
  return head_launch<false, H>(n, n0, k, x, p, seed, w1a, (const H*)b1a, (const H*)w2a,
                               (const H*)b2a, w1b, (const H*)b1b, (const H*)w2b, (const H*)b2b,
                               head, slope, work, out, stream);
}

extern "C" int dt_actor_head_x3(int32_t n, int32_t n0, int32_t k, const float* x,
                                const void* w1a, const float* b1a, const float* w2a,
                                const float* b2a, const void* w1b, const float* b1b,
                                const float* w2b, const float* b2b, int32_t head, float slope,
                                float* work, float* out, void* stream) {
  return dt_actor_head_x3_drop(n, n0, k, x, 0.0f, 0u, w1a, b1a, w2a, b2a, w1b, b1b, w2b, b2b,
                               head, slope, work, out, stream);
}

extern "C" int dt_conv32x_split(int32_t layer, int32_t n, const void* x, const float* wfrag,
                                const float* bias, const float* prev_part, const float* in_gamma,
                                const float* in_beta, float in_eps, void* y, float* part,
                                const float* out_gamma, const float* out_beta, float out_eps,
                                float slope, const dt_conv_set* set2, void* stream) {
  if (!x || !wfrag || !bias || !y || !prev_part || !in_gamma || !in_beta || n < 0) return DT_E_ARG;
  const bool last = layer == 4;
  if (last ? (!out_gamma || !out_beta) : !part) return DT_E_ARG;
  if (set2 && (set2->n0 < 0 || set2->n0 > n || !set2->wfrag || !set2->bias || !set2->in_gamma ||
               !set2->in_beta || (last && (!set2->out_gamma || !set2->out_beta))))
    return DT_E_ARG;
  if (n == 0) return DT_OK;
  WeightSplit ws{};
  if (set2) {
    ws.wfrag = set2->wfrag;
    ws.bias = set2->bias;
    ws.in_gamma = set2->in_gamma;
    ws.in_beta = set2->in_beta;
    ws.out_gamma = set2->out_gamma;
    ws.out_beta = set2->out_beta;
  }
  const int n0 = set2 ? set2->n0 : n;
  hipStream_t s = (hipStream_t)stream;
  switch (layer) {
    case 2:
      return launch_conv32x<57, 77, 27, 37, 2, 2, DTCONVX_NW, DTCONVX_DEPTH, false>(n, x, wfrag, bias, prev_part, in_gamma,
                                                      in_beta, in_eps, y, part, nullptr, nullptr,
                                                      0.f, slope, s, ws, n0);
    case 3:
      return launch_conv32x<27, 37, 12, 17, 2, 1, DTCONVX_NW, DTCONVX_DEPTH, false>(n, x, wfrag, bias, prev_part, in_gamma,
                                                      in_beta, in_eps, y, part, nullptr, nullptr,
                                                      0.f, slope, s, ws, n0);
    case 4:
      return launch_conv32x<12, 17, 9, 14, 1, 1, 4, DTCONVX_DEPTH, true>(n, x, wfrag, bias, prev_part, in_gamma,
                                                    in_beta, in_eps, y, nullptr, out_gamma,
                                                    out_beta, out_eps, slope, s, ws, n0);
    default:
      return DT_E_ARG;
  }
}
