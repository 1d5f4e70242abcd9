// The actor's first convolution (config.json actor: conv_2d 3 -> 32, 8x8,
// stride 2, then leaky_relu) as a gfx950 MFMA implicit GEMM that reads the
// observation ring in place, and conv2..conv4 (conv_2d 32 -> 32, 4x4) -- see
// include/dtactor.h (dt_conv1, dt_conv1_norm, dt_conv32).
//
// conv1s_kernel: persistent workgroups stream whole samples; the input rows go
// through an LDS ring as fp16 pixels; tiles of 32 output pixels x 32 channels
// with v_mfma_f32_32x32x16_f16 (A = weights, row = out channel; B = the im2col
// column of a pixel); out = bias + LeakyReLU as fp16 NHWC, and in reference
// mode the per-sample BatchNorm statistics (count / mean / M2 per channel).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "../../include/dtactor.h"
#include "dtconv_common.h"
#include "dtrender.h"   // dr::kPalGray: the grey levels of palette-index frames

// diagnostic builds only (tools/conv32_micro.py): bit 0 skips the prefetch
// loads, 1 the MFMA section, 2 the output stores, 3 the statistics, 4 the ring
// commit; the product build is 0
#ifdef DTCONV_STAMPS   // diagnostic: shader-clock stamps inside the steps of the layer whose input height is DTCONV_STAMPS (57: conv2, 27: conv3, 12: conv4)
__device__ unsigned long long g_cstamps[8 * 2 * 48 * 8];
#define CSTAMP(i)                                                                          \
  do {                                                                                     \
    if (IH == DTCONV_STAMPS && (threadIdx.x & 63) == 0 && threadIdx.x < 128 && blockIdx.x < 8 && \
        g < 48)                                                                            \
      g_cstamps[((blockIdx.x * 2 + (threadIdx.x >> 6)) * 48 + g) * 8 + (i)] =              \
          __builtin_amdgcn_s_memtime();                                                    \
  } while (0)
#else
#define CSTAMP(i) \
  do {            \
  } while (0)
#endif
#ifdef DTCONV1_STAMPS   // diagnostic: the same stamps inside conv1s_kernel's steps
__device__ unsigned long long g_c1stamps[8 * 2 * 48 * 8];
#define C1STAMP(i)                                                                         \
  do {                                                                                     \
    if ((threadIdx.x & 63) == 0 && threadIdx.x < 128 && blockIdx.x < 8 && g < 48)         \
      g_c1stamps[((blockIdx.x * 2 + (threadIdx.x >> 6)) * 48 + g) * 8 + (i)] =             \
          __builtin_amdgcn_s_memtime();                                                    \
  } while (0)
#else
#define C1STAMP(i) \
  do {             \
  } while (0)
#endif
#ifndef DTCONV_SKIP
#define DTCONV_SKIP 0
#endif
// conv1s_kernel: B-fragment groups in flight, 2..4
#ifndef DTCONV1_BDEPTH
#define DTCONV1_BDEPTH 2
#endif
// conv1s_kernel's reduction layout: 1 = K 192 (3-channel pixels, 12 MFMAs a
// tile), 0 = K 256 (4-channel pixels with a zero channel, 16 MFMAs a tile)
#ifndef DTCONV1_K192
#define DTCONV1_K192 1
#endif
// conv1s_kernel: resident workgroups a CU of the persistent grid; 0 = as many
// as the occupancy allows (diagnostic builds fix it)
#ifndef DTCONV1_PER
#define DTCONV1_PER 0
#endif

namespace {

using namespace dtconv;
using namespace dtconv::c1;

// One pixel's 32 channels as fp16 NHWC from a 32x32x16 MFMA tile (lane = pixel
// column, register r = channel (r&3) + 8*(r>>2) + 4h): v_permlane32_swap pairs
// the two half-waves' 4-channel groups, so each lane stores two 16-B chunks
// (channels 16m + 8h .. +7 at byte 32m + 16h) instead of four 8-B ones.
// `sample` is the sample's first element (wave-uniform), `px` the lane's pixel.
// Branch-free: the stores are buffer stores over the sample's bytes and an
// invalid lane's offset lies past them (the hardware drops it), so every path
// issues the same memory instructions and the compiler's vmcnt waits for the
// next prefetch stay exact (an `if (valid)` around the stores made them wait
// for the stores too).
template <int kPix>
__device__ __forceinline__ void store_px32(__half* sample, int px, const float (&v)[16], int h,
                                           bool valid) {
  constexpr int kBytes = kPix * 32 * 2;
  uint32_t u[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const __half2 v0 = __floats2half2_rn(v[4 * q + 0], v[4 * q + 1]);
    const __half2 v1 = __floats2half2_rn(v[4 * q + 2], v[4 * q + 3]);
    u[q][0] = *reinterpret_cast<const uint32_t*>(&v0);
    u[q][1] = *reinterpret_cast<const uint32_t*>(&v1);
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const auto r = __builtin_amdgcn_permlane32_swap(u[2 * m][e], u[2 * m + 1][e], false, false);
      u[2 * m][e] = r[0];
      u[2 * m + 1][e] = r[1];
    }
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(sample), 0, kBytes,
                                                      0x00020000);
  const int off = valid ? px * 64 + 16 * h : kBytes;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const u32x4 d = {u[2 * m][0], u[2 * m][1], u[2 * m + 1][0], u[2 * m + 1][1]};
    __builtin_amdgcn_raw_buffer_store_b128(d, rsrc, off + 32 * m, 0, 0);
  }
}

// ---- conv1 ----------------------------------------------------------------------
// A persistent workgroup of kSW waves streams whole samples (n = blockIdx.x,
// + gridDim.x, ...).  The input rows go through a ring of kSRing rows in LDS
// (fp16 pixels), each row read from HBM once per sample.  A step is kSW tiles
// of 32 consecutive output pixels, one per wave; while a step's MFMAs run, the
// rows of the step after next are in flight into registers, and the next
// step's rows (loaded a step earlier) are converted into the ring after the
// epilogue: one barrier per step (conv32_kernel's schedule).  Two workgroups
// per CU, so one's barrier leaves the other's MFMAs running.  Reference mode:
// per-lane Welford statistics over the sample, merged (Chan) into ONE
// (mean, M2) per sample and channel.
constexpr bool kK192 = DTCONV1_K192 != 0;
constexpr int kSPxB = kK192 ? 6 : 8;                    // bytes a ring pixel: fp16 x 3 (x 4)
constexpr int kSRowB = IW * kSPxB;                      // 960 (1280) B
constexpr int kSMfma = kK192 ? 12 : 16;                 // MFMAs a tile
constexpr int kSGrp = kK192 ? 3 : 4;                    // MFMAs a B-fragment group
#ifdef DTCONV_CHECK
// Bounds-checked diagnostic build (tests/test_gpu_actor.py): every frame-ring
// load of conv1s_kernel checks its float4 against the n x slots x 120 x 160
// ring and sets this word when it would read past it (round 2 fixed such a
// read on the last sample's row-free step).
__device__ unsigned int g_conv1_oob;
#define CONV1_CHECK(p)                                                          \
  do {                                                                          \
    const size_t e_ = (size_t)((p) - ringT);                                    \
    if (e_ + 4 > (size_t)n * (size_t)slots * plane) atomicOr(&g_conv1_oob, 1u); \
  } while (0)
#else
#define CONV1_CHECK(p) \
  do {                 \
  } while (0)
#endif

// kIdx: the ring holds palette-index frames (u8, dt_render_io.index): a load
// item is one 32-bit word of 4 pixels a frame instead of a float4, decoded to
// the same grey floats (dr::kPalGray) at the commit, so every fp16 value and
// every output equals the grey ring's.
template <bool kStats, bool kIdx>
__global__ void __launch_bounds__(kSThreads, 2)   // 2 waves / SIMD: <= 256 registers
conv1s_kernel(int n, const void* __restrict__ ring, int slots, int s0, int s1, int s2,
              const half8* __restrict__ wfrag, const float* __restrict__ bias,
              __half* __restrict__ y, float* __restrict__ partials, float slope, WeightSplit ws) {
  using Elem = typename std::conditional<kIdx, uint8_t, float>::type;
  using Item = typename std::conditional<kIdx, uint32_t, float4>::type;
  const Elem* __restrict__ ringT = static_cast<const Elem*>(ring);
  __shared__ __attribute__((aligned(16))) unsigned char rb[kSRing * kSRowB];
  __shared__ float s_gray[8];
  __shared__ float red[kSW][CO][3];
  __shared__ float s_bias[CO];
  __shared__ float s_c[CO];   // the sample's centre (kStats): its pixel-0 outputs
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

  // a thread's load items are fixed (row r_i, quad qq_i of the step's range);
  // only the range start and length change per step
  int it_r[kSPre], it_off[kSPre], it_lds[kSPre];
#pragma unroll
  for (int i = 0; i < kSPre; ++i) {
    const int q = tid + i * kSThreads;
    it_r[i] = q / kSQuads;
    it_off[i] = it_r[i] * IW + 4 * (q - it_r[i] * kSQuads);
    it_lds[i] = 4 * kSPxB * (q - it_r[i] * kSQuads);
  }
  // rows r0..r1 of the k-th sample into registers, one float4 per stacked
  // frame; every load issued on every path (items past the range re-load the
  // range's first quad, the sample is clamped), so the compiler's vmcnt waits
  // stay exact.  A step may add no rows (r0 = r1 + 1, up to IH at the end of a
  // sample): its loads then read the sample's row 0, never past the plane.
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
      CONV1_CHECK(p0 + off);
      CONV1_CHECK(p1 + off);
      CONV1_CHECK(p2 + off);
      pre[i][0] = *reinterpret_cast<const Item*>(p0 + off);
      pre[i][1] = *reinterpret_cast<const Item*>(p1 + off);
      pre[i][2] = *reinterpret_cast<const Item*>(p2 + off);
    }
  };
  // a load item's 4 pixels of one frame as grey floats
  auto px4 = [&](const Item& it, float (&o)[4]) __attribute__((always_inline)) {
    if constexpr (kIdx) {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = s_gray[(it >> (8 * e)) & 7u];
    } else {
      o[0] = it.x;
      o[1] = it.y;
      o[2] = it.z;
      o[3] = it.w;
    }
  };
  // fp16 4-channel pixels (channel 3 = 0) into the ring: row R of the stream
  // (k * IH + r) sits in slot R % kSRing
  auto commit = [&](const Item (&pre)[kSPre][3], int k, int r0, int r1) __attribute__((always_inline)) {
    const int rows = r1 - r0 + 1;
#pragma unroll
    for (int i = 0; i < kSPre; ++i) {
      if (it_r[i] >= rows) continue;
      const int slot = (k * IH + r0 + it_r[i]) & (kSRing - 1);
      float av[4], bv[4], cv[4];
      px4(pre[i][0], av);
      px4(pre[i][1], bv);
      px4(pre[i][2], cv);
      if constexpr (kK192) {
        // 4 pixels x 3 channels, pixel-major: (a0 b0)(c0 a1)(b1 c1)(a2 b2)(c2 a3)(b3 c3)
        const float f[12] = {av[0], bv[0], cv[0], av[1], bv[1], cv[1],
                             av[2], bv[2], cv[2], av[3], bv[3], cv[3]};
        uint32_t u[6];
#pragma unroll
        for (int e = 0; e < 6; ++e) {
          const __half2 hv = __floats2half2_rn(f[2 * e], f[2 * e + 1]);
          u[e] = *reinterpret_cast<const uint32_t*>(&hv);
        }
        uint2* dst = reinterpret_cast<uint2*>(rb + slot * kSRowB + it_lds[i]);   // 8-B aligned
        dst[0] = make_uint2(u[0], u[1]);
        dst[1] = make_uint2(u[2], u[3]);
        dst[2] = make_uint2(u[4], u[5]);
      } else {
        uint32_t u[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const __half2 lo = __floats2half2_rn(av[e], bv[e]);
          const __half2 hi = __floats2half2_rn(cv[e], 0.0f);
          u[2 * e] = *reinterpret_cast<const uint32_t*>(&lo);
          u[2 * e + 1] = *reinterpret_cast<const uint32_t*>(&hi);
        }
        u32x4* dst = reinterpret_cast<u32x4*>(rb + slot * kSRowB + it_lds[i]);
        dst[0] = u32x4{u[0], u[1], u[2], u[3]};
        dst[1] = u32x4{u[4], u[5], u[6], u[7]};
      }
    }
  };

  // A fragments.  K 192: MFMA s covers kernel rows ky = 2(s/3) + h (h = the
  // lane half) and 8 of the 24 (kx, c) values of a row, t = 8(s%3) + j ->
  // kx = t/3, c = t%3: a lane's 8 k are 16 contiguous bytes of a ring row.
  // Gathered once from the dt_conv1 fragment layout (include/dtactor.h).
  half8 wa[kSMfma];
  if constexpr (kK192) {
    const _Float16* wh = reinterpret_cast<const _Float16*>(wfrag);
    const int co = lane & 31, hh = lane >> 5;
#pragma unroll
    for (int s = 0; s < kSMfma; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ky = 2 * (s / 3) + hh, t = 8 * (s % 3) + e, kx = t / 3, c = t % 3;
        const int s1 = 2 * ky + kx / 4, l1 = co + 32 * ((kx & 3) >> 1), j1 = 4 * (kx & 1) + c;
        wa[s][e] = wh[(s1 * 64 + l1) * 8 + j1];
      }
  } else {
#pragma unroll
    for (int s = 0; s < kSMfma; ++s) wa[s] = wfrag[s * 64 + lane];
  }
  if (tid < CO) s_bias[tid] = bias[tid];
  if (kIdx && tid < 8) s_gray[tid] = dr::kPalGray[tid];
  float w_cnt = 0.0f, w_mean[16], w_m2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;

  auto step = [&](int g, int k, int j, Item (&nxt)[kSPre][3], const Item (&cur)[kSPre][3]) __attribute__((always_inline)) {
    const int ns = sample(k);
    const bool last_j = j + 1 == kSSteps;
    const int k1 = last_j ? k + 1 : k, j1 = last_j ? 0 : j + 1;   // step g+1
    const int k2 = (j1 + 1 == kSSteps) ? k1 + 1 : k1;             // step g+2
    C1STAMP(0);
    if (!(DTCONV_SKIP & 1)) issue(nxt, k2, s_first_new(j1), s_last_new(j1));

    const int t = kSW * j + wave;
    const int p = 32 * t + col;
    const bool valid = p < kSPix;
    const int pc = valid ? p : 0;
    const int oy = pc / OW, ox = pc - oy * OW;
    const int rbase = k * IH + 2 * oy;
    const int cx = kK192 ? 12 * ox : (2 * ox + 2 * h) * 8;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = s_bias[(r & 3) + 8 * (r >> 2) + 4 * h];
    // kernel rows in pairs (one group: kSGrp B fragments = kSGrp MFMAs);
    // DTCONV1_BDEPTH groups in flight while a group's MFMAs run
    constexpr int kBD = DTCONV1_BDEPTH;
    half8 bq[kBD][kSGrp];
    auto ld = [&](half8 (&b)[kSGrp], int gy) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < kSGrp; ++i) {
        if constexpr (kK192) {   // row 2gy + h, bytes 12 ox + 16 i: 4-B aligned
          using u32x4a = __attribute__((ext_vector_type(4), aligned(4))) uint32_t;
          const int off = ((rbase + 2 * gy + h) & (kSRing - 1)) * kSRowB + cx + 16 * i;
          const u32x4a w = *reinterpret_cast<const u32x4a*>(rb + off);
          b[i] = __builtin_bit_cast(half8, w);
        } else {
          const int ky = 2 * gy + (i >> 1), kx0 = (i & 1) * 4;
          const int off = ((rbase + ky) & (kSRing - 1)) * kSRowB + cx + kx0 * 8;
          b[i] = *reinterpret_cast<const half8*>(rb + off);
        }
      }
    };
    if (DTCONV_SKIP & 32) {   // diagnostic: MFMAs on fragments not read from LDS
#pragma unroll
      for (int q = 0; q < kBD; ++q)
#pragma unroll
        for (int i = 0; i < kSGrp; ++i) bq[q][i] = wa[i];
    }
    if (!(DTCONV_SKIP & 34))
#pragma unroll
      for (int gy = 0; gy < kBD - 1; ++gy) ld(bq[gy], gy);
#pragma unroll
    for (int gy = 0; gy < 4 && !(DTCONV_SKIP & 2); ++gy) {
      if (gy + kBD - 1 < 4 && !(DTCONV_SKIP & 32)) ld(bq[(gy + kBD - 1) % kBD], gy + kBD - 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < kSGrp; ++i)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa[kSGrp * gy + i], bq[gy % kBD][i], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    C1STAMP(1);
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = lrelu2(acc[r], slope);
    C1STAMP(2);
    if (kStats) centre_px32(v, s_c, j == 0 && wave == 0 && col == 0, j == 0, h);
    if (!(DTCONV_SKIP & 4)) store_px32<kSPix>(y + (size_t)ns * kSPix * CO, pc, v, h, valid);
    if (kStats && !(DTCONV_SKIP & 8)) {
      if (valid) {   // Welford over this lane's pixels
        w_cnt += 1.0f;
        const float inv = __builtin_amdgcn_rcpf(w_cnt);   // 1 ulp: an O(1e-7) relative weight error
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = v[r] - w_mean[r];
          w_mean[r] += d * inv;
          w_m2[r] += d * (v[r] - w_mean[r]);
        }
      }
      if (last_j) {   // the 32 lanes of each half (same 16 channels), then the waves
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
          for (int w = 0; w < kSW; ++w) {
            const float nb = red[w][tid][0];
            if (nb <= 0.0f) continue;
            const float tot = cnt + nb, d = red[w][tid][1] - mean;
            mean += d * (nb / tot);
            m2 += red[w][tid][2] + d * d * (cnt * nb / tot);
            cnt = tot;
          }
          float* pp = partials + ((size_t)ns * CO + tid) * 3;
          pp[0] = mean;
          pp[1] = m2;
          pp[2] = s_c[tid];
        }
        w_cnt = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;
      }
    }
    // step g+1's rows into the ring: their slots hold rows no wave reads in
    // this step; the barrier publishes them for the next
    C1STAMP(3);
    if (g + 1 < total && !(DTCONV_SKIP & 16)) commit(cur, k1, s_first_new(j), s_last_new(j));
    C1STAMP(4);
    __syncthreads();
    C1STAMP(5);
  };

  // prologue: step 0's rows into the ring, step 1's into registers
  Item pa[kSPre][3], pb[kSPre][3];
  issue(pa, 0, 0, s_hi(0));
  if (kIdx) __syncthreads();   // s_gray
  commit(pa, 0, 0, s_hi(0));
  if (total > 1) issue(pb, kSSteps == 1 ? 1 : 0, s_first_new(0), s_last_new(0));
  __syncthreads();
  // drain the prologue's loads: they land in other registers than the loop's
  // prefetch sets, and without this the compiler's wait analysis merges that
  // state into the loop header and waits for the previous step's prefetch
  // before every step's MFMAs (instead of at the commit that reads it)
  __builtin_amdgcn_s_waitcnt(0);
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

// Reference mode: y = (y - mean) / sqrt(var + eps) * gamma + beta in place from
// the sample's (mean, M2) per channel (biased variance: BatchNorm2d's
// train-mode normalisation of a batch of one).
__global__ void __launch_bounds__(256)
conv1_norm_kernel(__half* __restrict__ y, const float* __restrict__ partials,
                  const float* __restrict__ gamma, const float* __restrict__ beta, float eps) {
  __shared__ float sc[CO], sh[CO];
  const int n = blockIdx.x, tid = threadIdx.x;
  if (tid < CO) {
    const float* pp = partials + ((size_t)n * CO + tid) * 3;
    const float var = pp[1] / (float)(OH * OW);
    const float s = gamma[tid] / sqrtf(var + eps);
    sc[tid] = s;
    sh[tid] = beta[tid] - pp[0] * s;
  }
  __syncthreads();
  // 8 channels (16 B) per item
  uint4* base = reinterpret_cast<uint4*>(y + (size_t)n * OH * OW * CO);
  const int items = OH * OW * CO / 8;
  for (int i = tid; i < items; i += blockDim.x) {
    uint4 v = base[i];
    const int c0 = (i & 3) * 8;
    __half2* hv = reinterpret_cast<__half2*>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float2 f = __half22float2(hv[k]);
      hv[k] = __floats2half2_rn(f.x * sc[c0 + 2 * k] + sh[c0 + 2 * k],
                                f.y * sc[c0 + 2 * k + 1] + sh[c0 + 2 * k + 1]);
    }
    base[i] = v;
  }
}


// ---- the 32-channel 4x4 convolutions (conv2..conv4) ----------------------------------
// One template for config.json's conv_2d(32 -> 32, 4x4, stride ST) layers.
//
// A persistent workgroup streams whole samples (n = blockIdx.x, + gridDim.x, ...)
// through a ring of input rows in LDS.  A step is NW tiles of 32 consecutive
// output pixels, one per wave; while a step's MFMAs run, the input rows the
// NEXT step adds are already in flight into registers, and they are written to
// the ring (after the previous layer's BatchNorm, kIn 1) once the step's
// epilogue is done: one barrier per step, HBM loads overlapped with compute.
//
//   ring  input row r of the WG's k-th sample lives in slot (k*IH + r) % kRing
//         (ConvGeom::ring() rows: a step's rows plus its successor's); a row is
//         IW pixels x 64 B, stride-2 layers store the even then the odd
//         columns (a lane's neighbour reads the next pixel of the same plane),
//         and chunk c (8 channels) of the pixel at position pos sits at
//         16 * (c ^ ((pos >> 2) & 3)): 16 lanes of a ds_read_b128 group read
//         16 distinct 16-B slots of the 256-B bank row
//   in    kIn 1 (at ring commit, once per element): y = x * sc + sh with the previous layer's train-mode
//         batch-of-one BatchNorm, (sc, sh) from its statistics (Chan's merge)
//   mma   v_mfma_f32_32x32x16_f16, A = weights (32 steps of 16 k, held in
//         registers for the whole launch), B = the pixel's im2col column:
//         step s reads 8 channels of input pixel (ky, kx) = (s/8, (s/2)%4) at
//         channel 16*(s%2) + 8*h
//   out   bias + LeakyReLU, then kOut 0: fp16 NHWC + per-sample Welford
//         statistics (mean, M2) -> part[n][32][2]; 1: fp16 NHWC only (eval
//         mode, BN folded); 2: one step holds the whole sample: exact two-pass
//         statistics over the registers, BatchNorm, written flattened in NCHW
//         order (the reference's view(x.size(0), -1)) for the first linear;
//         3: flattened, no norm
template <int IH, int IW, int OH, int OW, int ST, int NW>
struct ConvGeom {
  static constexpr int kPix = OH * OW;
  static constexpr int kTiles = (kPix + 31) / 32;
  static constexpr int kSteps = (kTiles + NW - 1) / NW;
  static constexpr int kStepPix = 32 * NW;
  // input rows step j reads: lo(j) .. hi(j)
  __host__ __device__ static constexpr int lo(int j) { return ST * ((kStepPix * j) / OW); }
  __host__ __device__ static constexpr int hi(int j) {
    const int end = kStepPix * (j + 1) < kPix ? kStepPix * (j + 1) : kPix;
    const int r = ST * ((end - 1) / OW) + 3;
    return r < IH - 1 ? r : IH - 1;
  }
  // first row the step after j loads (its earlier rows are already in the ring)
  __host__ __device__ static constexpr int first_new(int j) {
    return (j + 1 == kSteps) ? 0 : (hi(j) + 1 > lo(j + 1) ? hi(j) + 1 : lo(j + 1));
  }
  __host__ __device__ static constexpr int last_new(int j) {
    return (j + 1 == kSteps) ? hi(0) : hi(j + 1);
  }
  // ring rows: step j's rows and its successor's held at once
  static constexpr int ring() {
    int m = 0;
    for (int j = 0; j < kSteps; ++j) {
      const int span = (j + 1 < kSteps) ? hi(j + 1) - lo(j) + 1 : (IH - lo(j)) + hi(0) + 1;
      m = span > m ? span : m;
    }
    return m;
  }
  // most rows one step's prefetch brings in
  static constexpr int max_new() {
    int m = 0;
    for (int j = 0; j < kSteps; ++j) {
      const int r = last_new(j) - first_new(j) + 1;
      m = r > m ? r : m;
    }
    return m;
  }
};

// (lo, hi) fp16 pair -> (fp16(lo * s0 + h0), fp16(hi * s1 + h1)): an f32 fma of
// the fp16 input rounded once, one v_fma_mix per element
__device__ __forceinline__ uint32_t norm_pair(uint32_t x, float s0, float h0, float s1, float h1) {
  uint32_t d;
  asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(d) : "v"(x), "v"(s0), "v"(h0));
  asm("v_fma_mixhi_f16 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "+v"(d) : "v"(x), "v"(s1), "v"(h1));
  return d;
}

// byte offset of (pixel px, 16-B chunk c) inside a ring row
template <int IW, int ST>
__device__ __forceinline__ int ring_off(int px, int c) {
  constexpr int kHalfW = (IW + 1) / 2;
  const int pos = ST == 2 ? ((px & 1) ? kHalfW + (px >> 1) : (px >> 1)) : px;
  return 64 * pos + 16 * (c ^ ((pos >> 2) & 3));
}

// conv4 (NW 4): its weights in LDS (32 KB) rather than 128 registers a lane,
// so two of its latency-bound workgroups share a CU (2 waves a SIMD, <= 256
// registers each); DTCONV4_WLDS 0 / DTCONV4_OCC 1 is round 3's register form
#ifndef DTCONV4_WLDS
#define DTCONV4_WLDS 1
#endif
#ifndef DTCONV4_OCC
#define DTCONV4_OCC (DTCONV4_WLDS ? 2 : 1)
#endif
template <int IH, int IW, int OH, int OW, int ST, int NW, int kIn, int kOut>
__global__ void __launch_bounds__(64 * NW, NW == 4 ? DTCONV4_OCC : 1)   // 1: one wave per SIMD, the full register file
conv32_kernel(int n, const __half* __restrict__ x, const half8* __restrict__ wfrag,
              const float* __restrict__ bias, const float* __restrict__ prev_part,
              const float* __restrict__ in_gamma, const float* __restrict__ in_beta, float in_eps,
              __half* __restrict__ y, float* __restrict__ part,
              const float* __restrict__ out_gamma, const float* __restrict__ out_beta,
              float out_eps, float slope, WeightSplit ws) {
  using G = ConvGeom<IH, IW, OH, OW, ST, NW>;
  constexpr int kRing = G::ring();
  constexpr int kRowU4 = IW * 4;                  // 16-B chunks per input row
  constexpr int kRowBytes = IW * 64;
  constexpr int kThreads = 64 * NW;
  constexpr int kPre = (G::max_new() * kRowU4 + kThreads - 1) / kThreads;
  static_assert(kOut < 2 || G::kSteps == 1, "the in-kernel norm needs the sample in one step");
  __shared__ __attribute__((aligned(16))) uint4 ring[kRing * kRowU4];
  __shared__ float s_sc[3][CO], s_sh[3][CO];   // input norm of samples k % 3
  __shared__ float red[NW][CO][3];
  __shared__ float s_mean[CO], s_rstd[CO], s_bias[CO];
  __shared__ float s_c[CO];   // the sample's centre (kOut 0): its pixel-0 outputs
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, h = lane >> 5;
  unsigned char* rb = reinterpret_cast<unsigned char*>(ring);

  const SplitPart sp = split_part(ws, n);
  if (sp.set2) {
    wfrag = static_cast<const half8*>(ws.wfrag);
    bias = ws.bias;
    in_gamma = ws.in_gamma;
    in_beta = ws.in_beta;
    out_gamma = ws.out_gamma;
    out_beta = ws.out_beta;
  }
  const int send = sp.send;
  const int total = sp.my * G::kSteps;
  if (total == 0) return;
  auto sample = [&](int k) __attribute__((always_inline)) { return sp.sbeg + sp.bid + k * sp.gdim; };

  // the previous layer's BatchNorm of the WG's k-th sample (threads < CO), in
  // two halves: the statistics loads are issued ahead of a step's prefetch
  // (so waiting for them never waits for the prefetch), merged after its MFMAs
  float st[2] = {0.0f, 0.0f};
  float gam = 0.0f, bet = 0.0f;
  auto stats_load = [&](int k) __attribute__((always_inline)) {
    // every thread, every step, sample clamped: a fixed count of loads on
    // every path keeps the compiler's vmcnt waits exact
    if (kIn == 1) {
      const int ns = sample(k) < send ? sample(k) : send - 1;
      const int c = tid & (CO - 1);
      const float* pp = prev_part + ((size_t)ns * CO + c) * 3;
      st[0] = pp[0];
      st[1] = pp[1];
      gam = in_gamma[c];
      bet = in_beta[c];
    }
  };
  auto stats_merge = [&](int k) __attribute__((always_inline)) {
    if (kIn == 1 && tid < CO) {
      const float mean = st[0], m2 = st[1], cnt = (float)(IH * IW);
      const float sc = gam / sqrtf(m2 / cnt + in_eps);
      s_sc[k % 3][tid] = sc;
      s_sh[k % 3][tid] = bet - mean * sc;
    }
  };
  // new rows r0..r1 of the k-th sample: chunk q = tid + i*kThreads of the
  // contiguous range into registers, later into the ring as they are
  auto issue = [&](u32x4 (&pre)[kPre], int k, int r0, int r1) __attribute__((always_inline)) {
    // unconditional (clamped sample; chunks past the rows are buffer loads
    // out of range, zeros the commit skips): see stats_load.  The whole chunk
    // offset is the VGPR offset: the raw-buffer range check covers the VGPR
    // and instruction offsets, not the SGPR one, so a chunk past `cnt` reads
    // zeros instead of the memory after the rows (the compiler folds the
    // constant part into the instruction offset: no address VALU a load)
    const int cnt = (r1 - r0 + 1) * kRowU4;
    const int ns = sample(k) < send ? sample(k) : send - 1;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<__half*>(x + ((size_t)ns * IH + r0) * IW * CO), 0, cnt * 16, 0x00020000);
#pragma unroll
    for (int i = 0; i < kPre; ++i)
      pre[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * (tid + i * kThreads), 0, 0);
  };
  // kIn 1: the previous layer's BatchNorm is applied here, once per input
  // element (a thread's chunks all hold channels 8*(tid&3)..+7: kThreads and
  // kRowU4 are multiples of 4), not on every B-fragment read of it
  auto commit = [&](const u32x4 (&pre)[kPre], int k, int r0, int r1) __attribute__((always_inline)) {
    const int cnt = (r1 - r0 + 1) * kRowU4;
    float csc[8], csh[8];
    if (kIn == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        csc[e] = s_sc[k % 3][8 * (tid & 3) + e];
        csh[e] = s_sh[k % 3][8 * (tid & 3) + e];
      }
    }
#pragma unroll
    for (int i = 0; i < kPre; ++i) {
      const int q = tid + i * kThreads;
      if (q >= cnt) continue;
      const int r = q / kRowU4, qq = q - r * kRowU4;
      const int slot = (k * IH + r0 + r) % kRing;
      u32x4 u = pre[i];
      if (kIn == 1 && !(DTCONV_SKIP & 64)) {   // (64: diagnostic, no norm)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          u[e] = norm_pair(u[e], csc[2 * e], csh[2 * e], csc[2 * e + 1], csh[2 * e + 1]);
      }
      *reinterpret_cast<u32x4*>(rb + slot * kRowBytes + ring_off<IW, ST>(qq >> 2, qq & 3)) = u;
    }
  };

  // weights and bias for the whole launch (row = out channel = lane & 31): in
  // registers, or for conv4 in LDS (kWL), read per MFMA
  constexpr bool kWL = NW == 4 && DTCONV4_WLDS;
  __shared__ __attribute__((aligned(16))) half8 wl[kWL ? 32 * 64 : 1];
  half8 wa[kWL ? 1 : 32];
  if constexpr (kWL) {
    for (int i = tid; i < 32 * 64; i += kThreads) wl[i] = wfrag[i];
  } else {
#pragma unroll
    for (int s = 0; s < 32; ++s) wa[s] = wfrag[s * 64 + lane];
  }
  if (tid < CO) s_bias[tid] = bias[tid];
  float w_cnt = 0.0f, w_mean[16], w_m2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;

  // One step.  At its start the ring holds step g's rows and registers `cur`
  // the rows of step g+1 (loaded during step g-1); it loads step g+2's new
  // rows into `nxt`, computes, and commits `cur` to the ring: HBM reads run
  // two steps ahead of the MFMAs.
  auto step = [&](int g, int k, int j, u32x4 (&nxt)[kPre], const u32x4 (&cur)[kPre]) __attribute__((always_inline)) {
    const int ns = sample(k);
    const bool last_j = j + 1 == G::kSteps;
    const int k1 = last_j ? k + 1 : k, j1 = last_j ? 0 : j + 1;   // step g+1
    const bool last_j1 = j1 + 1 == G::kSteps;
    const int k2 = last_j1 ? k1 + 1 : k1;                         // step g+2
    const bool stats2 = g + 2 < total && last_j1;   // step g+2 starts sample k2
    CSTAMP(0);
    stats_load(k2);
    if (!(DTCONV_SKIP & 1)) issue(nxt, k2, G::first_new(j1), G::last_new(j1));

    // this wave's tile
    const int t = NW * j + wave;
    const int p = 32 * t + col;
    const bool valid = p < G::kPix;
    const int pc = valid ? p : 0;
    const int oy = pc / OW, ox = pc - oy * OW;
    int row[4];
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) row[ky] = ((k * IH + ST * oy + ky) % kRing) * kRowBytes;
    int off[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) off[q] = ring_off<IW, ST>(ST * ox + (q >> 1), 2 * (q & 1) + h);
    // 4 groups (ky) of 8 B fragments: group g+1's LDS reads are in flight
    // while group g's MFMAs run
    f32x16 acc;   // starts at the bias
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = s_bias[(r & 3) + 8 * (r >> 2) + 4 * h];
    half8 bq[2][8];
    auto ld = [&](half8 (&b)[8], int gy) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = *reinterpret_cast<const half8*>(rb + row[gy] + off[i]);
    };
    auto mm = [&](half8 (&b)[8], int gy) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 8; ++i)   // the ring rows are already normalised (commit)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kWL ? wl[(8 * gy + i) * 64 + lane]
                                                         : wa[kWL ? 0 : 8 * gy + i],
                                                     b[i], acc, 0, 0, 0);
    };
    if (!(DTCONV_SKIP & 2)) ld(bq[0], 0);
#pragma unroll
    for (int gy = 0; gy < 4 && !(DTCONV_SKIP & 2); ++gy) {
      if (gy < 3) ld(bq[(gy + 1) & 1], gy + 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(bq[gy & 1], gy);
      __builtin_amdgcn_sched_barrier(0);
    }
    CSTAMP(1);
    if (stats2) stats_merge(k2);   // read by step g+2, after two barriers
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = lrelu2(acc[r], slope);
    CSTAMP(2);

    // epilogue
    if (kOut <= 1) {
      if (kOut == 0) centre_px32(v, s_c, j == 0 && wave == 0 && col == 0, j == 0, h);
      if (!(DTCONV_SKIP & 4)) store_px32<G::kPix>(y + (size_t)ns * G::kPix * CO, pc, v, h, valid);
      if (kOut == 0 && valid && !(DTCONV_SKIP & 8)) {   // Welford over this lane's pixels
        w_cnt += 1.0f;
        const float inv = 1.0f / w_cnt;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = v[r] - w_mean[r];
          w_mean[r] += d * inv;
          w_m2[r] += d * (v[r] - w_mean[r]);
        }
      }
      if (kOut == 0 && last_j) {
        // merge the 32 lanes of each half (same 16 channels), then the waves
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
          float* pp = part + ((size_t)ns * CO + tid) * 3;
          pp[0] = mean;
          pp[1] = m2;
          pp[2] = s_c[tid];
        }
        w_cnt = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;
      }
    } else {   // the whole sample is in this step: BatchNorm of a batch of one, flatten
      if (kOut == 2) {
        // per wave, two passes over its own 32 pixels (shuffles only: exact
        // mean, then M2 about it); the waves' (n, mean, M2) merged with
        // Chan's formula by threads < CO: two barriers a sample, not four
        // level by level over the 16 channels: each level's 16 shuffles are
        // in flight together (channel by channel, every shuffle waited for the
        // one before it: 160 dependent LDS round trips, 16k cycles a sample);
        // each channel's sums keep their order, so the bits are unchanged
        float nw = valid ? 1.0f : 0.0f;
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) nw += __shfl_xor(nw, o, 32);
        const float inw = nw > 0.0f ? 1.0f / nw : 0.0f;
        float sum[16], m2[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) sum[r] = valid ? v[r] : 0.0f;
#pragma unroll
        for (int o = 16; o > 0; o >>= 1)
#pragma unroll
          for (int r = 0; r < 16; ++r) sum[r] += __shfl_xor(sum[r], o, 32);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = valid ? v[r] - sum[r] * inw : 0.0f;
          m2[r] = d * d;
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1)
#pragma unroll
          for (int r = 0; r < 16; ++r) m2[r] += __shfl_xor(m2[r], o, 32);
        if (col == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int c = (r & 3) + 8 * (r >> 2) + 4 * h;
            red[wave][c][0] = nw;
            red[wave][c][1] = sum[r] * inw;
            red[wave][c][2] = m2[r];
          }
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
          const float sc = out_gamma[tid] / sqrtf(m2 / (float)G::kPix + out_eps);
          s_rstd[tid] = sc;
          s_mean[tid] = out_beta[tid] - mean * sc;   // the shift
        }
        __syncthreads();
      }
      {   // branch-free (see store_px32): invalid lanes store past the sample
        constexpr int kBytes = G::kPix * CO * 2;
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void*>(y + (size_t)ns * CO * G::kPix), 0, kBytes, 0x00020000);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int c = (r & 3) + 8 * (r >> 2) + 4 * h;
          const float o = kOut == 2 ? v[r] * s_rstd[c] + s_mean[c] : v[r];
          const __half ho = __float2half(o);
          __builtin_amdgcn_raw_buffer_store_b16(*reinterpret_cast<const unsigned short*>(&ho), rsrc,
                                                valid ? (c * G::kPix + p) * 2 : kBytes, 0, 0);
        }
      }
    }

    // step g+1's rows into the ring: their slots held rows no wave reads in
    // this step; the barrier publishes them for the next
    CSTAMP(3);
    if (g + 1 < total && !(DTCONV_SKIP & 16)) commit(cur, k1, G::first_new(j), G::last_new(j));
    CSTAMP(4);
    __syncthreads();
    CSTAMP(5);
  };

  // prologue: step 0's rows into the ring, step 1's into registers
  u32x4 pa[kPre], pb[kPre];
  stats_load(0);
  stats_merge(0);
  if (G::kSteps == 1 && total > 1) {
    stats_load(1);
    stats_merge(1);
  }
  __syncthreads();   // the merged statistics, read by commit
  issue(pa, 0, 0, G::hi(0));
  commit(pa, 0, 0, G::hi(0));
  if (total > 1)
    issue(pb, G::kSteps == 1 ? 1 : 0, G::first_new(0), G::last_new(0));
  __syncthreads();

  int k = 0, j = 0;
  for (int g = 0; g < total; g += 2) {
    step(g, k, j, pa, pb);
    if (++j == G::kSteps) { j = 0; ++k; }
    if (g + 1 < total) {
      step(g + 1, k, j, pb, pa);
      if (++j == G::kSteps) { j = 0; ++k; }
    }
  }
}

template <int IH, int IW, int OH, int OW, int ST, int NW, int kIn, int kOut>
int launch_conv32(int n, const void* x, const void* wfrag, const float* bias,
                  const float* prev_part, const float* ig, const float* ibt,
                  float ieps, void* y, float* part, const float* og, const float* obt, float oeps,
                  float slope, hipStream_t s, WeightSplit ws, int n0) {
  auto kern = conv32_kernel<IH, IW, OH, OW, ST, NW, kIn, kOut>;
  static int grid = 0;   // resident workgroups: one wave of them, persistent
  if (!grid) {
    int dev = 0, cus = 256, per = 1;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 64 * NW, 0) != hipSuccess ||
        per < 1)
      per = 1;
    grid = per * cus;
  }
  const int g = split_grid(ws, n, n0, grid);
  hipLaunchKernelGGL(kern, dim3(g), dim3(64 * NW), 0, s, n, (const __half*)x, (const half8*)wfrag,
                     bias, prev_part, ig, ibt, ieps, (__half*)y, part, og, obt, oeps,
                     slope, ws);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// waves (tiles per step) per layer: conv2 / conv3 two (2-3 rings per CU), conv4
// four (its 4 tiles in one step for the in-kernel norm)
constexpr int kConv2Waves = 2, kConv3Waves = 2, kConv4Waves = 4;

}  // namespace

namespace {
template <bool kIdx>
int conv1_launch(const void* ring, int32_t n, int32_t slots, const int32_t* order,
                 const void* wfrag, const float* bias, const dt_conv_set* set2, void* y,
                 float* partials, float slope, void* stream) {
  if (!ring || !wfrag || !bias || !y || !order || n < 0 || slots < 3) return DT_E_ARG;
  for (int i = 0; i < 3; ++i)
    if (order[i] < 0 || order[i] >= slots) return DT_E_ARG;
  if (set2 && (set2->n0 < 0 || set2->n0 > n || !set2->wfrag || !set2->bias)) return DT_E_ARG;
  if (n == 0) return DT_OK;
  static int grid = 0;   // resident workgroups, persistent
  if (!grid) {
    int dev = 0, cus = 256, per = 2;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, conv1s_kernel<true, kIdx>, kSThreads,
                                                     0) != hipSuccess ||
        per < 1)
      per = 1;
    if (DTCONV1_PER > 0 && DTCONV1_PER < per) per = DTCONV1_PER;
    grid = per * cus;
  }
  WeightSplit ws{};
  if (set2) {
    ws.wfrag = set2->wfrag;
    ws.bias = set2->bias;
  }
  const int g = split_grid(ws, n, set2 ? set2->n0 : n, grid);
  if (partials)
    hipLaunchKernelGGL((conv1s_kernel<true, kIdx>), dim3(g), dim3(kSThreads), 0,
                       (hipStream_t)stream, n, ring, slots, order[0], order[1], order[2],
                       (const half8*)wfrag, bias, (__half*)y, partials, slope, ws);
  else
    hipLaunchKernelGGL((conv1s_kernel<false, kIdx>), dim3(g), dim3(kSThreads), 0,
                       (hipStream_t)stream, n, ring, slots, order[0], order[1], order[2],
                       (const half8*)wfrag, bias, (__half*)y, nullptr, slope, ws);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}
}  // namespace

extern "C" int dt_conv1_split(const float* ring, int32_t n, int32_t slots, const int32_t* order,
                              const void* wfrag, const float* bias, const dt_conv_set* set2,
                              void* y, float* partials, float slope, void* stream) {
  return conv1_launch<false>(ring, n, slots, order, wfrag, bias, set2, y, partials, slope, stream);
}

extern "C" int dt_conv1_index_split(const uint8_t* ring, int32_t n, int32_t slots,
                                    const int32_t* order, const void* wfrag, const float* bias,
                                    const dt_conv_set* set2, void* y, float* partials, float slope,
                                    void* stream) {
  return conv1_launch<true>(ring, n, slots, order, wfrag, bias, set2, y, partials, slope, stream);
}

extern "C" int dt_conv1(const float* ring, int32_t n, int32_t slots, const int32_t* order,
                        const void* wfrag, const float* bias, void* y, float* partials,
                        float slope, void* stream) {
  return dt_conv1_split(ring, n, slots, order, wfrag, bias, nullptr, y, partials, slope, stream);
}

#ifdef DTCONV_STAMPS
extern "C" int dt_diag_convstamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cstamps), sizeof(g_cstamps)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef DTCONV1_STAMPS
extern "C" int dt_diag_convstamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c1stamps), sizeof(g_c1stamps)) == hipSuccess ? 0
                                                                                          : -1;
}
#endif
#ifdef DTCONV_CHECK
// diagnostic build only: the out-of-bounds word of conv1s_kernel (synchronous;
// clears it)
extern "C" int dt_diag_conv1_oob(unsigned int* out) {
  if (hipDeviceSynchronize() != hipSuccess) return DT_E_HIP;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_conv1_oob), sizeof(unsigned int)) != hipSuccess)
    return DT_E_HIP;
  const unsigned int zero = 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_conv1_oob), &zero, sizeof(zero)) == hipSuccess ? DT_OK
                                                                                      : DT_E_HIP;
}
#endif

extern "C" int dt_conv1_norm(void* y, int32_t n, const float* partials, const float* gamma,
                             const float* beta, float eps, void* stream) {
  if (!y || !partials || !gamma || !beta || n < 0) return DT_E_ARG;
  if (n == 0) return DT_OK;
  hipLaunchKernelGGL(conv1_norm_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, (__half*)y,
                     partials, gamma, beta, eps);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// conv2..conv4 of the reference actor (see include/dtactor.h)
extern "C" int dt_conv32_split(int32_t layer, int32_t n, const void* x, const void* wfrag,
                               const float* bias, const float* prev_part, const float* in_gamma,
                               const float* in_beta, float in_eps, void* y, float* part,
                               const float* out_gamma, const float* out_beta, float out_eps,
                               float slope, const dt_conv_set* set2, void* stream) {
  if (!x || !wfrag || !bias || !y || n < 0) return DT_E_ARG;
  const bool in = prev_part != nullptr;
  if (in && (!in_gamma || !in_beta)) return DT_E_ARG;
  if (set2 && (set2->n0 < 0 || set2->n0 > n || !set2->wfrag || !set2->bias ||
               (in && (!set2->in_gamma || !set2->in_beta)) ||
               ((out_gamma != nullptr) != (set2->out_gamma != nullptr)) ||
               ((out_beta != nullptr) != (set2->out_beta != nullptr))))
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
    case 2:   // 57x77 -> 27x37, stride 2; input norm from conv1's per-sample statistics
      if (in != (part != nullptr)) return DT_E_ARG;
      return in ? launch_conv32<57, 77, 27, 37, 2, kConv2Waves, 1, 0>(
                      n, x, wfrag, bias, prev_part, in_gamma, in_beta, in_eps, y, part,
                      nullptr, nullptr, 0.f, slope, s, ws, n0)
                : launch_conv32<57, 77, 27, 37, 2, kConv2Waves, 0, 1>(
                      n, x, wfrag, bias, nullptr, nullptr, nullptr, 0.f, y, nullptr, nullptr,
                      nullptr, 0.f, slope, s, ws, n0);
    case 3:   // 27x37 -> 12x17, stride 2; input norm from conv2's per-sample statistics
      if (in != (part != nullptr)) return DT_E_ARG;
      return in ? launch_conv32<27, 37, 12, 17, 2, kConv3Waves, 1, 0>(
                      n, x, wfrag, bias, prev_part, in_gamma, in_beta, in_eps, y, part,
                      nullptr, nullptr, 0.f, slope, s, ws, n0)
                : launch_conv32<27, 37, 12, 17, 2, kConv3Waves, 0, 1>(
                      n, x, wfrag, bias, nullptr, nullptr, nullptr, 0.f, y, nullptr, nullptr,
                      nullptr, 0.f, slope, s, ws, n0);
    case 4:   // 12x17 -> 9x14, stride 1, whole sample per step; its own norm in-kernel; flattened
      if (in != (out_gamma != nullptr)) return DT_E_ARG;
      return in ? launch_conv32<12, 17, 9, 14, 1, kConv4Waves, 1, 2>(
                      n, x, wfrag, bias, prev_part, in_gamma, in_beta, in_eps, y, nullptr,
                      out_gamma, out_beta, out_eps, slope, s, ws, n0)
                : launch_conv32<12, 17, 9, 14, 1, kConv4Waves, 0, 3>(
                      n, x, wfrag, bias, nullptr, nullptr, nullptr, 0.f, y, nullptr, nullptr,
                      nullptr, 0.f, slope, s, ws, n0);
    default:
      return DT_E_ARG;
  }
}

extern "C" int dt_conv32(int32_t layer, int32_t n, const void* x, const void* wfrag,
                         const float* bias, const float* prev_part, const float* in_gamma,
                         const float* in_beta, float in_eps, void* y, float* part,
                         const float* out_gamma, const float* out_beta, float out_eps,
                         float slope, void* stream) {
  return dt_conv32_split(layer, n, x, wfrag, bias, prev_part, in_gamma, in_beta, in_eps, y, part,
                         out_gamma, out_beta, out_eps, slope, nullptr, stream);
}
