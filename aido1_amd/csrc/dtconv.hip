// The actor's first convolution (config.json actor: conv_2d 3 -> 32, 8x8,
// stride 2, then leaky_relu) as a gfx950 MFMA implicit GEMM that reads the
// observation ring in place -- see include/dtactor.h (dt_conv1).
//
// Per workgroup: one sample x one band of kBand output rows.
//   load   the band's 2*kBand+6 input rows from the three f32 ring slots (in
//          the stack's oldest -> newest order), converted to fp16 as 4-channel
//          pixels (channel 3 = 0) in LDS: a row is 160 px x 8 B
//   mma    per wave, tiles of 32 output pixels x 32 channels with
//          v_mfma_f32_32x32x16_f16: A = weights (row = out channel), B = the
//          im2col column of a pixel (k = (ky, kx, c), 16 k per step = one
//          kernel row half: 2 px x 4 ch per lane half = one 16-B LDS read);
//          16 steps cover K = 8 x 8 x 4
//   out    bias + LeakyReLU, fp16 NHWC (each lane: one pixel, 16 channels as
//          four 8-B groups); with `partials`, the band's per-channel count /
//          mean / M2 by two passes over the register-resident outputs
//          (reference mode: the per-sample BatchNorm statistics, merged by
//          dt_conv1_norm with Chan's formula)
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "../../include/dtactor.h"

// diagnostic builds only (tools/conv32_micro.py): bit 0 skips the prefetch
// loads, 1 the MFMA section, 2 the output stores, 3 the statistics, 4 the ring
// commit; the product build is 0
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

namespace {

constexpr int IH = 120, IW = 160, OH = 57, OW = 77, CO = 32;
constexpr int kBand = 8;                     // output rows per workgroup
constexpr int kBands = (OH + kBand - 1) / kBand;
constexpr int kInRows = 2 * kBand + 6;       // input rows a band needs
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kBandPix = kBand * OW;                 // 616
constexpr int kTiles = (kBandPix + 31) / 32;         // 20
constexpr int kTilesPerWave = (kTiles + kWaves - 1) / kWaves;  // 5

using half8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;

__device__ __forceinline__ float lrelu(float v, float s) { return v > 0.0f ? v : v * s; }
// the same for 0 <= s <= 1 as two instructions (a multiply and a max)
__device__ __forceinline__ float lrelu2(float v, float s) { return fmaxf(v, v * s); }

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

// Persistent kernels: two workgroups per CU (the VGPR budget of these kernels),
// each striding over (sample, band) items with its weights held in registers.
int persistent_grid() {
  static int g = 0;
  if (!g) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    g = 2 * cus;
  }
  return g;
}

__global__ void __launch_bounds__(kThreads, 2)   // 2 waves / SIMD: <= 256 VGPRs
conv1_kernel(int n_items, const float* __restrict__ ring, int slots, int s0, int s1, int s2,
             const half8* __restrict__ wfrag, const float* __restrict__ bias,
             __half* __restrict__ y, float* __restrict__ partials, float slope) {
  __shared__ __attribute__((aligned(16))) uint2 img[kInRows * IW];   // 4 x fp16 per pixel
  __shared__ float red[kWaves][2][CO];
  __shared__ float mean_s[CO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // weights once per workgroup (persistent: the grid strides over items):
  // this lane's A fragments of the 16 k-steps (row = out channel)
  half8 wa[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) wa[s] = wfrag[s * 64 + lane];
  for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
  const int n = item / kBands, band = item - n * kBands;
  const int oy0 = band * kBand;
  const int rows_out = (OH - oy0) < kBand ? (OH - oy0) : kBand;
  const int band_pix = rows_out * OW;
  __syncthreads();   // the previous item's readers of img / red are done

  // ---- load: input rows 2*oy0 .. 2*oy0 + kInRows - 1, 4 px per item ----------------
  // all of the band's loads are issued before any is converted
  const float* base = ring + (size_t)n * slots * IH * IW;
  const float* p0 = base + (size_t)s0 * IH * IW;
  const float* p1 = base + (size_t)s1 * IH * IW;
  const float* p2 = base + (size_t)s2 * IH * IW;
  constexpr int kItems = kInRows * (IW / 4);
  constexpr int kPer = (kItems + kThreads - 1) / kThreads;
  float4 la[kPer], lb[kPer], lc[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int it = tid + k * kThreads;
    const int r = it / (IW / 4), q = it - r * (IW / 4);
    const int iy = 2 * oy0 + r;
    la[k] = lb[k] = lc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (it < kItems && iy < IH) {
      const size_t off = (size_t)iy * IW + 4 * q;
      la[k] = *reinterpret_cast<const float4*>(p0 + off);
      lb[k] = *reinterpret_cast<const float4*>(p1 + off);
      lc[k] = *reinterpret_cast<const float4*>(p2 + off);
    }
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int it = tid + k * kThreads;
    if (it >= kItems) continue;
    const int r = it / (IW / 4), q = it - r * (IW / 4);
    const float av[4] = {la[k].x, la[k].y, la[k].z, la[k].w};
    const float bv[4] = {lb[k].x, lb[k].y, lb[k].z, lb[k].w};
    const float cv[4] = {lc[k].x, lc[k].y, lc[k].z, lc[k].w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const __half2 lo = __floats2half2_rn(av[i], bv[i]);
      const __half2 hi = __floats2half2_rn(cv[i], 0.0f);
      uint2 px;
      px.x = *reinterpret_cast<const uint32_t*>(&lo);
      px.y = *reinterpret_cast<const uint32_t*>(&hi);
      img[r * IW + 4 * q + i] = px;
    }
  }
  __syncthreads();

  // ---- MFMA: tile t covers band pixels 32t .. 32t+31 ---------------------------------
  const int col = lane & 31, h = lane >> 5;
  float out[kTilesPerWave][16];
  float bco[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) bco[r] = bias[(r & 3) + 8 * (r >> 2) + 4 * h];
#pragma unroll
  for (int ti = 0; ti < kTilesPerWave; ++ti) {
    const int t = wave + kWaves * ti;
    const int p = 32 * t + col;                       // this lane's pixel (B column)
    const bool valid = t < kTiles && p < band_pix;
    const int pc = valid ? p : 0;
    const int oyl = pc / OW, ox = pc - oyl * OW;
    const uint2* src = img + (2 * oyl) * IW + 2 * ox + 2 * h;
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int ky = s >> 1, kx0 = (s & 1) * 4;
      const half8 bfrag = *reinterpret_cast<const half8*>(src + ky * IW + kx0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa[s], bfrag, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) out[ti][r] = valid ? lrelu(acc[r] + bco[r], slope) : 0.0f;
    if (valid) {   // channels (r&3) + 8*(r>>2) + 4h: four groups of 4 consecutive channels
      __half* dst = y + (((size_t)n * OH + oy0 + oyl) * OW + ox) * CO;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const __half2 v0 = __floats2half2_rn(out[ti][4 * g + 0], out[ti][4 * g + 1]);
        const __half2 v1 = __floats2half2_rn(out[ti][4 * g + 2], out[ti][4 * g + 3]);
        uint2 v;
        v.x = *reinterpret_cast<const uint32_t*>(&v0);
        v.y = *reinterpret_cast<const uint32_t*>(&v1);
        *reinterpret_cast<uint2*>(dst + 8 * g + 4 * h) = v;
      }
    }
  }
  if (partials) {
  // ---- band statistics per channel: two passes over the register-resident outputs ----
  // pass 1: sum -> band mean
  float acc16[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = 0.0f;
#pragma unroll
    for (int ti = 0; ti < kTilesPerWave; ++ti) v += out[ti][r];   // invalid pixels hold 0
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);   // over the 32 pixels
    acc16[r] = v;
  }
  if (col == 0)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave][0][(r & 3) + 8 * (r >> 2) + 4 * h] = acc16[r];
  __syncthreads();
  if (tid < CO) {
    float s = 0.0f;
    for (int w = 0; w < kWaves; ++w) s += red[w][0][tid];
    mean_s[tid] = s / (float)band_pix;
  }
  __syncthreads();
  // pass 2: M2 about the band mean
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float mu = mean_s[(r & 3) + 8 * (r >> 2) + 4 * h];
    float v = 0.0f;
#pragma unroll
    for (int ti = 0; ti < kTilesPerWave; ++ti) {
      const int t = wave + kWaves * ti;
      const bool valid = t < kTiles && 32 * t + col < band_pix;
      const float d = out[ti][r] - mu;
      v += valid ? d * d : 0.0f;
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
    acc16[r] = v;
  }
  if (col == 0)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave][1][(r & 3) + 8 * (r >> 2) + 4 * h] = acc16[r];
  __syncthreads();
  if (tid < CO) {
    float m2 = 0.0f;
    for (int w = 0; w < kWaves; ++w) m2 += red[w][1][tid];
    float* pp = partials + (((size_t)n * kBands + band) * CO + tid) * 2;
    pp[0] = mean_s[tid];
    pp[1] = m2;
  }
  }  // partials
  }  // item
}

// ---- conv1, streaming form (the default; DTCONV1_BANDED=1 selects conv1_kernel) ----
// A persistent workgroup of kSW waves streams whole samples (n = blockIdx.x,
// + gridDim.x, ...).  The input rows go through a ring of kSRing rows in LDS
// (fp16 4-channel pixels as in conv1_kernel), each row read from HBM once per
// sample (the banded form re-reads 1.375x for its halos).  A step is kSW tiles
// of 32 consecutive output pixels, one per wave; while a step's MFMAs run, the
// rows of the step after next are in flight into registers, and the next
// step's rows (loaded a step earlier) are converted into the ring after the
// epilogue: one barrier per step (conv32_kernel's schedule).  Two workgroups
// per CU, so one's barrier leaves the other's MFMAs running.  Reference mode:
// per-lane Welford statistics over the sample, merged (Chan) into ONE
// (mean, M2) per sample and channel: dt_conv1_bands() is 1.
constexpr int kSW = 4;
constexpr int kSThreads = 64 * kSW;
constexpr int kSPix = OH * OW;                          // 4389
constexpr int kSTiles = (kSPix + 31) / 32;              // 138
constexpr int kSSteps = (kSTiles + kSW - 1) / kSW;      // 35
constexpr int kSStepPix = 32 * kSW;
constexpr int kSRing = 32;                              // rows (a power of two)
constexpr bool kK192 = DTCONV1_K192 != 0;
constexpr int kSPxB = kK192 ? 6 : 8;                    // bytes a ring pixel: fp16 x 3 (x 4)
constexpr int kSRowB = IW * kSPxB;                      // 960 (1280) B
constexpr int kSMfma = kK192 ? 12 : 16;                 // MFMAs a tile
constexpr int kSGrp = kK192 ? 3 : 4;                    // MFMAs a B-fragment group
constexpr int kSQuads = IW / 4;                         // 4-pixel load items per row
__host__ __device__ constexpr int s_lo(int j) { return 2 * ((kSStepPix * j) / OW); }
__host__ __device__ constexpr int s_hi(int j) {
  const int end = kSStepPix * (j + 1) < kSPix ? kSStepPix * (j + 1) : kSPix;
  const int r = 2 * ((end - 1) / OW) + 7;
  return r < IH - 1 ? r : IH - 1;
}
__host__ __device__ constexpr int s_first_new(int j) {
  return (j + 1 == kSSteps) ? 0 : (s_hi(j) + 1 > s_lo(j + 1) ? s_hi(j) + 1 : s_lo(j + 1));
}
__host__ __device__ constexpr int s_last_new(int j) {
  return (j + 1 == kSSteps) ? s_hi(0) : s_hi(j + 1);
}
constexpr int s_span() {   // rows one step reads plus the rows its successor adds
  int m = 0;
  for (int j = 0; j < kSSteps; ++j) {
    const int span = (j + 1 < kSSteps) ? s_hi(j + 1) - s_lo(j) + 1 : (IH - s_lo(j)) + s_hi(0) + 1;
    m = span > m ? span : m;
  }
  return m;
}
constexpr int s_max_new() {
  int m = s_hi(0) + 1;
  for (int j = 0; j < kSSteps; ++j) {
    const int r = s_last_new(j) - s_first_new(j) + 1;
    m = r > m ? r : m;
  }
  return m;
}
static_assert(s_span() <= kSRing, "conv1 stream ring");
constexpr int kSPre = (s_max_new() * kSQuads + kSThreads - 1) / kSThreads;

#ifdef DTCONV_CHECK
// Bounds-checked diagnostic build (tests/test_gpu_actor.py): every frame-ring
// load of conv1s_kernel checks its float4 against the n x slots x 120 x 160
// ring and sets this word when it would read past it (round 2 fixed such a
// read on the last sample's row-free step).
__device__ unsigned int g_conv1_oob;
#define CONV1_CHECK(p)                                                          \
  do {                                                                          \
    const size_t e_ = (size_t)((p) - ring);                                     \
    if (e_ + 4 > (size_t)n * (size_t)slots * plane) atomicOr(&g_conv1_oob, 1u); \
  } while (0)
#else
#define CONV1_CHECK(p) \
  do {                 \
  } while (0)
#endif

template <bool kStats>
__global__ void __launch_bounds__(kSThreads, 2)   // 2 waves / SIMD: <= 256 registers
conv1s_kernel(int n, const float* __restrict__ ring, int slots, int s0, int s1, int s2,
              const half8* __restrict__ wfrag, const float* __restrict__ bias,
              __half* __restrict__ y, float* __restrict__ partials, float slope) {
  __shared__ __attribute__((aligned(16))) unsigned char rb[kSRing * kSRowB];
  __shared__ float red[kSW][CO][3];
  __shared__ float s_bias[CO];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, h = lane >> 5;
  const int my = n > (int)blockIdx.x ? (n - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int total = my * kSSteps;
  if (total == 0) return;
  auto sample = [&](int k) __attribute__((always_inline)) { return (int)blockIdx.x + k * (int)gridDim.x; };
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
  auto issue = [&](float4 (&pre)[kSPre][3], int k, int r0, int r1) __attribute__((always_inline)) {
    const int rows = r1 - r0 + 1;
    const int ns = sample(k) < n ? sample(k) : n - 1;
    const float* base = ring + (size_t)ns * slots * plane + (size_t)(rows > 0 ? r0 : 0) * IW;
    const float* p0 = base + (size_t)s0 * plane;
    const float* p1 = base + (size_t)s1 * plane;
    const float* p2 = base + (size_t)s2 * plane;
#pragma unroll
    for (int i = 0; i < kSPre; ++i) {
      const int off = it_r[i] < rows ? it_off[i] : 0;
      CONV1_CHECK(p0 + off);
      CONV1_CHECK(p1 + off);
      CONV1_CHECK(p2 + off);
      pre[i][0] = *reinterpret_cast<const float4*>(p0 + off);
      pre[i][1] = *reinterpret_cast<const float4*>(p1 + off);
      pre[i][2] = *reinterpret_cast<const float4*>(p2 + off);
    }
  };
  // fp16 4-channel pixels (channel 3 = 0) into the ring: row R of the stream
  // (k * IH + r) sits in slot R % kSRing
  auto commit = [&](const float4 (&pre)[kSPre][3], int k, int r0, int r1) __attribute__((always_inline)) {
    const int rows = r1 - r0 + 1;
#pragma unroll
    for (int i = 0; i < kSPre; ++i) {
      if (it_r[i] >= rows) continue;
      const int slot = (k * IH + r0 + it_r[i]) & (kSRing - 1);
      const float av[4] = {pre[i][0].x, pre[i][0].y, pre[i][0].z, pre[i][0].w};
      const float bv[4] = {pre[i][1].x, pre[i][1].y, pre[i][1].z, pre[i][1].w};
      const float cv[4] = {pre[i][2].x, pre[i][2].y, pre[i][2].z, pre[i][2].w};
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
  float w_cnt = 0.0f, w_mean[16], w_m2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;

  auto step = [&](int g, int k, int j, float4 (&nxt)[kSPre][3], const float4 (&cur)[kSPre][3]) __attribute__((always_inline)) {
    const int ns = sample(k);
    const bool last_j = j + 1 == kSSteps;
    const int k1 = last_j ? k + 1 : k, j1 = last_j ? 0 : j + 1;   // step g+1
    const int k2 = (j1 + 1 == kSSteps) ? k1 + 1 : k1;             // step g+2
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
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = lrelu2(acc[r], slope);
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
          float* pp = partials + ((size_t)ns * CO + tid) * 2;
          pp[0] = mean;
          pp[1] = m2;
        }
        w_cnt = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;
      }
    }
    // step g+1's rows into the ring: their slots hold rows no wave reads in
    // this step; the barrier publishes them for the next
    if (g + 1 < total && !(DTCONV_SKIP & 16)) commit(cur, k1, s_first_new(j), s_last_new(j));
    __syncthreads();
  };

  // prologue: step 0's rows into the ring, step 1's into registers
  float4 pa[kSPre][3], pb[kSPre][3];
  issue(pa, 0, 0, s_hi(0));
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

bool conv1_banded() {
  static int b = -1;
  if (b < 0) {
    const char* e = getenv("DTCONV1_BANDED");
    b = (e && e[0] == '1') ? 1 : 0;
  }
  return b == 1;
}
int conv1_bands() { return conv1_banded() ? kBands : 1; }
int conv1_band_rows() { return conv1_banded() ? kBand : OH; }

// Reference mode: merge the bands' (mean, M2) per sample and channel (Chan et
// al.), then y = (y - mean) / sqrt(var + eps) * gamma + beta in place (biased
// variance: BatchNorm2d's train-mode normalisation of a batch of one).
__global__ void __launch_bounds__(256)
conv1_norm_kernel(__half* __restrict__ y, const float* __restrict__ partials,
                  const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                  int bands, int band_rows) {
  __shared__ float sc[CO], sh[CO];
  const int n = blockIdx.x, tid = threadIdx.x;
  if (tid < CO) {
    const float* pp = partials + (size_t)n * bands * CO * 2;
    float cnt = 0.0f, mean = 0.0f, m2 = 0.0f;
    for (int b = 0; b < bands; ++b) {
      const int rows = (OH - b * band_rows) < band_rows ? (OH - b * band_rows) : band_rows;
      const float nb = (float)(rows * OW);
      const float mb = pp[(b * CO + tid) * 2], m2b = pp[(b * CO + tid) * 2 + 1];
      const float tot = cnt + nb;
      const float d = mb - mean;
      mean += d * (nb / tot);
      m2 += m2b + d * d * (cnt * nb / tot);
      cnt = tot;
    }
    const float var = m2 / cnt;
    const float s = gamma[tid] / sqrtf(var + eps);
    sc[tid] = s;
    sh[tid] = beta[tid] - mean * s;
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

// conv4 (NW 4) waves per SIMD: 1 holds its 317 registers; 2 spills ~60 (diagnostic)
#ifndef DTCONV4_OCC
#define DTCONV4_OCC 1
#endif
template <int IH, int IW, int OH, int OW, int ST, int NW, int kIn, int kOut, int kPrevRows>
__global__ void __launch_bounds__(64 * NW, NW == 4 ? DTCONV4_OCC : 1)   // 1: one wave per SIMD, the full register file
conv32_kernel(int n, const __half* __restrict__ x, const half8* __restrict__ wfrag,
              const float* __restrict__ bias, const float* __restrict__ prev_part,
              const float* __restrict__ in_gamma, const float* __restrict__ in_beta, float in_eps,
              __half* __restrict__ y, float* __restrict__ part,
              const float* __restrict__ out_gamma, const float* __restrict__ out_beta,
              float out_eps, float slope) {
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
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, h = lane >> 5;
  unsigned char* rb = reinterpret_cast<unsigned char*>(ring);

  const int my = n > (int)blockIdx.x ? (n - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int total = my * G::kSteps;
  if (total == 0) return;
  auto sample = [&](int k) __attribute__((always_inline)) { return (int)blockIdx.x + k * (int)gridDim.x; };

  // the previous layer's BatchNorm of the WG's k-th sample (threads < CO), in
  // two halves: the statistics loads are issued ahead of a step's prefetch
  // (so waiting for them never waits for the prefetch), merged after its MFMAs
  constexpr int kPB = (IH + kPrevRows - 1) / kPrevRows;
  float st[kIn == 1 ? kPB : 1][2];
  float gam = 0.0f, bet = 0.0f;
  auto stats_load = [&](int k) __attribute__((always_inline)) {
    // every thread, every step, sample clamped: a fixed count of loads on
    // every path keeps the compiler's vmcnt waits exact
    if (kIn == 1) {
      const int ns = sample(k) < n ? sample(k) : n - 1;
      const float* pp = prev_part + (size_t)ns * kPB * CO * 2;
      const int c = tid & (CO - 1);
#pragma unroll
      for (int q = 0; q < kPB; ++q) {
        st[q][0] = pp[(q * CO + c) * 2];
        st[q][1] = pp[(q * CO + c) * 2 + 1];
      }
      gam = in_gamma[c];
      bet = in_beta[c];
    }
  };
  auto stats_merge = [&](int k) __attribute__((always_inline)) {
    if (kIn == 1 && tid < CO) {
      float cnt = 0.0f, mean = 0.0f, m2 = 0.0f;
#pragma unroll
      for (int q = 0; q < kPB; ++q) {
        const int rq = (IH - q * kPrevRows) < kPrevRows ? (IH - q * kPrevRows) : kPrevRows;
        const float nb = (float)(rq * IW);
        const float tot = cnt + nb, d = st[q][0] - mean;
        mean += d * (nb / tot);
        m2 += st[q][1] + d * d * (cnt * nb / tot);
        cnt = tot;
      }
      const float sc = gam / sqrtf(m2 / cnt + in_eps);
      s_sc[k % 3][tid] = sc;
      s_sh[k % 3][tid] = bet - mean * sc;
    }
  };
  // new rows r0..r1 of the k-th sample: chunk q = tid + i*kThreads of the
  // contiguous range into registers, later into the ring as they are
  auto issue = [&](u32x4 (&pre)[kPre], int k, int r0, int r1) __attribute__((always_inline)) {
    // unconditional (clamped chunk and sample): see stats_load
    const int cnt = (r1 - r0 + 1) * kRowU4;
    const int ns = sample(k) < n ? sample(k) : n - 1;
    const u32x4* src = reinterpret_cast<const u32x4*>(x + ((size_t)ns * IH + r0) * IW * CO);
#pragma unroll
    for (int i = 0; i < kPre; ++i) {
      const int q = tid + i * kThreads;
      pre[i] = src[q < cnt ? q : cnt - 1];
    }
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
      if (kIn == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          u[e] = norm_pair(u[e], csc[2 * e], csh[2 * e], csc[2 * e + 1], csh[2 * e + 1]);
      }
      *reinterpret_cast<u32x4*>(rb + slot * kRowBytes + ring_off<IW, ST>(qq >> 2, qq & 3)) = u;
    }
  };

  // weights and bias for the whole launch (row = out channel = lane & 31)
  half8 wa[32];
#pragma unroll
  for (int s = 0; s < 32; ++s) wa[s] = wfrag[s * 64 + lane];
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
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(wa[8 * gy + i], b[i], acc, 0, 0, 0);
    };
    if (!(DTCONV_SKIP & 2)) ld(bq[0], 0);
#pragma unroll
    for (int gy = 0; gy < 4 && !(DTCONV_SKIP & 2); ++gy) {
      if (gy < 3) ld(bq[(gy + 1) & 1], gy + 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(bq[gy & 1], gy);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (stats2) stats_merge(k2);   // read by step g+2, after two barriers
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = lrelu2(acc[r], slope);

    // epilogue
    if (kOut <= 1) {
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
          float* pp = part + ((size_t)ns * CO + tid) * 2;
          pp[0] = mean;
          pp[1] = m2;
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
        float nw = valid ? 1.0f : 0.0f;
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) nw += __shfl_xor(nw, o, 32);
        const float inw = nw > 0.0f ? 1.0f / nw : 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float sum = valid ? v[r] : 0.0f;
#pragma unroll
          for (int o = 16; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 32);
          const float mw = sum * inw;
          const float d = valid ? v[r] - mw : 0.0f;
          float m2 = d * d;
#pragma unroll
          for (int o = 16; o > 0; o >>= 1) m2 += __shfl_xor(m2, o, 32);
          if (col == 0) {
            const int c = (r & 3) + 8 * (r >> 2) + 4 * h;
            red[wave][c][0] = nw;
            red[wave][c][1] = mw;
            red[wave][c][2] = m2;
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
    if (g + 1 < total && !(DTCONV_SKIP & 16)) commit(cur, k1, G::first_new(j), G::last_new(j));
    __syncthreads();
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

template <int IH, int IW, int OH, int OW, int ST, int NW, int kIn, int kOut, int kPrevRows = IH>
int launch_conv32(int n, const void* x, const void* wfrag, const float* bias,
                  const float* prev_part, const float* ig, const float* ibt,
                  float ieps, void* y, float* part, const float* og, const float* obt, float oeps,
                  float slope, hipStream_t s) {
  auto kern = conv32_kernel<IH, IW, OH, OW, ST, NW, kIn, kOut, kPrevRows>;
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
  const int g = n < grid ? n : grid;
  hipLaunchKernelGGL(kern, dim3(g), dim3(64 * NW), 0, s, n, (const __half*)x, (const half8*)wfrag,
                     bias, prev_part, ig, ibt, ieps, (__half*)y, part, og, obt, oeps,
                     slope);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// waves (tiles per step) per layer: conv2 / conv3 two (2-3 rings per CU), conv4
// four (its 4 tiles in one step for the in-kernel norm)
constexpr int kConv2Waves = 2, kConv3Waves = 2, kConv4Waves = 4;


// ---- conv1 + its BatchNorm + conv2 in one kernel (dt_conv12) ---------------------------
// One workgroup (4 waves, one per SIMD: 512 registers a lane) per sample.  A
// step is 4 tiles of 32 consecutive output pixels, one per wave (one
// accumulation chain issues at full MFMA rate: MI355X_MICROARCH.md).
//   A  conv1 as in conv1_kernel, but over the whole sample in 35 steps: the
//      input rows stream through an LDS ring (16 rows, fp16 4-channel pixels;
//      the next step's new rows are loaded during a step), both weight sets
//      sit in LDS, and each wave keeps its 35 tiles' outputs (bias +
//      LeakyReLU, fp16) in registers: the sample's 57 x 77 x 32 activation
//      never leaves the CU.
//   B  reference mode: the per-sample BatchNorm statistics of those outputs
//      (mean from the f32 values summed in A, M2 about it over the fp16
//      values the next layer reads), then the normalisation applied in the
//      registers (one v_fma_mix per element, as conv32's ring commit).
//   C  conv2 in 8 steps of 4 tiles: before each, the waves write the conv1 rows
//      it reads (at most 12) from their registers into a second LDS ring
//      (conv32's stride-2 row layout; it aliases A's ring), then the conv32
//      MFMA step and epilogue: fp16 NHWC out + per-sample Welford statistics.
// This removes conv1's 1.15 GB fp16 round trip through HBM per 4096 samples
// and the 1.375x re-read of band halos.
#ifdef DTSIM_STAMPS
// conv12_kernel per workgroup (diagnostics, tools/conv12_stamps.py): [0] real
// time at entry, [1] at exit, [2..7] shader clock after: entry, step-0 rows,
// phase A, phase B, phase C's row writes of step 0, the end
__device__ unsigned long long g_c12stamps[4096 * 8];
#define C12T(i)                                                                        \
  do {                                                                                 \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                        \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_c12stamps[blockIdx.x * 8 + (i)] = _t; \
  } while (0)
#define C12R(i)                                                                        \
  do {                                                                                 \
    const unsigned long long _t = __builtin_amdgcn_s_memrealtime();                    \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_c12stamps[blockIdx.x * 8 + (i)] = _t; \
  } while (0)
#else
#define C12T(i) \
  do {          \
  } while (0)
#define C12R(i) \
  do {          \
  } while (0)
#endif
constexpr int kFW = 4, kFT = 64 * kFW, kFU = 1;            // waves, threads, tiles per wave
constexpr int kFTiles = kFW * kFU;                          // tiles per step
constexpr int kFPix1 = OH * OW;                             // 4389
constexpr int kFSteps1 = ((kFPix1 + 31) / 32 + kFTiles - 1) / kFTiles;  // 18
constexpr int kFRing1 = 16;
constexpr int OH2 = 27, OW2 = 37, kFPix2 = OH2 * OW2;       // 999
constexpr int kFSteps2 = ((kFPix2 + 31) / 32 + kFTiles - 1) / kFTiles;  // 4
constexpr int kFRing2 = 12;
constexpr int kFRow2 = OW * 64;                             // bytes per conv2 ring row
constexpr int kFNew = 4;                                    // most rows a step adds
constexpr int kFPre = (kFNew * (IW / 4) + kFT - 1) / kFT;   // prefetch items a thread
constexpr int kF0 = 4;                                      // step 0's items a thread
constexpr int kFAgpr = 28;                                  // steps whose outputs sit in AGPRs
constexpr int kFDepth = 8;                                  // input prefetch distance, steps

__host__ __device__ constexpr int f_lo1(int j) { return 2 * ((32 * kFTiles * j) / OW); }
__host__ __device__ constexpr int f_hi1(int j) {
  const int e = 32 * kFTiles * (j + 1) - 1 < kFPix1 - 1 ? 32 * kFTiles * (j + 1) - 1 : kFPix1 - 1;
  const int r = 2 * (e / OW) + 7;
  return r < IH - 1 ? r : IH - 1;
}
// first row step j + 1 adds to the ring
__host__ __device__ constexpr int f_new1(int j) {
  return f_hi1(j) + 1 > f_lo1(j + 1) ? f_hi1(j) + 1 : f_lo1(j + 1);
}
__host__ __device__ constexpr int f_lo2(int j) { return 2 * ((32 * kFTiles * j) / OW2); }
__host__ __device__ constexpr int f_hi2(int j) {
  const int e = 32 * kFTiles * (j + 1) - 1 < kFPix2 - 1 ? 32 * kFTiles * (j + 1) - 1 : kFPix2 - 1;
  const int r = 2 * (e / OW2) + 3;
  return r < OH - 1 ? r : OH - 1;
}
constexpr bool f_rings_fit() {
  for (int j = 0; j + 1 < kFSteps1; ++j)
    if (f_hi1(j + 1) - f_lo1(j) + 1 > kFRing1 || f_hi1(j + 1) - f_new1(j) + 1 > kFNew)
      return false;
  for (int j = 0; j < kFSteps2; ++j)
    if (f_hi2(j) - f_lo2(j) + 1 > kFRing2) return false;
  return (f_hi1(0) - f_lo1(0) + 1) * (IW / 4) <= kF0 * kFT;
}
static_assert(f_rings_fit(), "dt_conv12 ring sizes");

struct FusedConvLds {
  half8 w1[16 * 64];
  half8 w2[32 * 64];
  union {
    uint2 in[kFRing1 * IW];                    // A: input rows, 4 x fp16 per pixel
    unsigned char c2[kFRing2 * kFRow2];        // C: conv1 rows, conv32 layout
  } ring;
  float b1[CO], b2[CO], sc[CO], sh[CO];
  float red[kFW][CO][3];
};

template <bool kRef>
__global__ void __launch_bounds__(kFT, 1)   // one wave per SIMD: 512 registers a lane
conv12_kernel(int n, const float* __restrict__ ring, int slots, int s0, int s1, int s2,
              const half8* __restrict__ w1frag, const float* __restrict__ b1,
              const float* __restrict__ g1, const float* __restrict__ be1, float eps1,
              const half8* __restrict__ w2frag, const float* __restrict__ b2,
              __half* __restrict__ y2, float* __restrict__ part2, float slope) {
  __shared__ __attribute__((aligned(16))) FusedConvLds S;
  C12R(0);
  C12T(2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, h = lane >> 5;
  for (int i = tid; i < 16 * 64; i += kFT) S.w1[i] = w1frag[i];
  for (int i = tid; i < 32 * 64; i += kFT) S.w2[i] = w2frag[i];
  if (tid < CO) {
    S.b1[tid] = b1[tid];
    S.b2[tid] = b2[tid];
  }
  const auto chan = [&](int r) { return (r & 3) + 8 * (r >> 2) + 4 * h; };
  // pixel of tile u of this wave in step j
  const auto pix = [&](int j, int u) { return 32 * (kFTiles * j + kFU * wave + u) + col; };

  {
    const int ns = blockIdx.x;
    const float* base = ring + (size_t)ns * slots * IH * IW;
    const float* q0 = base + (size_t)s0 * IH * IW;
    const float* q1 = base + (size_t)s1 * IH * IW;
    const float* q2 = base + (size_t)s2 * IH * IW;
    // input rows r0.., item i = (row r0 + i / 40, 4-pixel quad i % 40)
    const auto load = [&](int r0, int cnt, int i, float4& a, float4& b, float4& c) {
      if (i < cnt) {
        const size_t off = (size_t)(r0 + i / (IW / 4)) * IW + 4 * (i % (IW / 4));
        a = *reinterpret_cast<const float4*>(q0 + off);
        b = *reinterpret_cast<const float4*>(q1 + off);
        c = *reinterpret_cast<const float4*>(q2 + off);
      }
    };
    const auto put = [&](int r0, int cnt, int i, const float4& a, const float4& b,
                         const float4& c) {
      if (i < cnt) {
        const int r = r0 + i / (IW / 4), q = i % (IW / 4);
        uint2* dst = S.ring.in + (r % kFRing1) * IW + 4 * q;
        const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w},
                    cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const __half2 lo = __floats2half2_rn(av[e], bv[e]);
          const __half2 hi = __floats2half2_rn(cv[e], 0.0f);
          dst[e] = make_uint2(*reinterpret_cast<const uint32_t*>(&lo),
                              *reinterpret_cast<const uint32_t*>(&hi));
        }
      }
    };
    {
      constexpr int cnt = (f_hi1(0) - f_lo1(0) + 1) * (IW / 4);
      float4 a[kF0], b[kF0], c[kF0];
#pragma unroll
      for (int k = 0; k < kF0; ++k) load(f_lo1(0), cnt, tid + k * kFT, a[k], b[k], c[k]);
#pragma unroll
      for (int k = 0; k < kF0; ++k) put(f_lo1(0), cnt, tid + k * kFT, a[k], b[k], c[k]);
    }
    __syncthreads();
    C12T(3);

    // ---- A: conv1, outputs kept in registers ----
    float sum[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) sum[r] = 0.0f;
    uint32_t stg[kFSteps1][kFU][8];
    // the input rows step t adds are loaded kFDepth steps ahead (at step
    // t - kFDepth, into register set t % kFDepth) and written to the ring at
    // the end of step t - 1: ~kFDepth x 7.7 KB in flight per CU against HBM
    // latency.  zl is an opaque 0: the ring is read-only (__restrict__), so
    // without it the compiler issues every step's loads at kernel entry.
    float4 pa[kFDepth][kFPre], pb[kFDepth][kFPre], pc[kFDepth][kFPre];
    const auto issue = [&](int t) {   // step t's new rows (t >= 1)
      int zl;
      asm volatile("v_mov_b32 %0, 0" : "=v"(zl));
      const int d = t % kFDepth;
#pragma unroll
      for (int k = 0; k < kFPre; ++k)
        load(f_new1(t - 1), (f_hi1(t) - f_new1(t - 1) + 1) * (IW / 4), tid + zl + k * kFT,
             pa[d][k], pb[d][k], pc[d][k]);
    };
#pragma unroll
    for (int t = 1; t <= kFDepth && t < kFSteps1; ++t) issue(t);
#pragma unroll
    for (int j = 0; j < kFSteps1; ++j) {
      const bool more = j + 1 < kFSteps1;
      const int nr0 = more ? f_new1(j) : 0;
      const int ncnt = more ? (f_hi1(j + 1) - f_new1(j) + 1) * (IW / 4) : 0;
      if (j >= 1 && j + kFDepth < kFSteps1) issue(j + kFDepth);
      f32x16 acc[kFU];
      int rb0[kFU];
      const uint2* src[kFU];
      bool valid[kFU];
#pragma unroll
      for (int u = 0; u < kFU; ++u) {
        const int p = pix(j, u);
        valid[u] = p < kFPix1;
        const int pp = valid[u] ? p : 0;
        const int oy = pp / OW, ox = pp - oy * OW;
        rb0[u] = (2 * oy) % kFRing1;
        src[u] = S.ring.in + 2 * ox + 2 * h;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[u][r] = S.b1[chan(r)];
      }
      // k-step s + 1's fragments load while step s's MFMAs run (the sched
      // barriers keep the scheduler from hoisting all 48 loads at once)
      half8 af[2], bf[2][kFU];
      const auto frag1 = [&](int s, int b) {
        const int ky = s >> 1, kx0 = (s & 1) * 4;
        af[b] = S.w1[s * 64 + lane];
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
          const int rr = rb0[u] + ky >= kFRing1 ? rb0[u] + ky - kFRing1 : rb0[u] + ky;
          bf[b][u] = *reinterpret_cast<const half8*>(src[u] + rr * IW + kx0);
        }
      };
      frag1(0, 0);
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        if (s + 1 < 16) frag1(s + 1, (s + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < kFU; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s & 1], bf[s & 1][u], acc[u], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int u = 0; u < kFU; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float v0 = valid[u] ? lrelu(acc[u][2 * q], slope) : 0.0f;
          const float v1 = valid[u] ? lrelu(acc[u][2 * q + 1], slope) : 0.0f;
          sum[2 * q] += v0;
          sum[2 * q + 1] += v1;
          const __half2 hv = __floats2half2_rn(v0, v1);
          stg[j][u][q] = *reinterpret_cast<const uint32_t*>(&hv);
        }
      // pin this step's results here: otherwise the compiler sinks the
      // epilogue to the end and keeps every step's accumulator live.  The
      // first kFAgpr steps' outputs live in AGPRs (MFMA accumulators use 16),
      // the rest in VGPRs
#pragma unroll
      for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(sum[r]));
#pragma unroll
      for (int u = 0; u < kFU; ++u)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (j < kFAgpr)
            asm volatile("" : "+a"(stg[j][u][q]));
          else
            asm volatile("" : "+v"(stg[j][u][q]));
        }
      if (more) {
        const int d = (j + 1) % kFDepth;
#pragma unroll
        for (int k = 0; k < kFPre; ++k) put(nr0, ncnt, tid + k * kFT, pa[d][k], pb[d][k], pc[d][k]);
      }
      __syncthreads();
    }

    C12T(4);
    // ---- B: the sample's BatchNorm (reference mode), applied in the registers ----
    if (kRef) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = sum[r];
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
        if (col == 0) S.red[wave][chan(r)][0] = v;
      }
      __syncthreads();
      if (tid < CO) {
        float t = 0.0f;
        for (int w = 0; w < kFW; ++w) t += S.red[w][tid][0];
        S.sc[tid] = t / (float)kFPix1;   // the mean, for now
      }
      __syncthreads();
      // q outer: only one channel pair's mean is live at a time
      float m2[16];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float mu0 = S.sc[chan(2 * q)], mu1 = S.sc[chan(2 * q + 1)];
        float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
        for (int j = 0; j < kFSteps1; ++j)
#pragma unroll
          for (int u = 0; u < kFU; ++u)
            if (pix(j, u) < kFPix1) {
              const float2 f = __half22float2(__builtin_bit_cast(__half2, stg[j][u][q]));
              const float d0 = f.x - mu0, d1 = f.y - mu1;
              a0 += d0 * d0;
              a1 += d1 * d1;
            }
        m2[2 * q] = a0;
        m2[2 * q + 1] = a1;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = m2[r];
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 32);
        if (col == 0) S.red[wave][chan(r)][1] = v;
      }
      __syncthreads();
      if (tid < CO) {
        float t = 0.0f;
        for (int w = 0; w < kFW; ++w) t += S.red[w][tid][1];
        const float mean = S.sc[tid];
        const float scl = g1[tid] / sqrtf(t / (float)kFPix1 + eps1);
        S.sh[tid] = be1[tid] - mean * scl;
        S.sc[tid] = scl;
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float c0 = S.sc[chan(2 * q)], h0 = S.sh[chan(2 * q)];
        const float c1 = S.sc[chan(2 * q + 1)], h1 = S.sh[chan(2 * q + 1)];
#pragma unroll
        for (int j = 0; j < kFSteps1; ++j)
#pragma unroll
          for (int u = 0; u < kFU; ++u) {
            stg[j][u][q] = norm_pair(stg[j][u][q], c0, h0, c1, h1);
            if (j < kFAgpr) asm volatile("" : "+a"(stg[j][u][q]));   // back to its AGPR
          }
      }
    }

    C12T(5);
    // ---- C: conv2 from the registers through the second ring ----
    float w_cnt = 0.0f, w_mean[16], w_m2[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) w_mean[r] = w_m2[r] = 0.0f;
#pragma unroll
    for (int j2 = 0; j2 < kFSteps2; ++j2) {
      __syncthreads();   // A's ring / the previous step's readers are done
      // the conv1 rows f_lo2(j2)..f_hi2(j2) into the ring (row r in slot r % kFRing2).
      // zq is an opaque 0: without it the compiler computes every tile's row
      // and ring offsets once for all four steps and keeps them live (spills)
      int zq;
      asm volatile("v_mov_b32 %0, 0" : "=v"(zq));
#pragma unroll
      for (int j = 0; j < kFSteps1; ++j)
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
          const int p = pix(j, u) + zq;
          const int row = p / OW;
          if (p < kFPix1 && row >= f_lo2(j2) && row <= f_hi2(j2)) {
            const int ox = p - row * OW;
            unsigned char* dst = S.ring.c2 + (row % kFRing2) * kFRow2 + 8 * h;
#pragma unroll
            for (int g = 0; g < 4; ++g)
              *reinterpret_cast<uint2*>(dst + ring_off<OW, 2>(ox, g)) =
                  make_uint2(stg[j][u][2 * g], stg[j][u][2 * g + 1]);
          }
        }
      __syncthreads();
      if (j2 == 0) C12T(6);
      f32x16 acc[kFU];
      int row[kFU][4], off[kFU][8];
      bool valid[kFU];
      int pv[kFU];
#pragma unroll
      for (int u = 0; u < kFU; ++u) {
        const int p = pix(j2, u);
        valid[u] = p < kFPix2;
        pv[u] = p;
        const int pp = valid[u] ? p : 0;
        const int oy = pp / OW2, ox = pp - oy * OW2;
#pragma unroll
        for (int ky = 0; ky < 4; ++ky) row[u][ky] = ((2 * oy + ky) % kFRing2) * kFRow2;
#pragma unroll
        for (int q = 0; q < 8; ++q)
          off[u][q] = ring_off<OW, 2>(2 * ox + (q >> 1), 2 * (q & 1) + h);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[u][r] = S.b2[chan(r)];
      }
      half8 af[2], bf[2][kFU];
      const auto frag2 = [&](int s, int b) {
        af[b] = S.w2[s * 64 + lane];
#pragma unroll
        for (int u = 0; u < kFU; ++u)
          bf[b][u] = *reinterpret_cast<const half8*>(S.ring.c2 + row[u][s >> 3] + off[u][s & 7]);
      };
      frag2(0, 0);
#pragma unroll
      for (int s = 0; s < 32; ++s) {   // s = 8 ky + (kx, channel half)
        if (s + 1 < 32) frag2(s + 1, (s + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < kFU; ++u)
          acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[s & 1], bf[s & 1][u], acc[u], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int u = 0; u < kFU; ++u) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = lrelu(acc[u][r], slope);
        if (valid[u]) {
          __half* dst = y2 + ((size_t)ns * kFPix2 + pv[u]) * CO;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const __half2 v0 = __floats2half2_rn(v[4 * q + 0], v[4 * q + 1]);
            const __half2 v1 = __floats2half2_rn(v[4 * q + 2], v[4 * q + 3]);
            *reinterpret_cast<uint2*>(dst + 8 * q + 4 * h) =
                make_uint2(*reinterpret_cast<const uint32_t*>(&v0),
                           *reinterpret_cast<const uint32_t*>(&v1));
          }
          if (kRef) {   // Welford over this lane's pixels
            w_cnt += 1.0f;
            const float inv = 1.0f / w_cnt;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float d = v[r] - w_mean[r];
              w_mean[r] += d * inv;
              w_m2[r] += d * (v[r] - w_mean[r]);
            }
          }
        }
      }
    }
    if (kRef) {   // merge: the 32 lanes of each half, then the waves (conv32_kernel kOut 0)
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
          S.red[wave][chan(r)][0] = w_cnt;
          S.red[wave][chan(r)][1] = w_mean[r];
          S.red[wave][chan(r)][2] = w_m2[r];
        }
      __syncthreads();
      if (tid < CO) {
        float cnt = 0.0f, mean = 0.0f, m2 = 0.0f;
        for (int w = 0; w < kFW; ++w) {
          const float nb = S.red[w][tid][0];
          if (nb <= 0.0f) continue;
          const float tot = cnt + nb, d = S.red[w][tid][1] - mean;
          mean += d * (nb / tot);
          m2 += S.red[w][tid][2] + d * d * (cnt * nb / tot);
          cnt = tot;
        }
        float* pp2 = part2 + ((size_t)ns * CO + tid) * 2;
        pp2[0] = mean;
        pp2[1] = m2;
      }
    }
  }
  C12T(7);
  C12R(1);
}

}  // namespace

extern "C" int dt_conv1(const float* ring, int32_t n, int32_t slots, const int32_t* order,
                        const void* wfrag, const float* bias, void* y, float* partials,
                        float slope, void* stream) {
  if (!ring || !wfrag || !bias || !y || !order || n < 0 || slots < 3) return DT_E_ARG;
  for (int i = 0; i < 3; ++i)
    if (order[i] < 0 || order[i] >= slots) return DT_E_ARG;
  if (n == 0) return DT_OK;
  if (!conv1_banded()) {
    static int grid = 0;   // resident workgroups, persistent
    if (!grid) {
      int dev = 0, cus = 256, per = 2;
      if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, conv1s_kernel<true>, kSThreads, 0) !=
              hipSuccess || per < 1)
        per = 1;
      grid = per * cus;
    }
    const int g = n < grid ? n : grid;
    if (partials)
      hipLaunchKernelGGL(conv1s_kernel<true>, dim3(g), dim3(kSThreads), 0, (hipStream_t)stream, n,
                         ring, slots, order[0], order[1], order[2], (const half8*)wfrag, bias,
                         (__half*)y, partials, slope);
    else
      hipLaunchKernelGGL(conv1s_kernel<false>, dim3(g), dim3(kSThreads), 0, (hipStream_t)stream,
                         n, ring, slots, order[0], order[1], order[2], (const half8*)wfrag, bias,
                         (__half*)y, nullptr, slope);
    return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
  }
  const int items = n * kBands;
  const int grid = items < persistent_grid() ? items : persistent_grid();
  hipLaunchKernelGGL(conv1_kernel, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, items,
                     ring, slots, order[0], order[1], order[2], (const half8*)wfrag, bias,
                     (__half*)y, partials, slope);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

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
                     partials, gamma, beta, eps, conv1_bands(), conv1_band_rows());
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

extern "C" int32_t dt_conv1_bands(void) { return conv1_bands(); }

#ifdef DTSIM_STAMPS
extern "C" int dt_diag_c12stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c12stamps), sizeof(g_c12stamps)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int dt_conv12(const float* ring, int32_t n, int32_t slots, const int32_t* order,
                         const void* w1frag, const float* b1, const float* gamma1,
                         const float* beta1, float eps1, const void* w2frag, const float* b2,
                         void* y2, float* part2, float slope, void* stream) {
  if (!ring || !w1frag || !b1 || !w2frag || !b2 || !y2 || !order || n < 0 || slots < 3)
    return DT_E_ARG;
  const bool ref = gamma1 != nullptr;
  if (ref && (!beta1 || !part2)) return DT_E_ARG;
  for (int i = 0; i < 3; ++i)
    if (order[i] < 0 || order[i] >= slots) return DT_E_ARG;
  if (n == 0) return DT_OK;
  const int grid = n;   // one workgroup per sample
  if (ref)
    hipLaunchKernelGGL(conv12_kernel<true>, dim3(grid), dim3(kFT), 0, (hipStream_t)stream, n,
                       ring, slots, order[0], order[1], order[2], (const half8*)w1frag, b1,
                       gamma1, beta1, eps1, (const half8*)w2frag, b2, (__half*)y2, part2, slope);
  else
    hipLaunchKernelGGL(conv12_kernel<false>, dim3(grid), dim3(kFT), 0, (hipStream_t)stream, n,
                       ring, slots, order[0], order[1], order[2], (const half8*)w1frag, b1,
                       nullptr, nullptr, 0.0f, (const half8*)w2frag, b2, (__half*)y2, nullptr,
                       slope);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

// conv2..conv4 of the reference actor (see include/dtactor.h)
extern "C" int dt_conv32(int32_t layer, int32_t n, const void* x, const void* wfrag,
                         const float* bias, const float* prev_part, const float* in_gamma,
                         const float* in_beta, float in_eps, void* y, float* part,
                         const float* out_gamma, const float* out_beta, float out_eps,
                         float slope, void* stream) {
  if (!x || !wfrag || !bias || !y || n < 0) return DT_E_ARG;
  if (n == 0) return DT_OK;
  const bool in = prev_part != nullptr;
  if (in && (!in_gamma || !in_beta)) return DT_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  switch (layer) {
    case 2:   // 57x77 -> 27x37, stride 2; input norm from conv1's bands
      if (in != (part != nullptr)) return DT_E_ARG;
      if (in && conv1_banded())
        return launch_conv32<57, 77, 27, 37, 2, kConv2Waves, 1, 0, kBand>(
            n, x, wfrag, bias, prev_part, in_gamma, in_beta, in_eps, y, part, nullptr, nullptr,
            0.f, slope, s);
      return in ? launch_conv32<57, 77, 27, 37, 2, kConv2Waves, 1, 0, 57>(
                      n, x, wfrag, bias, prev_part, in_gamma, in_beta, in_eps, y, part,
                      nullptr, nullptr, 0.f, slope, s)
                : launch_conv32<57, 77, 27, 37, 2, kConv2Waves, 0, 1>(
                      n, x, wfrag, bias, nullptr, nullptr, nullptr, 0.f, y, nullptr, nullptr,
                      nullptr, 0.f, slope, s);
    case 3:   // 27x37 -> 12x17, stride 2; input norm from conv2's per-sample statistics
      if (in != (part != nullptr)) return DT_E_ARG;
      return in ? launch_conv32<27, 37, 12, 17, 2, kConv3Waves, 1, 0>(
                      n, x, wfrag, bias, prev_part, in_gamma, in_beta, in_eps, y, part,
                      nullptr, nullptr, 0.f, slope, s)
                : launch_conv32<27, 37, 12, 17, 2, kConv3Waves, 0, 1>(
                      n, x, wfrag, bias, nullptr, nullptr, nullptr, 0.f, y, nullptr, nullptr,
                      nullptr, 0.f, slope, s);
    case 4:   // 12x17 -> 9x14, stride 1, whole sample per step; its own norm in-kernel; flattened
      if (in != (out_gamma != nullptr)) return DT_E_ARG;
      return in ? launch_conv32<12, 17, 9, 14, 1, kConv4Waves, 1, 2>(
                      n, x, wfrag, bias, prev_part, in_gamma, in_beta, in_eps, y, nullptr,
                      out_gamma, out_beta, out_eps, slope, s)
                : launch_conv32<12, 17, 9, 14, 1, kConv4Waves, 0, 3>(
                      n, x, wfrag, bias, nullptr, nullptr, nullptr, 0.f, y, nullptr, nullptr,
                      nullptr, 0.f, slope, s);
    default:
      return DT_E_ARG;
  }
}
