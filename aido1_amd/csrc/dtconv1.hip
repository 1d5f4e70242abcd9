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

#include "../../include/dtactor.h"

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

__device__ __forceinline__ float lrelu(float v, float s) { return v > 0.0f ? v : v * s; }

__global__ void __launch_bounds__(kThreads)
conv1_kernel(const float* __restrict__ ring, int slots, int s0, int s1, int s2,
             const half8* __restrict__ wfrag, const float* __restrict__ bias,
             __half* __restrict__ y, float* __restrict__ partials, float slope) {
  __shared__ __attribute__((aligned(16))) uint2 img[kInRows * IW];   // 4 x fp16 per pixel
  __shared__ float red[kWaves][2][CO];
  const int n = blockIdx.x / kBands, band = blockIdx.x - n * kBands;
  const int oy0 = band * kBand;
  const int rows_out = (OH - oy0) < kBand ? (OH - oy0) : kBand;
  const int band_pix = rows_out * OW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- load: input rows 2*oy0 .. 2*oy0 + kInRows - 1, 4 px per item ----------------
  const float* base = ring + (size_t)n * slots * IH * IW;
  const float* p0 = base + (size_t)s0 * IH * IW;
  const float* p1 = base + (size_t)s1 * IH * IW;
  const float* p2 = base + (size_t)s2 * IH * IW;
  for (int it = tid; it < kInRows * (IW / 4); it += kThreads) {
    const int r = it / (IW / 4), q = it - r * (IW / 4);
    const int iy = 2 * oy0 + r;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, c = a;
    if (iy < IH) {
      const size_t off = (size_t)iy * IW + 4 * q;
      a = *reinterpret_cast<const float4*>(p0 + off);
      b = *reinterpret_cast<const float4*>(p1 + off);
      c = *reinterpret_cast<const float4*>(p2 + off);
    }
    const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w},
                cv[4] = {c.x, c.y, c.z, c.w};
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
  // weights: this lane's A fragments of the 16 k-steps (row = out channel)
  half8 wa[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) wa[s] = wfrag[s * 64 + lane];
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
  if (!partials) return;

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
  __shared__ float mean_s[CO];
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
}

// Reference mode: merge the bands' (mean, M2) per sample and channel (Chan et
// al.), then y = (y - mean) / sqrt(var + eps) * gamma + beta in place (biased
// variance: BatchNorm2d's train-mode normalisation of a batch of one).
__global__ void __launch_bounds__(256)
conv1_norm_kernel(__half* __restrict__ y, const float* __restrict__ partials,
                  const float* __restrict__ gamma, const float* __restrict__ beta, float eps) {
  __shared__ float sc[CO], sh[CO];
  const int n = blockIdx.x, tid = threadIdx.x;
  if (tid < CO) {
    const float* pp = partials + (size_t)n * kBands * CO * 2;
    float cnt = 0.0f, mean = 0.0f, m2 = 0.0f;
    for (int b = 0; b < kBands; ++b) {
      const float nb = (float)(((OH - b * kBand) < kBand ? (OH - b * kBand) : kBand) * OW);
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

}  // namespace

extern "C" int dt_conv1(const float* ring, int32_t n, int32_t slots, const int32_t* order,
                        const void* wfrag, const float* bias, void* y, float* partials,
                        float slope, void* stream) {
  if (!ring || !wfrag || !bias || !y || !order || n < 0 || slots < 3) return DT_E_ARG;
  for (int i = 0; i < 3; ++i)
    if (order[i] < 0 || order[i] >= slots) return DT_E_ARG;
  if (n == 0) return DT_OK;
  hipLaunchKernelGGL(conv1_kernel, dim3(n * kBands), dim3(kThreads), 0, (hipStream_t)stream,
                     ring, slots, order[0], order[1], order[2], (const half8*)wfrag, bias,
                     (__half*)y, partials, slope);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

extern "C" int dt_conv1_norm(void* y, int32_t n, const float* partials, const float* gamma,
                             const float* beta, float eps, void* stream) {
  if (!y || !partials || !gamma || !beta || n < 0) return DT_E_ARG;
  if (n == 0) return DT_OK;
  hipLaunchKernelGGL(conv1_norm_kernel, dim3(n), dim3(256), 0, (hipStream_t)stream, (__half*)y,
                     partials, gamma, beta, eps);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

extern "C" int32_t dt_conv1_bands(void) { return kBands; }
