// Shared pieces of the actor's convolution kernels: dtconv.hip (fp16 MFMA,
// the fast mode) and dtconvx.hip (the same chain at float32 accuracy on fp16
// MFMA, "x3").  Types, the LeakyReLU form, the two-weight-set split of a
// persistent grid, the per-sample centring of reference-mode outputs and the
// row-stream geometry of conv1 (120x160 input, 8x8 stride 2 -> 57x77).
#ifndef AIDO1_AMD_DTCONV_COMMON_H
#define AIDO1_AMD_DTCONV_COMMON_H

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dtconv {

using half8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;

constexpr int CO = 32;   // output channels of every conv of the actor

// LeakyReLU for 0 <= s <= 1 as two instructions (a multiply and a max)
__device__ __forceinline__ float lrelu2(float v, float s) { return fmaxf(v, v * s); }

// Reference mode keeps each sample's activations CENTRED: the stored value is
// v - c with c the sample's pixel-0 output of the channel, and the statistics
// are those of the stored values (M2 does not change, the mean moves by c), so
// the next layer's norm (x - mean) * invstd is unchanged.  A channel that is
// nearly flat over a frame is divided by a tiny standard deviation; stored
// uncentred its rounding (~2^-11 |v| in fp16) is amplified by that 1 / std,
// centred the rounding is of |v - c| ~ the channel's own spread.  The sample's
// first step publishes c (wave 0, pixel 0 = lanes 0 and 32) and a barrier
// makes it visible; later steps read it (rewritten only after the step barrier
// that ends the sample).  `first` is workgroup-uniform.  Register r of a
// 32x32 MFMA tile holds channel (r & 3) + 8 (r >> 2) + 4 h (h = lane half).
__device__ __forceinline__ void centre_px32(float (&v)[16], float* s_c, bool publish, bool first,
                                            int h) {
  if (publish)
#pragma unroll
    for (int r = 0; r < 16; ++r) s_c[(r & 3) + 8 * (r >> 2) + 4 * h] = v[r];
  if (first) __syncthreads();
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] -= s_c[(r & 3) + 8 * (r >> 2) + 4 * h];
}

// ---- two weight sets in one launch -----------------------------------------------
// Samples [0, n0) use the launch's weights, [n0, n) a second set (the exploiting
// explorers' actor): the persistent workgroups split in proportion, g0 for the
// first set, the rest for the second, and each loads only its own set.  One set:
// n0 = n, g0 = gridDim.x.
struct WeightSplit {
  int n0, g0;
  const void* wfrag;
  const float *bias, *in_gamma, *in_beta, *out_gamma, *out_beta;
};
struct SplitPart {
  bool set2;
  int bid, gdim, sbeg, send, my;   // this WG's index / count in its part, its samples
};
__device__ __forceinline__ SplitPart split_part(const WeightSplit& ws, int n) {
  SplitPart p;
  p.set2 = (int)blockIdx.x >= ws.g0;
  p.bid = p.set2 ? (int)blockIdx.x - ws.g0 : (int)blockIdx.x;
  p.gdim = p.set2 ? (int)gridDim.x - ws.g0 : ws.g0;
  p.sbeg = p.set2 ? ws.n0 : 0;
  p.send = p.set2 ? n : ws.n0;
  const int nloc = p.send - p.sbeg;
  p.my = nloc > p.bid ? (nloc - p.bid + p.gdim - 1) / p.gdim : 0;
  return p;
}
// host: the grid of a launch over n samples (n0 of them with the first set) on
// `grid` resident workgroups; fills ws.n0 / ws.g0
inline int split_grid(WeightSplit& ws, int n, int n0, int grid) {
  if (n0 <= 0 || n0 >= n) {   // one set
    ws.n0 = n;
    ws.g0 = n < grid ? n : grid;
    return ws.g0;
  }
  int g0 = (int)(((long long)grid * n0 + n / 2) / n);
  g0 = g0 < 1 ? 1 : (g0 > grid - 1 ? grid - 1 : g0);
  const int g1raw = grid - g0;
  ws.n0 = n0;
  ws.g0 = n0 < g0 ? n0 : g0;
  const int g1 = (n - n0) < g1raw ? (n - n0) : g1raw;
  return ws.g0 + g1;
}

// ---- conv1's row stream ------------------------------------------------------------
// A persistent workgroup of kSW waves streams whole samples through a ring of
// kSRing input rows in LDS; a step is kSW tiles of 32 consecutive output
// pixels, one per wave.  Step j reads input rows s_lo(j)..s_hi(j); the rows
// the step after it adds are s_first_new(j)..s_last_new(j) (the last step of
// a sample adds the next sample's first rows).
namespace c1 {
constexpr int IH = 120, IW = 160, OH = 57, OW = 77;
constexpr int kSW = 4;
constexpr int kSThreads = 64 * kSW;
constexpr int kSPix = OH * OW;                          // 4389
constexpr int kSTiles = (kSPix + 31) / 32;              // 138
constexpr int kSSteps = (kSTiles + kSW - 1) / kSW;      // 35
constexpr int kSStepPix = 32 * kSW;
constexpr int kSRing = 32;                              // rows (a power of two)
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
}  // namespace c1

// resident workgroups a CU of `kern` at `threads` (the persistent grids)
template <typename K>
inline int resident_grid(K kern, int threads, int cap) {
  int dev = 0, cus = 256, per = 1;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, threads, 0) != hipSuccess || per < 1)
    per = 1;
  if (cap > 0 && cap < per) per = cap;
  return per * cus;
}

}  // namespace dtconv

#endif  // AIDO1_AMD_DTCONV_COMMON_H
