// Observation path device code: the build-defined 120x160 top-down raster and
// the features/line_detector1.py LineDetectorHSV filter (OpenCV 8-bit
// semantics: cvtColor BGR2HSV, inRange, dilate MORPH_ELLIPSE, Canny L1 with
// apertureSize 3), one workgroup per image with the image resident in LDS.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dtsim.h"

namespace dr {

constexpr int H = DT_OBS_H, W = DT_OBS_W, NPIX = H * W;
constexpr int kThreads = 256;
constexpr float kRes = 0.01f;        // metres per pixel
constexpr float kInvRes = 100.0f;

// Raster bytes.  The background is a plain byte (floor / grass / road); the
// markings are OR-ed into it, so yellow and white can be drawn in any order
// and concurrently with the background fix-up: yellow sets bit 2 (4..6 =
// yellow over any background), white sets bits 0-2 (7 = white, also over
// yellow) — exactly "yellow drawn first, white over it" of the oracle.
// kPalette maps every byte value to its colour (packed B | G << 8 | R << 16).
enum : uint8_t { PAL_FLOOR = 0, PAL_OFFROAD = 1, PAL_ROAD = 2, PAL_RED = 3, PAL_YELLOW = 4,
                 PAL_WHITE = 7, PAL_N = 8 };
__host__ __device__ constexpr uint32_t rgb_pack(uint32_t r, uint32_t g, uint32_t b) {
  return b | (g << 8) | (r << 16);
}
constexpr uint32_t kYellowRgb = rgb_pack(255, 230, 0);
constexpr uint32_t kPalette[PAL_N] = {
    rgb_pack(0, 0, 0),        // floor / outside the map
    rgb_pack(72, 132, 52),    // grass (any non-drivable tile)
    rgb_pack(56, 56, 60),     // road surface
    rgb_pack(220, 30, 30),    // red stop line (never drawn: intersections carry no markings)
    kYellowRgb,               // yellow centre line over floor / grass / road
    kYellowRgb,
    kYellowRgb,
    rgb_pack(250, 250, 250)};  // white edge line
// The grey level of a palette byte: PreliminaryTransformer's rgb2gray of its
// colour (0.2125 R + 0.7154 G + 0.0721 B on [0, 1] channels in float64, then
// float32; utils/reward_shaping/env_utils.py:48-51).  A grey frame is this
// table applied to the frame's palette bytes, so a palette-index frame (u8)
// decodes to the grey frame bit for bit (dt_palette_gray, dt_conv1_index_split,
// dt_frame_gather).
__host__ __device__ constexpr float pal_gray_of(uint32_t p) {
  return (float)(((double)((p >> 16) & 255) * (1.0 / 255.0) * 0.2125 +
                  (double)((p >> 8) & 255) * (1.0 / 255.0) * 0.7154) +
                 (double)(p & 255) * (1.0 / 255.0) * 0.0721);
}
constexpr float kPalGray[PAL_N] = {pal_gray_of(kPalette[0]), pal_gray_of(kPalette[1]),
                                   pal_gray_of(kPalette[2]), pal_gray_of(kPalette[3]),
                                   pal_gray_of(kPalette[4]), pal_gray_of(kPalette[5]),
                                   pal_gray_of(kPalette[6]), pal_gray_of(kPalette[7])};

// OpenCV RGB2HSV_b fixed-point tables (hsv_shift = 12):
//   sdiv[i] = round((255 << 12) / i), hdiv180[i] = round((180 << 12) / (6 i)).
// No exact .5 ties exist for i < 256, so round = floor(x + 1/2) in integers.
struct HsvTables {
  int sdiv[256];
  int hdiv[256];
};
constexpr HsvTables make_hsv_tables() {
  HsvTables t{};
  for (int i = 1; i < 256; ++i) {
    t.sdiv[i] = (2 * (255 << 12) + i) / (2 * i);
    t.hdiv[i] = (2 * ((180 << 12) / 6) + i) / (2 * i);
  }
  return t;
}

// Line-detector parameters as the kernels use them.
struct LineDev {
  uint8_t lo[4][3], hi[4][3];  // white, yellow, red1, red3 ranges (red2/red4 = hi of 2,3)
  uint64_t dil_mask;           // k x k ellipse, bit (dy+3)*7 + (dx+3)
  int32_t dil_r;               // k / 2
  int32_t canny_lo, canny_hi;  // cvFloor of the thresholds (L1)
  uint32_t pal_bits[2];        // colour bits of palette entries 0-3 / 4-7 (one byte each)
};

// bits of the per-pixel work byte
constexpr uint8_t B_WHITE = 1, B_YELLOW = 2, B_RED = 4, B_DIR_SHIFT = 3;  // dir: 2 bits
constexpr uint8_t B_CAND = 0x20, B_EDGE = 0x40;

__host__ __device__ inline void bgr_to_hsv(const int* __restrict__ sdiv, const int* __restrict__ hdiv,
                                  int b, int g, int r, int& h, int& s, int& v) {
  v = b > g ? b : g;
  v = v > r ? v : r;
  int vmin = b < g ? b : g;
  vmin = vmin < r ? vmin : r;
  const int diff = v - vmin;
  const int vr = v == r ? -1 : 0;
  const int vg = v == g ? -1 : 0;
  s = (diff * sdiv[v] + (1 << 11)) >> 12;
  int hh = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
  hh = (hh * hdiv[diff] + (1 << 11)) >> 12;
  hh += hh < 0 ? 180 : 0;
  h = hh;
}

__host__ __device__ inline bool in_range(const uint8_t lo[3], const uint8_t hi[3], int h, int s, int v) {
  return lo[0] <= h && h <= hi[0] && lo[1] <= s && s <= hi[1] && lo[2] <= v && v <= hi[2];
}

__host__ __device__ inline uint8_t color_bits(const LineDev& L, int h, int s, int v) {
  uint8_t bits = 0;
  if (in_range(L.lo[0], L.hi[0], h, s, v)) bits |= B_WHITE;
  if (in_range(L.lo[1], L.hi[1], h, s, v)) bits |= B_YELLOW;
  if (in_range(L.lo[2], L.hi[2], h, s, v) || in_range(L.lo[3], L.hi[3], h, s, v)) bits |= B_RED;
  return bits;
}

// Sobel 3x3 (BORDER_REPLICATE) on the 3 channels of a BGR source, keeping the
// channel of largest |dx|+|dy| (first max in B, G, R order) as Canny does for
// multi-channel input.  Fetch(r, c) -> packed B | G<<8 | R<<16.
template <class Fetch>
__device__ inline void sobel_max(const Fetch& fetch, int r, int c, int hgt, int wid, int& dx,
                                 int& dy, int& mag) {
  const int r0 = r > 0 ? r - 1 : 0, r2 = r < hgt - 1 ? r + 1 : hgt - 1;
  const int c0 = c > 0 ? c - 1 : 0, c2 = c < wid - 1 ? c + 1 : wid - 1;
  const uint32_t p00 = fetch(r0, c0), p01 = fetch(r0, c), p02 = fetch(r0, c2);
  const uint32_t p10 = fetch(r, c0), p12 = fetch(r, c2);
  const uint32_t p20 = fetch(r2, c0), p21 = fetch(r2, c), p22 = fetch(r2, c2);
  mag = -1;
  dx = dy = 0;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const int sh = 8 * ch;
    const int a00 = (p00 >> sh) & 255, a01 = (p01 >> sh) & 255, a02 = (p02 >> sh) & 255;
    const int a10 = (p10 >> sh) & 255, a12 = (p12 >> sh) & 255;
    const int a20 = (p20 >> sh) & 255, a21 = (p21 >> sh) & 255, a22 = (p22 >> sh) & 255;
    const int gx = (a02 + 2 * a12 + a22) - (a00 + 2 * a10 + a20);
    const int gy = (a20 + 2 * a21 + a22) - (a00 + 2 * a01 + a02);
    const int m = (gx < 0 ? -gx : gx) + (gy < 0 ? -gy : gy);
    if (m > mag) {
      mag = m;
      dx = gx;
      dy = gy;
    }
  }
}

// Canny non-maximum-suppression direction class of (dx, dy):
// 0 = compare left/right, 1 = up/down, 2 = diagonal s = +1, 3 = diagonal s = -1.
__device__ inline uint8_t nms_dir(int dx, int dy) {
  constexpr int TG22 = 13573;  // (int)(tan(22.5 deg) * 2^15 + 0.5)
  const int x = dx < 0 ? -dx : dx;
  const int y = (dy < 0 ? -dy : dy) << 15;
  const int tg22x = x * TG22;
  if (y < tg22x) return 0;
  const int tg67x = tg22x + (x << 16);
  if (y > tg67x) return 1;
  return ((dx ^ dy) < 0) ? 3 : 2;
}

}  // namespace dr
