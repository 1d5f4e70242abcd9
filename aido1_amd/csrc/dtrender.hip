// Observation path: build-defined 120x160 ego-centric top-down raster of the
// lane markings fused with the features/line_detector1.py colour/edge filter
// and PreliminaryTransformer's grey conversion.  render_kernel (below, "fused
// render kernel") runs one 768-thread workgroup per environment and keeps the
// frame in LDS (~71 KB: 4-pixel palette words + a 16-bit work image) until its
// outputs are written: grey into the frame ring, four u8 masks.  Markings are
// Bresenham polylines (utils/bresenham.py semantics: both endpoints,
// major-axis swap, D = 2dy - dx).  line_detect_kernel is the standalone
// LineDetectorHSV on caller-supplied BGR images (dt_line_detect).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "dthandle.h"

namespace {

using namespace dr;

#ifdef DTSIM_STAMPS
// render_kernel per workgroup (diagnostics, tools/render_stamps.py): [0] real
// time at entry, [1] at exit, [2] HW_ID, [3] XCC_ID, [4..15] shader clock at
// the phase points RSTAMP(4..15) (thread 0, after the barrier that ends a phase)
__device__ unsigned long long g_renstamps[4096 * 24];
__device__ inline unsigned ren_hw_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
}
__device__ inline unsigned ren_xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v;
}
#define RENSTAMP(i, v)                                                              \
  do {                                                                              \
    if (threadIdx.x == 0 && e < 4096) g_renstamps[e * 24 + (i)] = (v); \
  } while (0)
#else
#define RENSTAMP(i, v) \
  do {                 \
  } while (0)
#endif
#define RENT(i) RENSTAMP(i, __builtin_amdgcn_s_memtime())

constexpr HsvTables kHsvHost = make_hsv_tables();
__constant__ HsvTables c_hsv = make_hsv_tables();

// ---- marking polylines (host, once per map) ----------------------------------
// Build-defined lane markings from the map's lane curves: per drivable tile and
// lane curve, 9 samples t = k/8 of the Bezier, offset along the curve's right
// normal: a white edge line (5 px wide, centred 0.26 tile to the lane's right)
// and, for curve 0 only, a dashed yellow centre line (0.20 tile to its left,
// every other of the 8 segments).  A line of width w is kW parallel polylines
// 0.7 px apart (closer than 1 px so curved thick lines have no holes): white 7
// (4.2 cm), yellow 4 (2.1 cm).  Intersection tiles get none.
// oracle/render_oracle.c restates this.
constexpr int kSegs = 8, kWhiteW = 7, kYellowW = 4;
constexpr double kWhiteOff = 0.26, kYellowOff = -0.20, kHalfStep = 0.0035;

void bez_host(const double* cp, double t, double& x, double& z, double& dx, double& dz) {
  const double u = 1.0 - t;
  const double c0 = u * u * u, c1 = 3.0 * t * (u * u), c2 = 3.0 * (t * t) * u, c3 = t * t * t;
  x = c0 * cp[0];
  z = c0 * cp[2];
  x = x + c1 * cp[3];
  z = z + c1 * cp[5];
  x = x + c2 * cp[6];
  z = z + c2 * cp[8];
  x = x + c3 * cp[9];
  z = z + c3 * cp[11];
  const double a0 = 3.0 * (u * u), a1 = 6.0 * u * t, a2 = 3.0 * (t * t);
  dx = a0 * (cp[3] - cp[0]);
  dz = a0 * (cp[5] - cp[2]);
  dx = dx + a1 * (cp[6] - cp[3]);
  dz = dz + a1 * (cp[8] - cp[5]);
  dx = dx + a2 * (cp[9] - cp[6]);
  dz = dz + a2 * (cp[11] - cp[8]);
}

void build_marks(const dt_map* m, double ts, std::vector<float4>& yellow,
                 std::vector<float4>& white) {
  const int T = m->width * m->height;
  for (int t = 0; t < T; ++t) {
    // lane markings on straight and curve tiles; intersections are plain road
    // (build-defined: their painted stop lines are not part of this raster)
    if (m->kind[t] <= 0 || m->kind[t] > DT_TILE_CURVE_RIGHT) continue;
    for (int c = 0; c < 2; ++c) {
      const double* cp = m->curves + (size_t)(m->curve_start[t] + c) * 12;
      double px[kSegs + 1], pz[kSegs + 1], rx[kSegs + 1], rz[kSegs + 1];
      for (int k = 0; k <= kSegs; ++k) {
        double dx, dz;
        bez_host(cp, (double)k / kSegs, px[k], pz[k], dx, dz);
        const double n = sqrt(dx * dx + dz * dz);
        rx[k] = (0.0 - dz) / n;  // right of the tangent: cross(tangent, up) = (-tz, tx)
        rz[k] = dx / n;
      }
      for (int w = 0; w < kWhiteW; ++w) {
        const double o = kWhiteOff * ts + (2 * w - (kWhiteW - 1)) * kHalfStep;
        for (int k = 0; k < kSegs; ++k)
          white.push_back(make_float4((float)(px[k] + o * rx[k]), (float)(pz[k] + o * rz[k]),
                                      (float)(px[k + 1] + o * rx[k + 1]),
                                      (float)(pz[k + 1] + o * rz[k + 1])));
      }
      if (c != 0) continue;
      for (int w = 0; w < kYellowW; ++w) {
        const double o = kYellowOff * ts + (2 * w - (kYellowW - 1)) * kHalfStep;
        for (int k = 0; k < kSegs; k += 2)
          yellow.push_back(make_float4((float)(px[k] + o * rx[k]), (float)(pz[k] + o * rz[k]),
                                       (float)(px[k + 1] + o * rx[k + 1]),
                                       (float)(pz[k + 1] + o * rz[k + 1])));
      }
    }
  }
}

LineDev to_line_dev(const dt_line_params& p) {
  LineDev L{};
  memcpy(L.lo[0], p.hsv_white1, 3);
  memcpy(L.hi[0], p.hsv_white2, 3);
  memcpy(L.lo[1], p.hsv_yellow1, 3);
  memcpy(L.hi[1], p.hsv_yellow2, 3);
  memcpy(L.lo[2], p.hsv_red1, 3);
  memcpy(L.hi[2], p.hsv_red2, 3);
  memcpy(L.lo[3], p.hsv_red3, 3);
  memcpy(L.hi[3], p.hsv_red4, 3);
  // getStructuringElement(MORPH_ELLIPSE, (k, k))
  const int k = p.dilation_kernel_size;
  const int r = k / 2;
  L.dil_r = r;
  L.dil_mask = 0;
  if (r == 0) {
    L.dil_mask = 1ull << (3 * 7 + 3);
  } else {
    const double inv_r2 = 1.0 / ((double)r * r);
    for (int i = 0; i < k; ++i) {
      const int dy = i - r;
      const int dxm = (int)lrint(r * sqrt((double)(r * r - dy * dy) * inv_r2));
      const int j1 = r - dxm < 0 ? 0 : r - dxm, j2 = r + dxm + 1 > k ? k : r + dxm + 1;
      for (int j = j1; j < j2; ++j) L.dil_mask |= 1ull << ((dy + 3) * 7 + (j - r + 3));
    }
  }
  double lo = p.canny_lo, hi = p.canny_hi;
  if (lo > hi) {
    const double t = lo;
    lo = hi;
    hi = t;
  }
  L.canny_lo = (int)floor(lo);
  L.canny_hi = (int)floor(hi);
  // colour bits of each palette entry (HSV + inRange once per parameter set)
  L.pal_bits[0] = L.pal_bits[1] = 0;
  for (int i = 0; i < PAL_N; ++i) {
    const uint32_t q = kPalette[i];
    int hh, ss, vv;
    bgr_to_hsv(kHsvHost.sdiv, kHsvHost.hdiv, q & 255, (q >> 8) & 255, (q >> 16) & 255, hh, ss, vv);
    L.pal_bits[i >> 2] |= (uint32_t)color_bits(L, hh, ss, vv) << (8 * (i & 3));
  }
  return L;
}

// ---- device passes -----------------------------------------------------------------
// LineDetectorHSV on caller images.  The per-pixel planes live in LDS (images
// of <= NPIX pixels, line_detect_kernel) or in a caller workspace in HBM (any
// size, line_detect_big_kernel); the passes only see the PixBuf pointers.
struct Lds {
  int16_t mag[NPIX];
  uint8_t work[NPIX];
  int sdiv[256];
  int hdiv[256];
};
struct PixBuf {
  int16_t* mag;     // [h*w] Sobel L1 magnitude (max over the channels)
  uint8_t* work;    // [h*w] colour bits | NMS direction | candidate / edge bits
  const int* sdiv;  // cvtColor's division tables (LDS)
  const int* hdiv;
};

__device__ inline void load_tables(int* sdiv, int* hdiv) {
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    sdiv[i] = c_hsv.sdiv[i];
    hdiv[i] = c_hsv.hdiv[i];
  }
}

// pass A for one pixel: Sobel/NMS dir + colour bits into work, magnitude into mag
template <class Fetch>
__device__ inline void pass_a_pixel(const Fetch& fetch, const PixBuf& S, const LineDev& L, int hgt,
                                    int wid, int r, int c) {
  int dx, dy, m;
  sobel_max(fetch, r, c, hgt, wid, dx, dy, m);
  const uint32_t p = fetch(r, c);
  int h, s, v;
  bgr_to_hsv(S.sdiv, S.hdiv, p & 255, (p >> 8) & 255, (p >> 16) & 255, h, s, v);
  const int idx = r * wid + c;
  S.mag[idx] = (int16_t)m;
  S.work[idx] = color_bits(L, h, s, v) | (uint8_t)(nms_dir(dx, dy) << B_DIR_SHIFT);
}

__device__ inline int mag_at(const PixBuf& S, int hgt, int wid, int r, int c) {
  return ((unsigned)r < (unsigned)hgt && (unsigned)c < (unsigned)wid) ? S.mag[r * wid + c] : 0;
}

// pass B: Canny NMS + thresholds
__device__ inline void pass_b(const PixBuf& S, const LineDev& L, int hgt, int wid) {
  const int np = hgt * wid;
  for (int idx = threadIdx.x; idx < np; idx += blockDim.x) {
    const int m = S.mag[idx];
    if (m <= L.canny_lo) continue;
    const int r = idx / wid, c = idx - r * wid;
    const int dir = (S.work[idx] >> B_DIR_SHIFT) & 3;
    bool keep;
    if (dir == 0) {
      keep = m > mag_at(S, hgt, wid, r, c - 1) && m >= mag_at(S, hgt, wid, r, c + 1);
    } else if (dir == 1) {
      keep = m > mag_at(S, hgt, wid, r - 1, c) && m >= mag_at(S, hgt, wid, r + 1, c);
    } else {
      const int s = dir == 2 ? 1 : -1;
      keep = m > mag_at(S, hgt, wid, r - 1, c - s) && m > mag_at(S, hgt, wid, r + 1, c + s);
    }
    if (keep) S.work[idx] |= (uint8_t)(B_CAND | (m > L.canny_hi ? B_EDGE : 0));
  }
}

// one hysteresis visit of a weak candidate: an edge if 8-connected to an edge
__device__ inline bool hyst_visit(const PixBuf& S, int hgt, int wid, int idx) {
  const uint8_t b = S.work[idx];
  if ((b & (B_CAND | B_EDGE)) != B_CAND) return false;
  const int r = idx / wid, c = idx - r * wid;
  bool hit = false;
  for (int dy = -1; dy <= 1 && !hit; ++dy) {
    const int rr = r + dy;
    if ((unsigned)rr >= (unsigned)hgt) continue;
    for (int dx = -1; dx <= 1; ++dx) {
      const int cc = c + dx;
      if ((unsigned)cc >= (unsigned)wid) continue;
      if (S.work[rr * wid + cc] & B_EDGE) {
        hit = true;
        break;
      }
    }
  }
  if (hit) S.work[idx] = b | B_EDGE;
  return hit;
}

// Canny hysteresis: candidates 8-connected to a strong pixel become edges
// (sweeps over every pixel to a fixed point; the result is the reachability
// closure, whatever order the sweeps visit in).
__device__ inline void hysteresis(const PixBuf& S, int hgt, int wid) {
  const int np = hgt * wid;
  for (;;) {
    int changed = 0;
    for (int idx = threadIdx.x; idx < np; idx += blockDim.x)
      if (hyst_visit(S, hgt, wid, idx)) changed = 1;
    if (!__syncthreads_or(changed)) break;
  }
}

// pass C for one pixel: dilated colour bits | edge bit (bit 3)
__device__ inline uint8_t pass_c_pixel(const PixBuf& S, const LineDev& L, int hgt, int wid, int r,
                                       int c) {
  uint8_t bits = 0;
  const int R = L.dil_r;
  for (int dy = -R; dy <= R; ++dy) {
    const int rr = r + dy;
    if ((unsigned)rr >= (unsigned)hgt) continue;
    for (int dx = -R; dx <= R; ++dx) {
      const int cc = c + dx;
      if ((unsigned)cc >= (unsigned)wid) continue;
      if (!((L.dil_mask >> ((dy + 3) * 7 + (dx + 3))) & 1ull)) continue;
      bits |= S.work[rr * wid + cc] & 7;
    }
  }
  if (S.work[r * wid + c] & B_EDGE) bits |= 8;
  return bits;
}

struct View {  // f32 camera frame of one env
  float cx, cz, dirx, dirz, rx, rz;
};

// the thread index, opaque to the compiler: with several decisions a
// workgroup (DTSIM_RENDER_SEQ) it would otherwise hoist tid-derived addresses
// out of the decision loop and spill them
__device__ __forceinline__ int opaque_tid() {
  int t = (int)threadIdx.x;
#if DTSIM_RENDER_SEQ
  asm volatile("" : "+v"(t));
#endif
  return t;
}

// DTSIM_RENDER_SEQ: a dt_render2/3 workgroup renders its env's decisions one
// after the other (one prologue and one dispatch for the group) instead of
// one workgroup an (env, decision)
#ifndef DTSIM_RENDER_SEQ
#define DTSIM_RENDER_SEQ 0
#endif
struct RenderArgs {
  const double* x;
  const double* z;
  const double* angle;
  const int8_t* kind;
  int32_t width, height;
  float inv_ts;
  double cam_fwd;
  const float4* marks;
  int32_t n_yellow, n_white;
  float* gray;
  uint8_t* index;   // [n, slots, 120, 160] palette bytes (dt_render_io.index), or null
  int32_t slots, slot;
  const uint8_t* fresh;
  uint8_t* masks;
  uint8_t* rgb;
  uint16_t* spill;   // per env kSpillHalves: entries and list of slots >= list_cap
  int32_t list_cap;  // listed words kept in LDS (<= kListCap)
  LineDev line;
  int32_t n;
  uint32_t* sched;   // dispatch order state (kSchedHead + cost[n] + perm[2][n]), or null
  uint32_t launch;   // the handle's render launch count (host side): perm[launch & 1] is read
  // dt_render2 / dt_render3: parts = 2 or 3 consecutive decisions in the
  // same grid (block P b + p renders env perm[b] of decision p; decision 0 is
  // the fields above, 1 and 2 these: pose, ring slot, fresh flags, masks)
  int32_t parts;
  int32_t slot2, slot3;
  const double* pose2;      // [3, n]
  const double* pose3;
  const uint8_t* fresh2;
  const uint8_t* fresh3;
  uint8_t* masks2;
  uint8_t* masks3;
};

// ---- fused render kernel ----------------------------------------------------------
// One 512-thread workgroup per env, four per CU (LDS <= 40 KB, <= 64 VGPRs):
// 16 envs a CU at 4096 envs are exactly four rounds.  The frame is 4-pixel
// words of raster bytes (img; a palette index in bits 0-2 of each byte);
// Canny's work entries exist only for the LISTED words (a word whose
// 3x3-pixel neighbourhood is not one colour: every other word has Sobel 0 and
// its masks are its own colour bits).  A listed word's slot + 1 lives in the
// spare bits 3-7 of its own bytes (slot1_of), so no word -> slot map takes
// LDS.  Phases, a barrier apart:
//   0a  background of every 16-pixel span decided by its end pixels (uniform:
//       one 16-B store; otherwise zeroed and listed) + projection of the
//       marking segments, the visible ones listed
//   0b  listed spans resolved a word at a time, OR-ed in, beside the markings
//       drawn with Bresenham, OR-ed in (raster byte encoding, dtrender.h):
//       order-free, so one pass
//   1   every 16-pixel quad: neighbourhood uniformity of its 4 words;
//       non-uniform words get a slot (the list)
//   2a  listed words: SWAR 3-channel Sobel -> entry (mag | dir); the slot + 1
//       into the word's spare bits
//   2b  listed words: Canny NMS + double threshold; weak pixels listed
//   3   hysteresis over the weak list to a fixed point
//   4   outputs: grey (float4 stores into the frame ring); masks: colour bits
//       via a v_perm LUT, for quads with a listed word SWAR ellipse dilation
//       and edge bits, 16 px per lane, four 16-B stores
// Slots past list_cap (a frame with more than kListCap non-uniform words:
// never on the shipped maps) keep their entries in a per-env global spill
// area; the workgroup then runs the phases' spill instantiation.
#ifndef DTSIM_MARK_PARTS
#define DTSIM_MARK_PARTS 2  // lanes per marking segment (draw_line_part)
#endif
#ifndef DTSIM_RENDER_THREADS
#define DTSIM_RENDER_THREADS 512
#endif
constexpr int kRenderThreads = DTSIM_RENDER_THREADS;
// diagnostic builds only (tools/render_phase_valu.sh): the workgroup returns
// after phase group k (1: background spans + projection, 2: + fix-up and
// markings, 3: + uniformity, 4: + Canny), so SQ_INSTS_VALU per build splits the
// kernel's instruction count by phase; the product build never stops
#ifdef DTSIM_RENDER_STOP_AT
#define RENDER_STOP(k) \
  if ((k) == DTSIM_RENDER_STOP_AT) return
#else
#define RENDER_STOP(k)
#endif
constexpr int WPR = W / 4;          // words per row
constexpr int NW = NPIX / 4;        // words per image
constexpr int QPR = WPR / 4;        // 16-pixel quads per row
constexpr int NQ = NW / 4;          // quads per image (also the background spans)
constexpr int kListCap = 1984;      // listed words kept in LDS (loop_empty: median 631, max 1412)
constexpr int kWeakCap = 512;
constexpr int kSegRecs = 2176;     // uint2 segment records (phase 0, over the entry area)
constexpr int kSpillHalves = 5 * NW;         // global spill per env: 4 entries + 1 list word
enum { kNSpan = 0, kNSeg = 1, kNList = 2, kNQuad = 3, kNWeak = 4, kNCnt = 8 };
constexpr uint16_t WK_MAG = 0x7FF, WK_DIR_SHIFT = 11, WK_CAND = 1 << 13, WK_EDGE = 1 << 14;

struct RenderLds {
  uint32_t img[NW];   // raster bytes; from phase 2a a listed word's slot + 1 in bits 3-7
  union {
    struct {
      uint16_t ent[4 * kListCap];  // slot s: the work entries of its 4 pixels
      uint16_t list[kListCap];     // slot s -> word
    } w;
    struct {
      uint2 seg[kSegRecs];         // phase 0: visible segments (yellow up, white down)
      uint16_t qlist[NQ];          // phase 0: the non-uniform background spans
    } p;
  } u;
  uint16_t weak[kWeakCap];
  uint32_t pal_swar[PAL_N];
  float pal_gray[PAL_N];
  uint32_t bits_lo, bits_hi;  // colour bits of raster bytes 0-3 / 4-7 (one byte each)
  View view[3];         // the camera of each decision the workgroup renders
  int32_t cnt[kNCnt];
  int32_t env;          // this workgroup's env (the dispatch order's entry)
  unsigned long long t0;  // shader clock at entry (the env's recorded cost)
  int8_t kind[dt::kMaxLdsTiles];
};
static_assert(sizeof(RenderLds) <= 163840 / 4, "four render workgroups per CU");
static_assert(sizeof(((RenderLds*)0)->u.p) <= sizeof(((RenderLds*)0)->u.w), "phase-0 lists");
// segments projected in one round (loads issued at entry): 4 per lane, and
// their records must fit the record area
constexpr int kMarkFast = 4 * kRenderThreads < kSegRecs ? 4 * kRenderThreads : kSegRecs;

__device__ inline uint32_t swar_of(uint32_t bgr) {  // B | G << 10 | R << 20
  return (bgr & 255u) | (((bgr >> 8) & 255u) << 10) | (((bgr >> 16) & 255u) << 20);
}

// Sobel of one pixel from its 3x3 SWAR neighbourhood; returns max-channel m
// (first max in B, G, R order) and that channel's (dx, dy).
__device__ inline int sobel_swar(uint32_t a00, uint32_t a01, uint32_t a02, uint32_t a10,
                                 uint32_t a12, uint32_t a20, uint32_t a21, uint32_t a22,
                                 int& dx, int& dy) {
  const uint32_t px = a02 + (a12 << 1) + a22, nx = a00 + (a10 << 1) + a20;
  const uint32_t py = a20 + (a21 << 1) + a22, ny = a00 + (a01 << 1) + a02;
  int best = -1;
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const int sh = 10 * ch;
    const int gx = (int)((px >> sh) & 1023u) - (int)((nx >> sh) & 1023u);
    const int gy = (int)((py >> sh) & 1023u) - (int)((ny >> sh) & 1023u);
    const int m = (gx < 0 ? -gx : gx) + (gy < 0 ? -gy : gy);
    if (m > best) {
      best = m;
      dx = gx;
      dy = gy;
    }
  }
  return best;
}

// b (< 256) in all four bytes: one v_perm, not a 32-bit multiply
__device__ inline uint32_t splat_byte(uint32_t b) { return __builtin_amdgcn_perm(0u, b, 0u); }

// bytes of 0 / 1 -> 0 / 255: each 16-bit half (b0 + 256 b1) times 255 is
// b0 * 0xFF + b1 * 0xFF00 (no carry past the half), one full-rate packed
// 16-bit multiply (the constant in an SGPR: VOP3P takes no literal here),
// where shift + subtract took two instructions
__device__ inline uint32_t bytes01_to_ff(uint32_t m) {
  uint32_t r;
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(m), "s"(0x00FF00FFu));
  return r;
}

// A listed word's slot + 1 (0: not listed) in the spare bits 3-7 of its raster
// bytes 0..2 (13 bits: a slot < NW).  Readers of raster bytes mask kPalMask.
constexpr uint32_t kPalMask = 0x07070707u;
__device__ __forceinline__ uint32_t slot1_enc(uint32_t s1) {
  return ((s1 & 31u) << 3) | (((s1 >> 5) & 31u) << 11) | ((s1 >> 10) << 19);
}
__device__ __forceinline__ int slot1_of(uint32_t w) {
  return (int)(__builtin_amdgcn_ubfe(w, 3, 5) | (__builtin_amdgcn_ubfe(w, 11, 5) << 5) |
               (__builtin_amdgcn_ubfe(w, 19, 3) << 10));
}

// byte-lane shift of a row of words: result byte i = pixel (i + d) (0 outside)
__device__ inline uint32_t shift_bytes(uint32_t prev, uint32_t cur, uint32_t next, int d) {
  if (d == 0) return cur;
  if (d > 0) return (cur >> (8 * d)) | (next << (32 - 8 * d));
  return (cur << (-8 * d)) | (prev >> (32 + 8 * d));
}

__device__ inline int lane_prefix(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// A slot for each of up to N items per lane (every lane of the wave calls):
// the lane counts (0..N) are summed and prefix-summed bit-plane by bit-plane
// with one ballot per bit, and lane 0 reserves the wave's slots with one LDS
// atomic.
template <int N>
__device__ inline void wave_slotsN(int32_t* counter, const bool* want, int* slot) {
  constexpr int NB = N < 2 ? 1 : (N < 4 ? 2 : (N < 8 ? 3 : (N < 16 ? 4 : 5)));
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) cnt += want[k] ? 1u : 0u;
  uint64_t b[NB];
  int total = 0;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    b[i] = __ballot((cnt >> i) & 1u);
    total += __popcll(b[i]) << i;
  }
  if (total == 0) return;  // wave-uniform
  int base = 0;
  if ((threadIdx.x & 63) == 0) base = atomicAdd(counter, total);
  base = __builtin_amdgcn_readlane(base, 0);
  int next = base;
#pragma unroll
  for (int i = 0; i < NB; ++i) next += lane_prefix(b[i]) << i;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    slot[k] = next;
    next += want[k] ? 1 : 0;
  }
}

__device__ inline void wave_slots4(int32_t* counter, const bool want[4], int slot[4]) {
  wave_slotsN<4>(counter, want, slot);
}

// One item per lane: its slot (ballot prefix, one LDS atomic per wave).
__device__ inline int wave_slot1(int32_t* counter, bool want) {
  const uint64_t b = __ballot(want);
  if (b == 0) return 0;  // wave-uniform
  int base = 0;
  if ((threadIdx.x & 63) == 0) base = atomicAdd(counter, __popcll(b));
  base = __builtin_amdgcn_readlane(base, 0);
  return base + lane_prefix(b);
}

// wave_slots4 + the stores: item k of a lane goes to list[slot] (dropped past cap;
// the count still grows, so the caller sees the overflow).
__device__ inline void wave_push4(int32_t* counter, uint16_t* list, int cap, const bool want[4],
                                  const uint16_t value[4]) {
  int slot[4];
  wave_slots4(counter, want, slot);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (want[k] && slot[k] < cap) list[slot[k]] = value[k];
}

// wave_slots4 for two lists at once: one LDS atomic on a packed counter
// (list A in the low 16 bits, list B in the high 16 bits; each < 65536).
__device__ inline void wave_slots4x2(int32_t* counter, const bool wa[4], const bool wb[4],
                                     int sa[4], int sb[4]) {
  const uint32_t ca = (uint32_t)wa[0] + wa[1] + wa[2] + wa[3];
  const uint32_t cb = (uint32_t)wb[0] + wb[1] + wb[2] + wb[3];
  const uint64_t a0 = __ballot(ca & 1u), a1 = __ballot(ca & 2u), a2 = __ballot(ca & 4u);
  const uint64_t b0 = __ballot(cb & 1u), b1 = __ballot(cb & 2u), b2 = __ballot(cb & 4u);
  const uint32_t ta = __popcll(a0) + 2 * __popcll(a1) + 4 * __popcll(a2);
  const uint32_t tb = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
  if ((ta | tb) == 0u) return;  // wave-uniform
  int base = 0;
  if ((threadIdx.x & 63) == 0) base = atomicAdd(counter, (int)(ta | (tb << 16)));
  base = __builtin_amdgcn_readlane(base, 0);
  int na = (base & 0xFFFF) + lane_prefix(a0) + 2 * lane_prefix(a1) + 4 * lane_prefix(a2);
  int nb = (int)((uint32_t)base >> 16) + lane_prefix(b0) + 2 * lane_prefix(b1) +
           4 * lane_prefix(b2);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    sa[k] = na;
    na += wa[k] ? 1 : 0;
    sb[k] = nb;
    nb += wb[k] ? 1 : 0;
  }
}

using lds_u32 = __attribute__((address_space(3))) uint32_t;

// OR a raster byte into the image (ds_or_b32: order-free against the other
// markings and the background fix-up of phase 0b)
__device__ __forceinline__ void or_pixel(lds_u32* img, uint32_t ad, uint32_t col) {
  __hip_atomic_fetch_or(img + (ad >> 2), col << (8 * (ad & 3u)), __ATOMIC_RELAXED,
                        __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Pixels [xa, xb) of the Bresenham line (utils/bresenham.py:6-34) from (x0, y0)
// to (x1, y1), the same pixels in the same order as the sequential walk: its
// minor coordinate after x major steps is y(x) = floor((2 dy x + dx) / (2 dx))
// (dx > 0; 0 for a single point) and its decision variable D(x) = 2 dy (x + 1)
// - dx - 2 dx y(x), so a part starts where the walk would be (the quotient is
// exact: it is at least 1 / (2 dx) from the next integer, far above float
// rounding; checked exhaustively for dx <= 420).
__device__ inline void draw_line_part(lds_u32* img, int x0, int y0, int x1, int y1, uint32_t col,
                                      int part, int parts) {
  int dx = x1 - x0, dy = y1 - y0;
  const int xsign = dx > 0 ? 1 : -1, ysign = dy > 0 ? 1 : -1;
  dx = dx < 0 ? -dx : dx;
  dy = dy < 0 ? -dy : dy;
  int xx, xy, yx, yy;
  if (dx > dy) {
    xx = xsign; xy = 0; yx = 0; yy = ysign;
  } else {
    const int t = dx; dx = dy; dy = t;
    xx = 0; xy = ysign; yx = xsign; yy = 0;
  }
  const int n = dx + 1;
  const int xa = (n * part) / parts, xb = (n * (part + 1)) / parts;
  if (xa >= xb) return;
  const int ya = dx > 0 ? (int)floorf((float)(2 * dy * xa + dx) / (float)(2 * dx)) : 0;
  int D = 2 * dy * (xa + 1) - dx - 2 * dx * ya;
  int px = x0 + xa * xx + ya * yx, py = y0 + xa * xy + ya * yy;
  int ad = py * W + px;  // pixel (byte) address, stepped with the pixel
  const int amaj = xy * W + xx, amin = yy * W + yx;
  for (int x = xa; x < xb; ++x) {
    if ((unsigned)px < (unsigned)W && (unsigned)py < (unsigned)H) or_pixel(img, (uint32_t)ad, col);
    const bool st = D >= 0;
    px += xx + (st ? yx : 0);
    py += xy + (st ? yy : 0);
    ad += amaj + (st ? amin : 0);
    D += 2 * dy - (st ? 2 * dx : 0);
  }
}

__device__ inline int proj(float v) {  // round-to-nearest pixel, clamped far off-screen
  v = floorf(v + 0.5f);
  v = v < -100000.0f ? -100000.0f : (v > 100000.0f ? 100000.0f : v);
  return (int)v;
}

// a segment's pixel endpoints, or false when it is culled (wholly off one
// side of the frame, or degenerate: a segment is <= ~10 px at 1 cm/px)
__device__ inline bool project_seg(const View& V, float4 q, int& c0, int& r0, int& c1, int& r1) {
  const float ax = q.x - V.cx, az = q.y - V.cz, bx = q.z - V.cx, bz = q.w - V.cz;
  const float fa = ax * V.dirx + az * V.dirz, la = ax * V.rx + az * V.rz;
  const float fb = bx * V.dirx + bz * V.dirz, lb = bx * V.rx + bz * V.rz;
  c0 = proj(la * kInvRes + 79.5f);
  r0 = proj(119.5f - fa * kInvRes);
  c1 = proj(lb * kInvRes + 79.5f);
  r1 = proj(119.5f - fb * kInvRes);
  if ((c0 < 0 && c1 < 0) || (c0 >= W && c1 >= W) || (r0 < 0 && r1 < 0) || (r0 >= H && r1 >= H))
    return false;
  const int len = (c1 > c0 ? c1 - c0 : c0 - c1) + (r1 > r0 ? r1 - r0 : r0 - r1);
  return len <= 400;
}

__device__ inline uint2 seg_pack(int c0, int r0, int c1, int r1) {
  return make_uint2((uint32_t)(uint16_t)c0 | ((uint32_t)(uint16_t)r0 << 16),
                    (uint32_t)(uint16_t)c1 | ((uint32_t)(uint16_t)r1 << 16));
}

__device__ inline void seg_draw(lds_u32* img, uint2 v, uint32_t col, int part, int parts) {
  draw_line_part(img, (int)(int16_t)(v.x & 0xFFFFu), (int)(int16_t)(v.x >> 16),
                 (int)(int16_t)(v.y & 0xFFFFu), (int)(int16_t)(v.y >> 16), col, part, parts);
}

__device__ __forceinline__ uint32_t bg_color(const RenderLds& S, const RenderArgs& a, float fi,
                                             float fj) {
  if (fi >= 0.0f && fj >= 0.0f && fi < (float)a.width && fj < (float)a.height) {
    const int k = S.kind[__mul24((int)fj, a.width) + (int)fi];  // 24-bit: full-rate multiply
    return k > 0 ? PAL_ROAD : (k == 0 ? PAL_OFFROAD : PAL_FLOOR);
  }
  return PAL_FLOOR;
}

__device__ inline View view_of(double x, double z, double ang, double cam_fwd) {
  double sd, cd;
  sincos(ang, &sd, &cd);
  View v;
  v.cx = (float)(x + cam_fwd * cd);
  v.cz = (float)(z + cam_fwd * (-sd));
  v.dirx = (float)cd;
  v.dirz = -(float)sd;
  v.rx = (float)sd;
  v.rz = (float)cd;
  return v;
}

// Where the work entries and the list of a slot live: LDS below cap; with
// kSpill, the per-env global spill area at and above it.
template <bool kSpill>
struct Slots {
  RenderLds& S;
  uint16_t* gent;   // spill: entries of slot s at [4 s]
  uint16_t* glist;  // spill: word of slot s at [s]
  int cap;
  __device__ uint2 ent4(int s) const {
    if (!kSpill || s < cap) return *reinterpret_cast<const uint2*>(S.u.w.ent + 4 * s);
    return *reinterpret_cast<const uint2*>(gent + 4 * s);
  }
  __device__ void set_ent4(int s, uint2 v) const {
    if (!kSpill || s < cap)
      *reinterpret_cast<uint2*>(S.u.w.ent + 4 * s) = v;
    else
      *reinterpret_cast<uint2*>(gent + 4 * s) = v;
  }
  __device__ uint16_t ent(int s, int i) const {
    if (!kSpill || s < cap) return S.u.w.ent[4 * s + i];
    return gent[4 * s + i];
  }
  __device__ void set_ent(int s, int i, uint16_t v) const {
    if (!kSpill || s < cap)
      S.u.w.ent[4 * s + i] = v;
    else
      gent[4 * s + i] = v;
  }
  __device__ int word(int s) const {
    if (!kSpill || s < cap) return S.u.w.list[s];
    return glist[s];
  }
  // work entry of pixel (r, c): 0 outside the image and in unlisted words
  __device__ uint32_t at(int r, int c) const {
    if ((unsigned)r >= (unsigned)H || (unsigned)c >= (unsigned)W) return 0u;
    const int s = slot1_of(S.img[r * WPR + (c >> 2)]);
    return s ? (uint32_t)ent(s - 1, c & 3) : 0u;
  }
};

// phase 4 for one listed quad and a dilation radius known at compile time:
// the ellipse offsets become constant byte shifts (one v_alignbyte each) and
// the structuring-element test a scalar branch.
template <int R, bool kSpill>
__device__ __forceinline__ void quad_masks(const RenderLds& S, const Slots<kSpill>& sl,
                                           const LineDev& L, uint8_t* mb, int q) {
  const uint32_t blo = S.bits_lo, bhi = S.bits_hi;
  const uint64_t dmask = L.dil_mask;
  const int r = q / QPR, cw0 = 4 * (q - r * QPR);
  uint32_t dil[4] = {0, 0, 0, 0};
#pragma unroll
  for (int dy = -R; dy <= R; ++dy) {
    const int rr = r + dy;
    if ((unsigned)rr >= (unsigned)H) continue;
    const uint32_t* row = S.img + rr * WPR;
    const uint4 cur = *reinterpret_cast<const uint4*>(row + cw0);
    // does this row's part of the element reach past the quad's words?  (a
    // scalar test: the 3 x 3 ellipse, the default, is a cross, whose outer
    // rows need no side words)
    bool side = false;
#pragma unroll
    for (int dx = -R; dx <= R; ++dx)
      side |= dx != 0 && ((dmask >> ((dy + 3) * 7 + (dx + 3))) & 1ull) != 0ull;
    // raster bytes (slot bits masked) -> colour-bit bytes (v_perm LUT); 0
    // outside the image
    const uint32_t wv[6] = {
        side && cw0 > 0 ? __builtin_amdgcn_perm(bhi, blo, row[cw0 - 1] & kPalMask) : 0u,
        __builtin_amdgcn_perm(bhi, blo, cur.x & kPalMask),
        __builtin_amdgcn_perm(bhi, blo, cur.y & kPalMask),
        __builtin_amdgcn_perm(bhi, blo, cur.z & kPalMask),
        __builtin_amdgcn_perm(bhi, blo, cur.w & kPalMask),
        side && cw0 + 4 < WPR ? __builtin_amdgcn_perm(bhi, blo, row[cw0 + 4] & kPalMask) : 0u};
#pragma unroll
    for (int dx = -R; dx <= R; ++dx) {
      if (!((dmask >> ((dy + 3) * 7 + (dx + 3))) & 1ull)) continue;  // uniform
#pragma unroll
      for (int j = 0; j < 4; ++j) dil[j] |= shift_bytes(wv[j], wv[j + 1], wv[j + 2], dx);
    }
  }
  // edge bytes from the work entries of the quad's listed words
  const uint4 own = *reinterpret_cast<const uint4*>(S.img + r * WPR + cw0);
  const uint32_t ow[4] = {own.x, own.y, own.z, own.w};
  uint32_t edg[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int s = slot1_of(ow[j]);
    const uint2 v = s ? sl.ent4(s - 1) : make_uint2(0u, 0u);
    // the high byte of each 16-bit entry (v_perm), EDGE = its bit 6
    edg[j] = (__builtin_amdgcn_perm(v.y, v.x, 0x07050301u) >> 6) & 0x01010101u;
  }
  uint32_t o[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[0][j] = bytes01_to_ff(dil[j] & 0x01010101u);
    o[1][j] = bytes01_to_ff((dil[j] >> 1) & 0x01010101u);
    o[2][j] = bytes01_to_ff((dil[j] >> 2) & 0x01010101u);
    o[3][j] = bytes01_to_ff(edg[j]);
  }
  const int p0 = r * W + 4 * cw0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    *reinterpret_cast<uint4*>(mb + k * NPIX + p0) = make_uint4(o[k][0], o[k][1], o[k][2], o[k][3]);
}

// Phases 2a-3 (Sobel, NMS, hysteresis) on the listed words.
template <bool kSpill>
__device__ __forceinline__ void canny(const RenderArgs& a, RenderLds& S, int e,
                                                int nlist) {
  const int tid = opaque_tid();
  constexpr int T = kRenderThreads;
  const LineDev& L = a.line;
  Slots<kSpill> sl{S, a.spill + (size_t)e * kSpillHalves, a.spill + (size_t)e * kSpillHalves + 4 * NW,
                   a.list_cap};

  // phase 2a: gradients of the listed words
  for (int s = tid; s < nlist; s += T) {
    const int w = sl.word(s);
    const int r = w / WPR, cw = w - r * WPR;
    const int rows[3] = {r > 0 ? r - 1 : 0, r, r < H - 1 ? r + 1 : H - 1};
    uint32_t nb[3][6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const uint32_t* rowp = S.img + rows[k] * WPR;
      const uint32_t m = rowp[cw] & kPalMask;   // (other lanes set slot bits meanwhile)
      // BORDER_REPLICATE: the pixel left of column 0 is column 0, right of 159 is 159
      const uint32_t lb = cw > 0 ? (rowp[cw - 1] >> 24) & 7u : (m & 255u);
      const uint32_t rb = cw < WPR - 1 ? rowp[cw + 1] & 7u : (m >> 24);
      nb[k][0] = S.pal_swar[lb];
      nb[k][1] = S.pal_swar[m & 255u];
      nb[k][2] = S.pal_swar[(m >> 8) & 255u];
      nb[k][3] = S.pal_swar[(m >> 16) & 255u];
      nb[k][4] = S.pal_swar[m >> 24];
      nb[k][5] = S.pal_swar[rb];
    }
    uint32_t out[2] = {0u, 0u};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int dx, dy;
      const int m = sobel_swar(nb[0][i], nb[0][i + 1], nb[0][i + 2], nb[1][i], nb[1][i + 2],
                               nb[2][i], nb[2][i + 1], nb[2][i + 2], dx, dy);
      const uint32_t v = (uint32_t)m | ((uint32_t)nms_dir(dx, dy) << WK_DIR_SHIFT);
      out[i >> 1] |= v << (16 * (i & 1));
    }
    sl.set_ent4(s, make_uint2(out[0], out[1]));
    // the word's slot + 1 into its spare bits (this lane is the word's only
    // writer; concurrent readers mask them off)
    __hip_atomic_fetch_or((lds_u32*)S.img + w, slot1_enc((uint32_t)s + 1u), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  RENT(9);

  // phase 2b: NMS + double threshold on the listed words, branch-free: the
  // entries of the 3 x 3 word neighbourhood are read once (0 outside the
  // image and for unlisted words: their Sobel is 0), each pixel's two
  // neighbours selected by its direction class
  constexpr int U = 1;
  for (int s0 = 0; s0 < nlist; s0 += U * T) {
    if (s0 + (tid & ~63) >= nlist) break;   // wave-uniform: nothing left for this wave
    bool want[4 * U];
    uint16_t wk[4 * U];
    uint2 nv[U];
    bool upd[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int s = s0 + tid + u * T;
      const bool act = s < nlist;
      const int sc = act ? s : nlist - 1;
      const int w = sl.word(sc);
      const int r = w / WPR, cw = w - r * WPR, c0 = 4 * cw;
      const uint2 cur = sl.ent4(sc);
      uint2 nb[3][3];
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy) {
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          if (dy == 0 && dx == 0) {
            nb[1][1] = cur;
            continue;
          }
          const int rr = r + dy, cc = cw + dx;
          const bool in = (unsigned)rr < (unsigned)H && (unsigned)cc < (unsigned)WPR;
          const int slot = slot1_of(S.img[in ? rr * WPR + cc : w]);
          const uint2 v = sl.ent4(slot > 0 ? slot - 1 : 0);
          nb[dy + 1][dx + 1] = (in && slot > 0) ? v : make_uint2(0u, 0u);
        }
      }
      // magnitudes of the 3 x 6 pixel block around the word
      uint32_t M[3][6];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        M[k][0] = (nb[k][0].y >> 16) & WK_MAG;
        M[k][1] = nb[k][1].x & WK_MAG;
        M[k][2] = (nb[k][1].x >> 16) & WK_MAG;
        M[k][3] = nb[k][1].y & WK_MAG;
        M[k][4] = (nb[k][1].y >> 16) & WK_MAG;
        M[k][5] = nb[k][2].x & WK_MAG;
      }
      const uint32_t vv[4] = {cur.x & 0xFFFFu, cur.x >> 16, cur.y & 0xFFFFu, cur.y >> 16};
      uint32_t setb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = (int)(vv[i] & WK_MAG);
        const int dir = (int)(vv[i] >> WK_DIR_SHIFT) & 3;
        // dir 0: (0,-1)/(0,+1); 1: (-1,0)/(+1,0); 2: (-1,-1)/(+1,+1); 3: (-1,+1)/(+1,-1).
        // Selected with all-ones masks, not a select chain: the chain becomes an
        // indexed read of M, which the compiler then keeps in scratch memory.
        const uint32_t d0 = 0u - (uint32_t)(dir == 0), d1 = 0u - (uint32_t)(dir == 1),
                       d2 = 0u - (uint32_t)(dir == 2), d3 = 0u - (uint32_t)(dir == 3);
        const int n1 = (int)((d0 & M[1][i]) | (d1 & M[0][i + 1]) | (d2 & M[0][i]) |
                             (d3 & M[0][i + 2]));
        const int n2 = (int)((d0 & M[1][i + 2]) | (d1 & M[2][i + 1]) | (d2 & M[2][i + 2]) |
                             (d3 & M[2][i]));
        const bool keep = act && m > L.canny_lo && m > n1 && (dir >= 2 ? m > n2 : m >= n2);
        const bool strong = m > L.canny_hi;
        setb[i] = keep ? (strong ? (uint32_t)(WK_CAND | WK_EDGE) : (uint32_t)WK_CAND) : 0u;
        want[4 * u + i] = keep && !strong;
        wk[4 * u + i] = (uint16_t)(r * W + c0 + i);
      }
      // only this lane writes these four entries; neighbours read only the
      // magnitude bits, which do not change
      upd[u] = (setb[0] | setb[1] | setb[2] | setb[3]) != 0u;
      nv[u] = make_uint2(cur.x | setb[0] | (setb[1] << 16), cur.y | setb[2] | (setb[3] << 16));
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (upd[u]) sl.set_ent4(s0 + tid + u * T, nv[u]);
    int slot[4 * U];
#pragma unroll
    for (int k = 0; k < 4 * U; ++k) slot[k] = 0;
    wave_slotsN<4 * U>(&S.cnt[kNWeak], want, slot);
#pragma unroll
    for (int k = 0; k < 4 * U; ++k)
      if (want[k] && slot[k] < kWeakCap) S.weak[slot[k]] = wk[k];
  }
  __syncthreads();
  RENT(10);

  // phase 3: hysteresis (weak candidates 8-connected to an edge become edges)
  const int nweak = S.cnt[kNWeak];
  if (nweak > 0) {
    const bool overflow = nweak > kWeakCap;
    const int cnt = overflow ? 4 * nlist : nweak;
    for (;;) {
      int changed = 0;
      for (int i = tid; i < cnt; i += T) {
        int idx;
        if (overflow) {
          const int w = sl.word(i >> 2);
          const int r = w / WPR;
          idx = r * W + 4 * (w - r * WPR) + (i & 3);
        } else {
          idx = S.weak[i];
        }
        const int r = idx / W, c = idx - r * W;
        const uint32_t b = sl.at(r, c);
        if ((b & (WK_CAND | WK_EDGE)) != WK_CAND) continue;
        bool hit = false;
        for (int dy = -1; dy <= 1 && !hit; ++dy)
          for (int dx = -1; dx <= 1; ++dx)
            if (sl.at(r + dy, c + dx) & WK_EDGE) {
              hit = true;
              break;
            }
        if (hit) {
          sl.set_ent(slot1_of(S.img[r * WPR + (c >> 2)]) - 1, c & 3, (uint16_t)(b | WK_EDGE));
          changed = 1;
        }
      }
      if (!__syncthreads_or(changed)) break;
    }
  }
  RENT(11);

}

// Output phase: grey of every pixel and the four masks of every quad, no
// barrier after.  Grey: a wave's 64 quads are 256 consecutive words, stored as
// four 1-KB wave instructions (lane l of store j writes word 64 j + l of the
// wave's run).  Masks: a lane per quad, consecutive lanes consecutive 16-B
// pieces of each plane, so every line of a plane is written whole by one
// instruction: a quad without a listed word (and radius <= 1) takes its own
// colour bits, the others the dilation + edge path.
// kIdx: the frame goes out as palette bytes (a.index) instead of grey floats
// (a.gray): two instantiations, so the grey path keeps its register budget.
template <bool kSpill, bool kIdx, bool kBigR>
__device__ __forceinline__ void write_outputs(const RenderArgs& a, RenderLds& S, int e,
                                              uint8_t* mbase, int half) {
  const int tid = opaque_tid();
  constexpr int T = kRenderThreads;
  const LineDev& L = a.line;
  const Slots<kSpill> sl{S, a.spill + (size_t)e * kSpillHalves,
                         a.spill + (size_t)e * kSpillHalves + 4 * NW, a.list_cap};
  const uint8_t* fr = half == 0 ? a.fresh : (half == 1 ? a.fresh2 : a.fresh3);
  const bool fresh = fr != nullptr && fr[e] != 0;
  const int slot = half == 0 ? a.slot : (half == 1 ? a.slot2 : a.slot3);
  // a decision of a group never writes a later decision's slot (the later
  // one writes it for every env, so such a store is dead and would race),
  // and writes no frame for an env a later decision refills
  const int skip = half < a.parts - 1 ? (half == 0 ? a.slot2 : a.slot3) : -1;
  const int skip2 = half == 0 && a.parts == 3 ? a.slot3 : -1;
  const bool dead = (half < 1 && a.parts >= 2 && a.fresh2 != nullptr && a.fresh2[e] != 0) ||
                    (half < 2 && a.parts == 3 && a.fresh3 != nullptr && a.fresh3[e] != 0);
  float* gbase = !kIdx && a.gray && !dead ? a.gray + (size_t)e * a.slots * NPIX : nullptr;
  uint8_t* ibase = kIdx && !dead ? a.index + (size_t)e * a.slots * NPIX : nullptr;
  const uint32_t blo = S.bits_lo, bhi = S.bits_hi;
  const bool quick_masks = L.dil_r <= 1;
  const int lane = tid & 63;
  for (int q0 = 0; q0 < NQ; q0 += T) {
    const int wbase = 4 * (q0 + (tid - lane));
    if (gbase || ibase) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int w = wbase + 64 * j + lane;
        if (w < NW) {
          const uint32_t v = S.img[w] & kPalMask;
          if (kIdx) {   // the palette bytes themselves (4 pixels a word)
            if (fresh) {
#pragma clang loop vectorize(disable) interleave(disable)
              for (int k = 0; k < a.slots; ++k)
                if (k != skip && k != skip2) *reinterpret_cast<uint32_t*>(ibase + k * NPIX + 4 * w) = v;
            } else {
              *reinterpret_cast<uint32_t*>(ibase + slot * NPIX + 4 * w) = v;
            }
          }
          if (!kIdx) {
            float4 g;
            g.x = S.pal_gray[v & 255u];
            g.y = S.pal_gray[(v >> 8) & 255u];
            g.z = S.pal_gray[(v >> 16) & 255u];
            g.w = S.pal_gray[v >> 24];
            if (fresh) {
#pragma clang loop vectorize(disable) interleave(disable)
              for (int k = 0; k < a.slots; ++k)
                if (k != skip && k != skip2) *reinterpret_cast<float4*>(gbase + k * NPIX + 4 * w) = g;
            } else {
              *reinterpret_cast<float4*>(gbase + slot * NPIX + 4 * w) = g;
            }
          }
        }
      }
    }
    const int q = q0 + tid;
    if (q < NQ) {
      if (mbase) {
        const uint4 m = *reinterpret_cast<const uint4*>(S.img + 4 * q);
        // a quad without a listed word (and radius <= 1) is its own colour bits,
        // and the dilation path gives it the same bytes: so a wave takes the
        // quick path only when all its quads may, else every lane the dilation
        // path (a wave of 64 quads spans six rows and usually holds a listed
        // word: running both paths under divergence cost both)
        const bool uni = quick_masks && ((m.x | m.y | m.z | m.w) & ~kPalMask) == 0u;
        if (__ballot(!uni) == 0) {   // wave-uniform
          const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
          uint32_t o[3][4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t cb = __builtin_amdgcn_perm(bhi, blo, mw[j]);
            o[0][j] = bytes01_to_ff(cb & 0x01010101u);
            o[1][j] = bytes01_to_ff((cb >> 1) & 0x01010101u);
            o[2][j] = bytes01_to_ff((cb >> 2) & 0x01010101u);
          }
#pragma unroll
          for (int k = 0; k < 3; ++k)
            *reinterpret_cast<uint4*>(mbase + k * NPIX + 16 * q) =
                make_uint4(o[k][0], o[k][1], o[k][2], o[k][3]);
          *reinterpret_cast<uint4*>(mbase + 3 * NPIX + 16 * q) = make_uint4(0u, 0u, 0u, 0u);
        } else {
          // radius 2-3 (kernel sizes 5, 7) in their own kernel: their
          // unrolled ellipses held 450 SGPR spills in every instantiation
          if (kBigR) {
            if (L.dil_r == 2) quad_masks<2>(S, sl, L, mbase, q);
            else quad_masks<3>(S, sl, L, mbase, q);
          } else {
            if (L.dil_r == 0) quad_masks<0>(S, sl, L, mbase, q);
            else quad_masks<1>(S, sl, L, mbase, q);
          }
        }
      }
      if (a.rgb) {
        const uint4 m = *reinterpret_cast<const uint4*>(S.img + 4 * q);
        uint8_t* o = a.rgb + ((size_t)e * NPIX + 16 * q) * 3;
        const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
        for (int i = 0; i < 16; ++i) {
          const uint32_t p = kPalette[(mw[i >> 2] >> (8 * (i & 3))) & 7u];
          o[3 * i + 0] = (p >> 16) & 255;
          o[3 * i + 1] = (p >> 8) & 255;
          o[3 * i + 2] = p & 255;
        }
      }
    }
  }
}

// ---- dispatch order: longest measured renders first ---------------------------------
// A launch's time is its drain: once the last workgroups are dispatched (~80 %
// of the launch) the CUs finish between 0.77 and 1.0 of it,
// because a frame with many listed words or markings takes up to twice the
// median.  Greedy dispatch in blockIdx order is list scheduling; with the
// longest jobs first (LPT) the tail holds only short ones.  Each workgroup
// records its env's cost (shader cycles from entry to exit); block n - 512
// (dispatched about 512 workgroups before the end, so it finishes in the
// drain, when its CU idles anyway; launches of <= 512 workgroups run at once
// and keep the identity order)
// counting-sorts the envs by recorded cost, descending, into the order the
// NEXT launch dispatches in (poses move 3 sim steps a decision, so a frame's
// cost predicts the next one's; respawned envs' guesses are stale, and costs
// not yet recorded are the last launch's).  Block b renders env
// perm[launch & 1][b], launch the handle's host-side launch count passed as an
// argument.  One state a handle, so its launches run one after another: a
// launch captured into a HIP graph (replayed later, perhaps beside eager ones)
// uses the identity order and does not touch the state, and an eager launch
// on another stream than the last one's waits for that launch (an event,
// dt_render_launch).  No device-wide
// counter: an agent-scope atomic on one address from every workgroup
// serialises at memory across the 8 XCDs (a start ticket taken that way cost
// 0.15 ms a 4096-env launch).  The order is only a schedule:
// every env is rendered exactly once a launch and its outputs do not depend
// on it.  State (per handle, dt_render_init): kSchedHead unused words, then
// cost[n] (u32 cycles), perm[2][n] (i32, both the identity at first).
constexpr int kSchedHead = 16;
constexpr int kSchedTail = 512;      // workgroups started after the builder
constexpr int kSchedBuckets = 1024;  // cost >> 8 (256-cycle buckets), clamped
constexpr int kSchedMaxN = (int)(sizeof(((RenderLds*)0)->u) / sizeof(uint16_t));

__device__ __forceinline__ uint32_t* sched_cost(const RenderArgs& a) { return a.sched + kSchedHead; }
__device__ __forceinline__ int32_t* sched_perm(const RenderArgs& a, uint32_t launch) {
  return (int32_t*)(a.sched + kSchedHead) + (size_t)a.n * (1 + (launch & 1u));
}

// the whole workgroup: envs sorted by recorded cost, descending, into the
// next launch's order (a permutation whatever the costs read: each is read
// once, its bucket kept in LDS for both passes)
__device__ __forceinline__ void sched_build(const RenderArgs& a, RenderLds& S, uint32_t launch) {
  const int tid = threadIdx.x;
  constexpr int T = kRenderThreads;
  const int n = a.n;
  uint32_t* hist = S.img;                       // [kSchedBuckets] (the image is written out)
  uint16_t* key = (uint16_t*)&S.u;              // [n] bucket of env i
  const uint32_t* cost = sched_cost(a);
#ifdef DTSIM_SCHED_IDENTITY   // diagnostic: the mechanism without the reordering
  for (int i = tid; i < n; i += T) sched_perm(a, launch + 1u)[i] = i;
  return;
#endif
  for (int i = tid; i < kSchedBuckets; i += T) hist[i] = 0u;
  __syncthreads();
  for (int i = tid; i < n; i += T) {
    const uint32_t c = __hip_atomic_load(const_cast<uint32_t*>(cost + i), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t b = (kSchedBuckets - 1) - min(c >> 8, (uint32_t)(kSchedBuckets - 1));
    key[i] = (uint16_t)b;                        // ascending bucket = descending cost
    atomicAdd(&hist[b], 1u);
  }
  __syncthreads();
  if (tid < 64) {   // exclusive scan, one wave: 16 buckets a lane
    constexpr int P = kSchedBuckets / 64;
    uint32_t v[P], sum = 0;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      v[k] = hist[P * tid + k];
      sum += v[k];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t t = __shfl_up(inc, d, 64);
      if (tid >= d) inc += t;
    }
    uint32_t base = inc - sum;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      hist[P * tid + k] = base;
      base += v[k];
    }
  }
  __syncthreads();
  int32_t* next = sched_perm(a, launch + 1u);
  for (int i = tid; i < n; i += T) next[atomicAdd(&hist[key[i]], 1u)] = i;
}

// the builder's ticket
__device__ __forceinline__ uint32_t sched_builder(const RenderArgs& a) {
#if DTSIM_RENDER_SEQ
  return (uint32_t)(a.n - kSchedTail);             // one block an env: n > kSchedTail
#else
  return (uint32_t)(a.parts * a.n - kSchedTail);   // dt_render: n > kSchedTail
#endif
}

// exit of a workgroup: its cost (thread 0, no wait); the builder sorts
__device__ __forceinline__ void sched_exit(const RenderArgs& a, RenderLds& S, int e) {
  if (threadIdx.x == 0) {
    const unsigned long long dt = __builtin_amdgcn_s_memtime() - S.t0;
    __hip_atomic_store(sched_cost(a) + e, dt > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)dt,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (blockIdx.x == sched_builder(a) && a.n <= kSchedMaxN) {
    __syncthreads();                      // every wave past its outputs: LDS is free
    sched_build(a, S, a.launch);
  }
}

// One env of render_kernel.
template <bool kIdx, bool kBigR>
__device__ __forceinline__ void render_env(const RenderArgs& a, RenderLds& S, int e, int half,
                                           int vi
#ifdef DTSIM_EARLY_MARKS
                                           , const float4 (&mq)[4]
#endif
) {
  const int tid = opaque_tid();
  constexpr int T = kRenderThreads;
  const LineDev& L = a.line;
  const int nmark = a.n_yellow + a.n_white;
  const bool mfast = nmark <= kMarkFast;
#ifdef DTSIM_STAMPS
  RENSTAMP(0, __builtin_amdgcn_s_memrealtime());
  RENSTAMP(2, ren_hw_id());
  RENSTAMP(3, ren_xcc_id());
#endif
  RENT(4);
  int32_t* const C = S.cnt;
  const View V = S.view[vi];
  lds_u32* const img = (lds_u32*)S.img;
#ifndef DTSIM_EARLY_MARKS
  // the marking segments' loads (L2-resident), first used after the background
  float4 mq[4];
  if (mfast) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int sidx = tid + k * T;
      mq[k] = sidx < nmark ? a.marks[sidx] : make_float4(-1e9f, -1e9f, -1e9f, -1e9f);
    }  // (mfast: nmark <= kMarkFast <= 4 T)
  }
#endif

  // phase 0a: background.  Tiles are convex and each coordinate is a monotone
  // float function of the column, so along a row the tile index steps
  // monotonically: a 16-pixel span whose end pixels lie in one tile, or in two
  // edge-adjacent tiles of one colour, is that colour (every pixel between is
  // in one of the two): one 16-byte store.  The others are zeroed and listed;
  // 0b resolves them a word per lane.
  const auto tile_f = [&](int r, int c, float& fi, float& fj) {
    const float f = (119.5f - (float)r) * kRes;
    const float bx = V.cx + f * V.dirx, bz = V.cz + f * V.dirz;
    const float l = ((float)c - 79.5f) * kRes;
    const float wx = bx + l * V.rx, wz = bz + l * V.rz;
    fi = floorf(wx * a.inv_ts);
    fj = floorf(wz * a.inv_ts);
  };
  for (int q0 = 0; q0 < NQ; q0 += T) {
    const int q = q0 + tid;
    bool want = false;
    if (q < NQ) {
      const int r = q / QPR, c0 = 16 * (q - r * QPR);
      float fi0, fj0, fi1, fj1;
      tile_f(r, c0, fi0, fj0);
      tile_f(r, c0 + 15, fi1, fj1);
      const uint32_t col0 = bg_color(S, a, fi0, fj0);
      bool uni = fi0 == fi1 && fj0 == fj1;
      if (!uni && fabsf(fi1 - fi0) + fabsf(fj1 - fj0) == 1.0f)
        uni = bg_color(S, a, fi1, fj1) == col0;
      const uint32_t wd = uni ? splat_byte(col0) : 0u;
      *reinterpret_cast<uint4*>(S.img + 4 * q) = make_uint4(wd, wd, wd, wd);
      want = !uni;
    }
    const int slot = wave_slot1(&C[kNSpan], want);
    if (want) S.u.p.qlist[slot] = (uint16_t)q;
  }
  RENT(18);
  // ... and the markings' projection: every lane projects up to four segments
  // and lists the visible ones (pixel endpoints as int16 x 4; yellow from the
  // bottom of the record area, white from the top)
  if (mfast) {
    bool vy[4], vw[4];
    int cc0[4], rr0[4], cc1[4], rr1[4], sy[4], sw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int sidx = tid + k * T;
      const bool v = sidx < nmark && project_seg(V, mq[k], cc0[k], rr0[k], cc1[k], rr1[k]);
      vy[k] = v && sidx < a.n_yellow;
      vw[k] = v && sidx >= a.n_yellow;
    }
    wave_slots4x2(&C[kNSeg], vy, vw, sy, sw);  // yellow count | white count << 16
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (vy[k]) S.u.p.seg[sy[k]] = seg_pack(cc0[k], rr0[k], cc1[k], rr1[k]);
      if (vw[k]) S.u.p.seg[kSegRecs - 1 - sw[k]] = seg_pack(cc0[k], rr0[k], cc1[k], rr1[k]);
    }
  }
  __syncthreads();
  RENT(5);
  RENDER_STOP(1);

  // phase 0b: the listed spans' words and the marking segments (DTSIM_MARK_PARTS
  // lanes per segment), all OR-ed into the image in one pass
  constexpr int kParts = DTSIM_MARK_PARTS;
  {
    const int nspan = C[kNSpan];
    const int ny = mfast ? (C[kNSeg] & 0xFFFF) : 0, nw = mfast ? (int)((uint32_t)C[kNSeg] >> 16) : 0;
    const int nbg = 4 * nspan, items = nbg + kParts * (ny + nw);
    for (int i = tid; i < items; i += T) {
      if (i < nbg) {
        const int q = S.u.p.qlist[i >> 2];
        const int r = q / QPR, c = 16 * (q - r * QPR) + 4 * (i & 3);
        float fi[4], fj[4];
        tile_f(r, c, fi[0], fj[0]);
        tile_f(r, c + 3, fi[3], fj[3]);
        const uint32_t col0 = bg_color(S, a, fi[0], fj[0]);
        uint32_t wd;
        if (fi[0] == fi[3] && fj[0] == fj[3]) {
          wd = splat_byte(col0);
        } else {
          tile_f(r, c + 1, fi[1], fj[1]);
          tile_f(r, c + 2, fi[2], fj[2]);
          wd = col0;
#pragma unroll
          for (int k = 1; k < 4; ++k) wd |= bg_color(S, a, fi[k], fj[k]) << (8 * k);
        }
        __hip_atomic_fetch_or(img + 4 * q + (i & 3), wd, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        const int j = i - nbg, sidx = j / kParts;
        const bool yel = sidx < ny;
        seg_draw(img, S.u.p.seg[yel ? sidx : kSegRecs - 1 - (sidx - ny)], yel ? PAL_YELLOW : PAL_WHITE,
                 j - sidx * kParts, kParts);
      }
    }
  }
  if (!mfast) {
    // more segments than one projection round: batches of 4 T per colour, each
    // listed, then drawn (order-free, so batches need no order)
    int listed = 0;
#pragma unroll 1
    for (int colr = 0; colr < 2; ++colr) {
      const float4* seg = colr == 0 ? a.marks : a.marks + a.n_yellow;
      const int nseg = colr == 0 ? a.n_yellow : a.n_white;
      const uint32_t col = colr == 0 ? PAL_YELLOW : PAL_WHITE;
#pragma unroll 1
      for (int b0 = 0; b0 < nseg; b0 += kMarkFast) {
        bool vis[4];
        int cc0[4], rr0[4], cc1[4], rr1[4], slot[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int sidx = b0 + tid + k * T;
          const bool in = tid + k * T < kMarkFast && sidx < nseg;
          const float4 q = in ? seg[sidx] : make_float4(-1e9f, -1e9f, -1e9f, -1e9f);
          vis[k] = in && project_seg(V, q, cc0[k], rr0[k], cc1[k], rr1[k]);
        }
        wave_slots4(&C[kNSeg], vis, slot);
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (vis[k]) S.u.p.seg[slot[k] % kSegRecs] = seg_pack(cc0[k], rr0[k], cc1[k], rr1[k]);
        __syncthreads();
        const int end = C[kNSeg];
        for (int i = listed * kParts + tid; i < end * kParts; i += T)
          seg_draw(img, S.u.p.seg[(i / kParts) % kSegRecs], col, i % kParts, kParts);
        listed = end;
        __syncthreads();
      }
    }
  }
  __syncthreads();
  RENT(6);
  RENDER_STOP(2);

  // phase 1: per 16-pixel quad (4 words of a row): the 3 x 6-word neighbourhood
  // decides each word's uniformity exactly (all 18 pixels around it one
  // byte).  Non-uniform words get a slot (the list); a quad with one takes
  // the dilation path of the output phase (every quad does when the dilation
  // radius is >= 2: uniformity only covers +-1 pixel).
  uint8_t* const mb0 = half == 0 ? a.masks : (half == 1 ? a.masks2 : a.masks3);
  uint8_t* mbase = mb0 ? mb0 + (size_t)e * 4 * NPIX : nullptr;
  constexpr int kQuadPer = (NQ + T - 1) / T;  // quads per lane (3 at 512 threads)
  if (mbase) {
    bool non[4 * kQuadPer];
#pragma unroll
    for (int k = 0; k < kQuadPer; ++k) {
      // straight-line over the lane's quads (clamped, flagged): their LDS
      // reads and tests interleave
      const int qq = tid + k * T;
      const bool act = qq < NQ;
      const int q = act ? qq : NQ - 1;
      const int r = q / QPR, cw0 = 4 * (q - r * QPR);
      uint32_t m[3][4], lw[3], rw[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        int rr = r - 1 + i;
        rr = rr < 0 ? 0 : (rr > H - 1 ? H - 1 : rr);
        const uint32_t* row = S.img + rr * WPR;
        const uint4 v = *reinterpret_cast<const uint4*>(row + cw0);
        m[i][0] = v.x;
        m[i][1] = v.y;
        m[i][2] = v.z;
        m[i][3] = v.w;
        // side words at the image edge clamp to the quad's own edge word:
        // BORDER_REPLICATE repeats the edge pixel, already compared
        lw[i] = row[cw0 > 0 ? cw0 - 1 : cw0];
        rw[i] = row[cw0 + 4 < WPR ? cw0 + 4 : cw0 + 3];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t rep = splat_byte(m[1][j] & 255u);
        // per row the word's 6-pixel span as two byte-shifted words (v_alignbyte):
        // pixels 4j-1 .. 4j+2 and 4j+1 .. 4j+4, each compared with the splat
        uint32_t diff = 0u;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const uint32_t lft = j > 0 ? m[i][j - 1] : lw[i], rgt = j < 3 ? m[i][j + 1] : rw[i];
          diff |= (__builtin_amdgcn_alignbyte(m[i][j], lft, 3u) ^ rep) |
                  (__builtin_amdgcn_alignbyte(rgt, m[i][j], 1u) ^ rep);
        }
        non[4 * k + j] = act && diff != 0u;
      }
    }
    int slot[4 * kQuadPer];
#pragma unroll
    for (int k = 0; k < 4 * kQuadPer; ++k) slot[k] = 0;
    wave_slotsN<4 * kQuadPer>(&C[kNList], non, slot);
    uint16_t* gl = a.spill + (size_t)e * kSpillHalves + 4 * NW;
#pragma unroll
    for (int k = 0; k < kQuadPer; ++k) {
      const int q = tid + k * T;
      if (q < NQ) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int w = 4 * q + j;
          const int sj = slot[4 * k + j];
          if (non[4 * k + j]) {
            if (sj < a.list_cap)
              S.u.w.list[sj] = (uint16_t)w;
            else
              gl[sj] = (uint16_t)w;
          }
        }
      }
    }
  }
  __syncthreads();
  RENT(8);
  RENDER_STOP(3);

  // phases 2-3, then the outputs
  const int nlist = C[kNList];
  if (nlist <= a.list_cap) {
    if (mbase) canny<false>(a, S, e, nlist);
    RENT(13);
    RENDER_STOP(4);
    write_outputs<false, kIdx, kBigR>(a, S, e, mbase, half);
  } else {
    if (mbase) canny<true>(a, S, e, nlist);
    RENT(13);
    RENDER_STOP(4);
    write_outputs<true, kIdx, kBigR>(a, S, e, mbase, half);
  }
#ifdef DTSIM_STAMPS
  // every wave's end (real time): [19 + w/2] for waves 1,3,5,7 -> [19..22]
  if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) & 1 && e < 4096)
    g_renstamps[e * 24 + 19 + (threadIdx.x >> 7)] = __builtin_amdgcn_s_memrealtime();
  RENSTAMP(12, (unsigned long long)C[kNList] | ((unsigned long long)C[kNWeak] << 32));
  RENSTAMP(15, (unsigned long long)C[kNSeg]);
  RENSTAMP(14, __builtin_amdgcn_s_memtime());
  RENSTAMP(1, __builtin_amdgcn_s_memrealtime());
#endif
}

// One workgroup per env, four per CU.
// waves_per_eu(8): four 512-thread workgroups per CU need <= 64 VGPRs
#ifndef DTSIM_RENDER_WPE
#define DTSIM_RENDER_WPE 8
#endif
// kIdx: palette-byte frames (a.index) instead of grey floats; kBigR: a
// dilation radius of 2-3.  Both are fixed for a launch: the host picks.
template <bool kIdx, bool kBigR>
__global__ __launch_bounds__(kRenderThreads) __attribute__((amdgpu_waves_per_eu(DTSIM_RENDER_WPE))) void
render_kernel(RenderArgs a) {
  __shared__ __attribute__((aligned(16))) RenderLds S;
  const int tid = threadIdx.x;
#ifdef DTSIM_STAMPS
  // the entry times, stored under the env this block renders (known after
  // the dispatch-order lookup below), like every other stamp
  const unsigned long long t16 = __builtin_amdgcn_s_memtime(), t17 = __builtin_amdgcn_s_memrealtime();
#endif
  const LineDev& L = a.line;
  if (tid < PAL_N) {
    const uint32_t p = kPalette[tid];
    S.pal_swar[tid] = swar_of(p);
    S.pal_gray[tid] = kPalGray[tid];
  }
  if (tid == 0) {
    S.bits_lo = L.pal_bits[0];
    S.bits_hi = L.pal_bits[1];
#pragma unroll
    for (int i = 0; i < kNCnt; ++i) S.cnt[i] = 0;
  }
  for (int i = tid; i < a.width * a.height; i += kRenderThreads) S.kind[i] = a.kind[i];
  // the camera frame, once per workgroup (wave 1; wave 0 has the palette), of
  // the env the dispatch order gives this block
  // dt_render2: blocks 2b and 2b + 1 render env perm[b] of the two decisions;
  // DTSIM_RENDER_SEQ: block b renders env perm[b] of every decision in turn
#if DTSIM_RENDER_SEQ
  const int nseq = a.parts, blk = (int)blockIdx.x, half0 = 0;
#else
  const int nseq = 1;
  const int blk = (int)blockIdx.x / a.parts;
  const int half0 = (int)blockIdx.x - blk * a.parts;
#endif
  int e = blk;
#ifdef DTSIM_EARLY_MARKS
  float4 mq[4];
  {
    const int nmark = a.n_yellow + a.n_white;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int sidx = tid + k * kRenderThreads;
      mq[k] = nmark <= kMarkFast && sidx < nmark ? a.marks[sidx]
                                                 : make_float4(-1e9f, -1e9f, -1e9f, -1e9f);
    }
  }
#endif
  if (tid >= 64 && tid < 64 + nseq) {
    const int vi = tid - 64, half = half0 + vi;
    if (a.sched) {
      const int p = sched_perm(a, a.launch)[blk];
      e = (unsigned)p < (unsigned)a.n ? p : blk;   // (always a permutation)
    }
    if (vi == 0) {
      S.env = e;
      S.t0 = __builtin_amdgcn_s_memtime();
    }
    if (half) {
      const size_t n = (size_t)a.n;
      const double* ps = half == 1 ? a.pose2 : a.pose3;
      S.view[vi] = view_of(ps[e], ps[n + e], ps[2 * n + e], a.cam_fwd);
    } else {
      S.view[vi] = view_of(a.x[e], a.z[e], a.angle[e], a.cam_fwd);
    }
  }
  __syncthreads();
  e = __builtin_amdgcn_readfirstlane(S.env);   // uniform: kept in an SGPR, as blockIdx was
#ifdef DTSIM_STAMPS
  RENSTAMP(16, t16);
  RENSTAMP(17, t17);
#endif
  for (int vi = 0; vi < nseq; ++vi) {
    if (vi > 0) {   // the previous decision's outputs are read out of LDS: reset
      __syncthreads();
      if (tid < kNCnt) S.cnt[tid] = 0;
      __syncthreads();
    }
    render_env<kIdx, kBigR>(a, S, e, half0 + vi, vi
#ifdef DTSIM_EARLY_MARKS
               , mq
#endif
    );
  }
  if (a.sched) sched_exit(a, S, e);
}

// LineDetectorHSV on caller BGR images (one workgroup per image, <= 19200 px).
__global__ __launch_bounds__(kThreads) void line_detect_kernel(LineDev L, const uint8_t* bgr,
                                                               int hgt, int wid, uint8_t* masks,
                                                               uint8_t* hsv) {
  __shared__ __attribute__((aligned(16))) uint32_t src[NPIX];
  __shared__ __attribute__((aligned(16))) Lds S;
  const int e = blockIdx.x, np = hgt * wid;
  const PixBuf B{S.mag, S.work, S.sdiv, S.hdiv};
  const uint8_t* in = bgr + (size_t)e * np * 3;
  for (int p = threadIdx.x; p < np; p += blockDim.x)
    src[p] = (uint32_t)in[3 * p] | ((uint32_t)in[3 * p + 1] << 8) | ((uint32_t)in[3 * p + 2] << 16);
  load_tables(S.sdiv, S.hdiv);
  __syncthreads();
  const auto fetch = [&](int r, int c) -> uint32_t { return src[r * wid + c]; };
  for (int p = threadIdx.x; p < np; p += blockDim.x) {
    const int r = p / wid, c = p - r * wid;
    pass_a_pixel(fetch, B, L, hgt, wid, r, c);
    if (hsv) {
      int h, s, v;
      const uint32_t q = src[p];
      bgr_to_hsv(S.sdiv, S.hdiv, q & 255, (q >> 8) & 255, (q >> 16) & 255, h, s, v);
      uint8_t* o = hsv + ((size_t)e * np + p) * 3;
      o[0] = (uint8_t)h;
      o[1] = (uint8_t)s;
      o[2] = (uint8_t)v;
    }
  }
  __syncthreads();
  pass_b(B, L, hgt, wid);
  __syncthreads();
  hysteresis(B, hgt, wid);
  uint8_t* mb = masks + (size_t)e * 4 * np;
  for (int p = threadIdx.x; p < np; p += blockDim.x) {
    const int r = p / wid, c = p - r * wid;
    const uint8_t b = pass_c_pixel(B, L, hgt, wid, r, c);
    mb[p] = b & 1 ? 255 : 0;
    mb[np + p] = b & 2 ? 255 : 0;
    mb[2 * np + p] = b & 4 ? 255 : 0;
    mb[3 * np + p] = b & 8 ? 255 : 0;
  }
}

// The same on images of any size (e.g. the 640x480 camera frame of
// duckietown_rl/env.py:12-16): one 1024-thread workgroup per image, the
// magnitude / work planes and the weak-candidate list in the caller's
// workspace (line_ws_stride bytes an image, L2-resident while the workgroup
// runs).  Hysteresis sweeps only the listed weak candidates (strong pixels
// are edges already, the rest never become edges) to the same fixed point.
constexpr int kBigThreads = 1024;
__host__ __device__ inline size_t line_ws_stride(int np) {
  return ((size_t)np * 2 + 255) / 256 * 256 + ((size_t)np + 255) / 256 * 256 + (size_t)np * 4;
}
__global__ __launch_bounds__(kBigThreads) void line_detect_big_kernel(LineDev L, const uint8_t* bgr,
                                                                      int hgt, int wid,
                                                                      uint8_t* masks, uint8_t* hsv,
                                                                      unsigned char* ws) {
  __shared__ int sdiv[256], hdiv[256];
  __shared__ int nweak;
  const int e = blockIdx.x, np = hgt * wid;
  unsigned char* base = ws + (size_t)e * line_ws_stride(np);
  int16_t* mag = reinterpret_cast<int16_t*>(base);
  uint8_t* work = base + ((size_t)np * 2 + 255) / 256 * 256;
  int32_t* weak = reinterpret_cast<int32_t*>(work + ((size_t)np + 255) / 256 * 256);
  const PixBuf B{mag, work, sdiv, hdiv};
  const uint8_t* in = bgr + (size_t)e * np * 3;
  load_tables(sdiv, hdiv);
  if (threadIdx.x == 0) nweak = 0;
  __syncthreads();
  const auto fetch = [&](int r, int c) -> uint32_t {
    const uint8_t* q = in + 3 * ((size_t)r * wid + c);
    return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16);
  };
  for (int p = threadIdx.x; p < np; p += blockDim.x) {
    const int r = p / wid, c = p - r * wid;
    pass_a_pixel(fetch, B, L, hgt, wid, r, c);
    if (hsv) {
      int h, s, v;
      const uint32_t q = fetch(r, c);
      bgr_to_hsv(sdiv, hdiv, q & 255, (q >> 8) & 255, (q >> 16) & 255, h, s, v);
      uint8_t* o = hsv + ((size_t)e * np + p) * 3;
      o[0] = (uint8_t)h;
      o[1] = (uint8_t)s;
      o[2] = (uint8_t)v;
    }
  }
  __syncthreads();
  pass_b(B, L, hgt, wid);
  __syncthreads();
  for (int p = threadIdx.x; p < np; p += blockDim.x)
    if ((work[p] & (B_CAND | B_EDGE)) == B_CAND) weak[atomicAdd(&nweak, 1)] = p;
  __syncthreads();
  const int nw = nweak;
  for (;;) {
    int changed = 0;
    for (int i = threadIdx.x; i < nw; i += blockDim.x)
      if (hyst_visit(B, hgt, wid, weak[i])) changed = 1;
    if (!__syncthreads_or(changed)) break;
  }
  uint8_t* mb = masks + (size_t)e * 4 * np;
  for (int p = threadIdx.x; p < np; p += blockDim.x) {
    const int r = p / wid, c = p - r * wid;
    const uint8_t b = pass_c_pixel(B, L, hgt, wid, r, c);
    mb[p] = b & 1 ? 255 : 0;
    mb[np + p] = b & 2 ? 255 : 0;
    mb[2 * np + p] = b & 4 ? 255 : 0;
    mb[3 * np + p] = b & 8 ? 255 : 0;
  }
}


// ---- LineDetectorHSV._HoughLine: cv2.HoughLinesP(edge, 1, pi/180, ...) ------------
// (features/line_detector1.py:63-70).  The progressive probabilistic Hough
// transform is sequential over its random point order (each visited point
// changes the accumulator and the mask the next ones see), so one wave runs
// one image: the 180 angles' votes and their max are lane-parallel (angles
// lane, lane + 64, lane + 128), the walks along a found line wave-uniform.
// The accumulator lives in LDS as int16 counts over the rho range an h x w
// image reaches (counts go negative: a kept line takes back the votes of
// every pixel it clears, visited or not, as OpenCV does), the mask as bits,
// the point list in the rest of the LDS (an image with more edge pixels than
// fit, ~16k at 120 x 160, is flagged: counts[e] = -1).  The random
// order is OpenCV's RNG(~0) multiply-with-carry; oracle/hough_oracle.c
// restates the same algorithm on the CPU.
constexpr int kHoughAngles = 180;
struct HoughTab {
  float cs[2 * kHoughAngles];   // (float)(cos(n*theta)/rho), (float)(sin(n*theta)/rho), host-built
};

// the accumulator, mask-bit and point-list layout (LDS or workspace), bytes
__host__ __device__ inline size_t hough_acc_bytes(int numangle, int nr) {
  return ((size_t)2 * numangle * nr + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t hough_mask_bytes(int np) {
  return (((size_t)np + 31) / 32 * 4 + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t hough_ws_stride(int numangle, int nr, int np) {
  return (hough_acc_bytes(numangle, nr) + hough_mask_bytes(np) + (size_t)np * 4 + 255) & ~(size_t)255;
}

// kBig: the three arrays in the caller's workspace (hough_ws_stride bytes an
// image, 32-bit point indices) instead of LDS, for images past the LDS; lane 0's
// writes to the point list and the mask are then made visible to the wave's
// other lanes with a workgroup fence (vector stores/loads, no LDS ordering).
template <typename PtT, bool kBig>
__global__ __launch_bounds__(64) void hough_kernel(const uint8_t* __restrict__ img, int h, int w,
                                                   HoughTab tab, int numangle, int numrho, int rlo,
                                                   int nr, int threshold, int min_len, int gap,
                                                   int max_lines, int max_pts,
                                                   int32_t* __restrict__ lines,
                                                   int32_t* __restrict__ counts,
                                                   int32_t* __restrict__ trace,
                                                   unsigned char* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) unsigned char hl[];
  const int e = blockIdx.x, lane = threadIdx.x, np = h * w;
  unsigned char* hb = kBig ? ws + (size_t)e * hough_ws_stride(numangle, nr, np) : hl;
  int16_t* acc = reinterpret_cast<int16_t*>(hb);                      // [numangle][nr]
  uint32_t* mask = reinterpret_cast<uint32_t*>(hb + hough_acc_bytes(numangle, nr));  // bits
  PtT* pts = reinterpret_cast<PtT*>(reinterpret_cast<unsigned char*>(mask) +
                                    hough_mask_bytes(np));                           // [max_pts]
  const auto sync_wave = [&]() {
    if (kBig) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
  };
  const uint8_t* im = img + (size_t)e * np;
  for (int i = lane; i < (numangle * nr + 1) / 2; i += 64) reinterpret_cast<uint32_t*>(acc)[i] = 0u;
  // the edge pixels in row-major order (ballot compaction keeps the order);
  // the mask as bits, one 32-bit word per half-ballot
  int count = 0;
  for (int p0 = 0; p0 < np; p0 += 64) {
    const int p = p0 + lane;
    const bool on = p < np && im[p] != 0;
    const uint64_t b = __ballot(on);
    if (lane == 0 && p0 < np) mask[p0 >> 5] = (uint32_t)b;
    if (lane == 0 && p0 + 32 < np) mask[(p0 >> 5) + 1] = (uint32_t)(b >> 32);
    const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    if (on && count + pre < max_pts) pts[count + pre] = (PtT)p;
    count += __popcll(b);
  }
  const auto on_mask = [&](int q) { return (mask[q >> 5] >> (q & 31)) & 1u; };
  float c3[3], s3[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int n = lane + 64 * t;
    c3[t] = n < numangle ? tab.cs[2 * n] : 0.0f;
    s3[t] = n < numangle ? tab.cs[2 * n + 1] : 0.0f;
  }
  // rho r lives in row r - rlo of acc (OpenCV's r + (numrho - 1) / 2 is the
  // same cell shifted: only the reachable range is kept)
  const int roff = -rlo;
  (void)numrho;
  const int shift = 16;
  uint64_t state = ~0ull;
  int nlines = 0;
  bool overflow = count > max_pts;
  int32_t* out = lines + (size_t)e * max_lines * 4;
  int it = 0;
  bool truncated = false;
  sync_wave();
  __syncthreads();
  for (; count > 0 && !overflow; count--, ++it) {
    state = (uint64_t)(uint32_t)state * 4164903690ull + (uint32_t)(state >> 32);
    const int idx = (int)((uint32_t)state % (uint32_t)count);
    const int p = pts[idx];
    const int last = pts[count - 1];
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) pts[idx] = (PtT)last;
    sync_wave();
    const int i = p / w, j = p - i * w;
    if (!on_mask(p)) continue;
    // vote: the first angle reaching the largest count
    int bv = threshold - 1, bn = 0;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int n = lane + 64 * t;
      if (n < numangle) {
        const int r = __float2int_rn((float)j * c3[t] + (float)i * s3[t]) + roff;
        int16_t* a = acc + n * nr + r;
        const int v = (int)*a + 1;
        overflow |= v > 32767;
        *a = (int16_t)v;
        if (bv < v) {   // n increases with t: strict keeps the first
          bv = v;
          bn = n;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int ov = __shfl_xor(bv, o), on = __shfl_xor(bn, o);
      const bool take = ov > bv || (ov == bv && on < bn);
      bv = take ? ov : bv;
      bn = take ? on : bn;
    }
    if (trace && e == 0 && lane == 0 && it < 4096) {
      trace[4 * it] = idx;
      trace[4 * it + 1] = p;
      trace[4 * it + 2] = bv;
      trace[4 * it + 3] = bn;
    }
    if (bv < threshold) continue;   // wave-uniform (the reduced values)
    const float a = -tab.cs[2 * bn + 1], b = tab.cs[2 * bn];
    int x0 = j, y0 = i, dx0, dy0;
    const bool xflag = fabsf(a) > fabsf(b);
    if (xflag) {
      dx0 = a > 0.0f ? 1 : -1;
      dy0 = __float2int_rn(b * (float)(1 << shift) / fabsf(a));
      y0 = (y0 << shift) + (1 << (shift - 1));
    } else {
      dy0 = b > 0.0f ? 1 : -1;
      dx0 = __float2int_rn(a * (float)(1 << shift) / fabsf(b));
      x0 = (x0 << shift) + (1 << (shift - 1));
    }
    int ex[2] = {0, 0}, ey[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      int g = 0, x = x0, y = y0;
      const int dx = k ? -dx0 : dx0, dy = k ? -dy0 : dy0;
      for (;; x += dx, y += dy) {
        const int j1 = xflag ? x : x >> shift, i1 = xflag ? y >> shift : y;
        if (j1 < 0 || j1 >= w || i1 < 0 || i1 >= h) break;
        if (on_mask(i1 * w + j1)) {
          g = 0;
          ey[k] = i1;
          ex[k] = j1;
        } else if (++g > gap) {
          break;
        }
      }
    }
    const bool good = abs(ex[1] - ex[0]) >= min_len || abs(ey[1] - ey[0]) >= min_len;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      int x = x0, y = y0;
      const int dx = k ? -dx0 : dx0, dy = k ? -dy0 : dy0;
      for (;; x += dx, y += dy) {
        const int j1 = xflag ? x : x >> shift, i1 = xflag ? y >> shift : y;
        const int q = i1 * w + j1;
        if (on_mask(q)) {
          if (good) {
#pragma unroll
            for (int t = 0; t < 3; ++t) {
              const int n = lane + 64 * t;
              if (n < numangle) {
                const int r = __float2int_rn((float)j1 * c3[t] + (float)i1 * s3[t]) + roff;
                const int v = (int)acc[n * nr + r] - 1;
                overflow |= v < -32768;
                acc[n * nr + r] = (int16_t)v;
              }
            }
          }
          sync_wave();
          if (lane == 0) mask[q >> 5] &= ~(1u << (q & 31));
          sync_wave();
        }
        if (i1 == ey[k] && j1 == ex[k]) break;
      }
    }
    if (good) {
      if (lane == 0) {
        out[4 * nlines] = ex[0];
        out[4 * nlines + 1] = ey[0];
        out[4 * nlines + 2] = ex[1];
        out[4 * nlines + 3] = ey[1];
      }
      if (++nlines >= max_lines) {
        // OpenCV has no cap: points still unvisited may hold more lines
        truncated = count > 1;
        break;
      }
    }
    overflow = __ballot(overflow) != 0;
  }
  const bool any_over = __ballot(overflow) != 0;
  if (lane == 0) counts[e] = any_over ? -1 : (truncated ? -2 : nlines);
}

}  // namespace

int dt_render_init(dt_handle* h, const dt_map* map) {
  std::vector<float4> yellow, white;
  build_marks(map, h->cfg.road_tile_size, yellow, white);
  h->n_yellow = (int)yellow.size();
  h->n_white = (int)white.size();
  std::vector<float4> all(yellow);
  all.insert(all.end(), white.begin(), white.end());
  if (!all.empty()) {
    if (hipMalloc(&h->mark_buf, all.size() * sizeof(float4)) != hipSuccess) {
      h->err = "hipMalloc(markings) failed";
      return DT_E_HIP;
    }
    if (hipMemcpy(h->mark_buf, all.data(), all.size() * sizeof(float4), hipMemcpyHostToDevice) !=
        hipSuccess) {
      h->err = "hipMemcpy(markings) failed";
      return DT_E_HIP;
    }
  }
  dt_default_line_params(&h->line_params);
  h->line = to_line_dev(h->line_params);
  // overflow store of the render's listed words (RenderLds: slots past the
  // LDS list; never touched on the shipped maps, sized for a whole frame)
  if (hipMalloc(&h->render_spill, (size_t)h->n * kSpillHalves * sizeof(uint16_t)) != hipSuccess) {
    h->err = "hipMalloc(render spill) failed";
    return DT_E_HIP;
  }
  // dispatch order state (render_kernel: longest measured renders first)
  std::vector<uint32_t> sch((size_t)kSchedHead + 3 * (size_t)h->n, 0u);
  for (int k = 0; k < 2; ++k)
    for (int i = 0; i < h->n; ++i) sch[kSchedHead + (size_t)h->n * (1 + k) + i] = (uint32_t)i;
  if (hipMalloc(&h->render_sched, sch.size() * sizeof(uint32_t)) != hipSuccess ||
      hipMemcpy(h->render_sched, sch.data(), sch.size() * sizeof(uint32_t),
                hipMemcpyHostToDevice) != hipSuccess) {
    h->err = "render dispatch order state: hipMalloc / hipMemcpy failed";
    return DT_E_HIP;
  }
  return DT_OK;
}

void dt_render_free(dt_handle* h) {
  if (h->mark_buf) (void)hipFree(h->mark_buf);
  h->mark_buf = nullptr;
  if (h->render_spill) (void)hipFree(h->render_spill);
  h->render_spill = nullptr;
  if (h->render_sched) (void)hipFree(h->render_sched);
  h->render_sched = nullptr;
  if (h->render_done) (void)hipEventDestroy(h->render_done);
  h->render_done = nullptr;
}

extern "C" {

#ifdef DTSIM_STAMPS
int dt_diag_renstamps(unsigned long long* out) {  // render_kernel per-workgroup stamps
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_renstamps), sizeof(g_renstamps)) == hipSuccess ? 0 : -1;
}
#endif

int dt_default_line_params(dt_line_params* p) {
  if (!p) return DT_E_ARG;
  const uint8_t v[8][3] = {{0, 0, 150},    {180, 60, 255},  {25, 140, 100}, {45, 255, 255},
                           {0, 140, 100},  {15, 255, 255},  {165, 140, 100}, {180, 255, 255}};
  memcpy(p->hsv_white1, v[0], 3);
  memcpy(p->hsv_white2, v[1], 3);
  memcpy(p->hsv_yellow1, v[2], 3);
  memcpy(p->hsv_yellow2, v[3], 3);
  memcpy(p->hsv_red1, v[4], 3);
  memcpy(p->hsv_red2, v[5], 3);
  memcpy(p->hsv_red3, v[6], 3);
  memcpy(p->hsv_red4, v[7], 3);
  p->dilation_kernel_size = 3;
  p->canny_lo = 80;
  p->canny_hi = 200;
  return DT_OK;
}

int dt_set_line_params(dt_handle* h, const dt_line_params* p) {
  if (!h || !p) return DT_E_ARG;
  if (p->dilation_kernel_size < 1 || p->dilation_kernel_size > 7 ||
      (p->dilation_kernel_size & 1) == 0) {
    h->err = "dilation_kernel_size must be odd, 1..7";
    return DT_E_ARG;
  }
  h->line_params = *p;
  h->line = to_line_dev(*p);
  return DT_OK;
}

static int render_launch(dt_handle* h, const dt_render_io* io, const dt_render_io* io2,
                         const dt_render_io* io3, void* stream);

int dt_render(dt_handle* h, const dt_render_io* io, void* stream) {
  return render_launch(h, io, nullptr, nullptr, stream);
}

// a later decision of a group against the first: the same ring, its own slot
// and masks, a pose snapshot, no rgb
static bool group_ok(const dt_render_io* a, const dt_render_io* b) {
  return a->pose && b->pose && !a->rgb && !b->rgb && a->gray == b->gray && a->index == b->index &&
         a->gray_slots == b->gray_slots && a->list_cap == b->list_cap &&
         (a->masks == nullptr) == (b->masks == nullptr) && (!a->masks || a->masks != b->masks) &&
         (!(a->gray || a->index) || a->gray_slot != b->gray_slot) && b->gray_slot >= 0 &&
         b->gray_slot < (b->gray_slots < 1 ? 1 : b->gray_slots);
}

int dt_render2(dt_handle* h, const dt_render_io* io_a, const dt_render_io* io_b, void* stream) {
  if (!h || !io_a || !io_b) return DT_E_ARG;
  if (!group_ok(io_a, io_b)) {
    h->err = "dt_render2: two decisions of one ring: poses given, the same ring, "
             "different slots, separate masks, no rgb";
    return DT_E_ARG;
  }
  return render_launch(h, io_a, io_b, nullptr, stream);
}

int dt_render3(dt_handle* h, const dt_render_io* io_a, const dt_render_io* io_b,
               const dt_render_io* io_c, void* stream) {
  if (!h || !io_a || !io_b || !io_c) return DT_E_ARG;
  if (!group_ok(io_a, io_b) || !group_ok(io_a, io_c) || !group_ok(io_b, io_c)) {
    h->err = "dt_render3: three decisions of one ring: poses given, the same ring, "
             "different slots, separate masks, no rgb";
    return DT_E_ARG;
  }
  return render_launch(h, io_a, io_b, io_c, stream);
}

static int render_launch(dt_handle* h, const dt_render_io* io, const dt_render_io* io2,
                         const dt_render_io* io3, void* stream) {
  if (!h || !io) return DT_E_ARG;
  if (io->gray && io->index) {
    h->err = "dt_render: gray and index are two formats of one frame ring: give one";
    return DT_E_ARG;
  }
  if ((io->gray || io->index) &&
      (io->gray_slots < 1 || io->gray_slot < 0 || io->gray_slot >= io->gray_slots)) {
    h->err = "dt_render: gray_slot out of range";
    return DT_E_ARG;
  }
  if (io->list_cap < 0) {
    h->err = "dt_render: list_cap must be >= 0";
    return DT_E_ARG;
  }
  DevGuard dg(h->device);
  RenderArgs a{};
  const size_t n = (size_t)h->n;
  a.x = io->pose ? io->pose : h->st.x;
  a.z = io->pose ? io->pose + n : h->st.z;
  a.angle = io->pose ? io->pose + 2 * n : h->st.angle;
  a.kind = h->map.kind;
  a.width = h->map.width;
  a.height = h->map.height;
  a.inv_ts = (float)(1.0 / h->cfg.road_tile_size);
  a.cam_fwd = h->cfg.camera_forward_dist;
  a.marks = (const float4*)h->mark_buf;
  a.n_yellow = h->n_yellow;
  a.n_white = h->n_white;
  a.gray = io->gray;
  a.index = io->index;
  a.slots = io->gray_slots < 1 ? 1 : io->gray_slots;
  a.slot = io->gray_slot;
  a.fresh = io->fresh;
  a.masks = io->masks;
  a.rgb = io->rgb;
  a.line = h->line;
  a.n = h->n;
  a.spill = (uint16_t*)h->render_spill;
#ifndef DTSIM_NO_SCHED   // diagnostic builds only (A/B of the dispatch order)
  // a launch of <= kSchedTail workgroups runs all at once: no drain to order.
  // The order state is one per handle, double-buffered by the host's launch
  // count, so its launches must run one after another: a launch being
  // captured into a graph (replayed later, beside anything) keeps the
  // identity order and leaves the state alone, and an eager launch on a
  // stream other than the previous one's waits for that launch first.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing((hipStream_t)stream, &cap) != hipSuccess)
    cap = hipStreamCaptureStatusNone;
  a.sched = h->n > kSchedTail && cap == hipStreamCaptureStatusNone
                ? (uint32_t*)h->render_sched : nullptr;
  if (a.sched) {
    if (!h->render_done)
      // ordering on this device only: no system-scope fence (with one, the
      // record after every launch cost the config-3 bench 2 % of its rate)
      HIP_OR_FAIL(h, hipEventCreateWithFlags(&h->render_done,
                                             hipEventDisableTiming | hipEventDisableSystemFence));
    if (h->render_pending && (hipStream_t)stream != h->render_stream)
      HIP_OR_FAIL(h, hipStreamWaitEvent((hipStream_t)stream, h->render_done, 0));
  }
  a.launch = h->render_launches++;
#endif
  a.list_cap = io->list_cap > 0 && io->list_cap < kListCap ? io->list_cap : kListCap;
  a.parts = 1;
  if (io2) {
    a.parts = 2;
    a.slot2 = io2->gray_slot;
    a.pose2 = io2->pose;
    a.fresh2 = io2->fresh;
    a.masks2 = io2->masks;
  }
  if (io3) {
    a.parts = 3;
    a.slot3 = io3->gray_slot;
    a.pose3 = io3->pose;
    a.fresh3 = io3->fresh;
    a.masks3 = io3->masks;
  }
  const int grid = DTSIM_RENDER_SEQ ? h->n : a.parts * h->n;
  const bool big_r = a.line.dil_r >= 2;
  auto* kern = a.index ? (big_r ? render_kernel<true, true> : render_kernel<true, false>)
                       : (big_r ? render_kernel<false, true> : render_kernel<false, false>);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kRenderThreads), 0, (hipStream_t)stream, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    h->err = std::string("dt_render launch: ") + hipGetErrorString(e);
    return DT_E_HIP;
  }
  if (a.sched) {
    HIP_OR_FAIL(h, hipEventRecord(h->render_done, (hipStream_t)stream));
    h->render_stream = (hipStream_t)stream;
    h->render_pending = true;
  }
  return DT_OK;
}

int dt_palette_gray(float* gray8) {
  if (!gray8) return DT_E_ARG;
  for (int i = 0; i < PAL_N; ++i) gray8[i] = kPalGray[i];
  return DT_OK;
}

int dt_render_order(dt_handle* h, uint32_t* launches, uint32_t* cost, int32_t* order) {
  if (!h || !h->render_sched) return DT_E_ARG;
  DevGuard dg(h->device);
  HIP_OR_FAIL(h, hipDeviceSynchronize());
  const uint32_t* base = (const uint32_t*)h->render_sched;
  if (launches) *launches = h->render_launches;
  const size_t n = (size_t)h->n;
  if (cost)
    HIP_OR_FAIL(h, hipMemcpy(cost, base + kSchedHead, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (order)
    HIP_OR_FAIL(h, hipMemcpy(order, base + kSchedHead + n * (1 + (h->render_launches & 1u)),
                             n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return DT_OK;
}

int dt_copy_pose(dt_handle* h, double* pose, void* stream) {
  if (!h || !pose) return DT_E_ARG;
  DevGuard dg(h->device);
  // x, z and angle are consecutive n-double planes of the state buffer (dt_create)
  HIP_OR_FAIL(h, hipMemcpyAsync(pose, h->st.x, 3 * (size_t)h->n * sizeof(double),
                                hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return DT_OK;
}

// diagnostics (tools/hough_debug.py): image 0's visit order into this buffer
static int32_t* hough_trace = nullptr;
extern "C" int dt_diag_hough_trace(int32_t* device_buf) {
  hough_trace = device_buf;
  return 0;
}

namespace {
struct HoughGeom {
  HoughTab tab;
  int numangle, numrho, rlo, nr;
};
// cv2.HoughLinesP(edge, 1, np.pi / 180, ...): rho and theta as OpenCV's float
// parameters, the table as OpenCV builds it (double trig, rounded to float)
HoughGeom hough_geom(int height, int width) {
  HoughGeom G{};
  const float rho = 1.0f, theta = (float)(3.141592653589793 / 180.0);
  G.numangle = (int)lrint(3.141592653589793 / theta);
  for (int k = 0; k < G.numangle && k < kHoughAngles; ++k) {
    G.tab.cs[2 * k] = (float)(cos((double)k * theta) * (1.0f / rho));
    G.tab.cs[2 * k + 1] = (float)(sin((double)k * theta) * (1.0f / rho));
  }
  G.numrho = (int)lrintf((float)((width + height) * 2 + 1) / rho);
  // the rho an h x w image reaches: r(x, y) is linear, so its extremes per
  // angle are at the corners (the kernel's float math and rounding)
  int rlo = 1 << 30, rhi = -(1 << 30);
  for (int k = 0; k < G.numangle && k < kHoughAngles; ++k)
    for (int cy = 0; cy < 2; ++cy)
      for (int cx = 0; cx < 2; ++cx) {
        const float xx = (float)(cx * (width - 1)), yy = (float)(cy * (height - 1));
        const int r = (int)lrintf(xx * G.tab.cs[2 * k] + yy * G.tab.cs[2 * k + 1]);
        rlo = r < rlo ? r : rlo;
        rhi = r > rhi ? r : rhi;
      }
  G.rlo = rlo;
  G.nr = rhi - rlo + 1;
  return G;
}
bool hough_args_ok(const uint8_t* edge, int32_t n, int32_t height, int32_t width,
                   int32_t threshold, int32_t max_lines, const int32_t* lines,
                   const int32_t* counts) {
  return edge && lines && counts && n >= 0 && height > 0 && width > 0 && max_lines > 0 &&
         threshold >= 1 && (int64_t)height * width <= (int64_t)1 << 30;
}
}  // namespace

size_t dt_hough_workspace(int32_t n, int32_t height, int32_t width) {
  if (n <= 0 || height <= 0 || width <= 0) return 0;
  const HoughGeom G = hough_geom(height, width);
  return (size_t)n * hough_ws_stride(G.numangle, G.nr, height * width);
}

int dt_hough_lines_ws(const uint8_t* edge, int32_t n, int32_t height, int32_t width,
                      int32_t threshold, int32_t min_line_length, int32_t max_line_gap,
                      int32_t max_lines, int32_t* lines, int32_t* counts, void* workspace,
                      size_t workspace_bytes, void* stream) {
  if (!hough_args_ok(edge, n, height, width, threshold, max_lines, lines, counts)) return DT_E_ARG;
  if (n == 0) return DT_OK;
  const HoughGeom G = hough_geom(height, width);
  if (G.numangle > kHoughAngles) return DT_E_ARG;
  const int np = height * width;
  if (workspace) {  // any size: the arrays in the workspace
    if (workspace_bytes < (size_t)n * hough_ws_stride(G.numangle, G.nr, np)) return DT_E_ARG;
    hipLaunchKernelGGL((hough_kernel<uint32_t, true>), dim3(n), dim3(64), 0, (hipStream_t)stream,
                       edge, height, width, G.tab, G.numangle, G.numrho, G.rlo, G.nr, threshold,
                       min_line_length, max_line_gap, max_lines, np, lines, counts, hough_trace,
                       (unsigned char*)workspace);
    return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
  }
  if (np > 65536) return DT_E_ARG;   // 16-bit point indices in LDS
  const size_t fixed = hough_acc_bytes(G.numangle, G.nr) + hough_mask_bytes(np);
  if (fixed + 2 * 1024 > 160 * 1024) return DT_E_ARG;
  // the point list takes the rest of the LDS (an image with more edge
  // pixels than that is flagged with counts = -1)
  int max_pts = (int)((160 * 1024 - fixed) / 2);
  max_pts = max_pts > np ? np : max_pts;
  const size_t lds = fixed + 2 * (size_t)max_pts;
  static bool attr = false;   // dynamic LDS past 64 KB must be allowed per kernel
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&hough_kernel<uint16_t, false>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
      return DT_E_HIP;
    attr = true;
  }
  hipLaunchKernelGGL((hough_kernel<uint16_t, false>), dim3(n), dim3(64), lds, (hipStream_t)stream,
                     edge, height, width, G.tab, G.numangle, G.numrho, G.rlo, G.nr, threshold,
                     min_line_length, max_line_gap, max_lines, max_pts, lines, counts, hough_trace,
                     (unsigned char*)nullptr);
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_hough_lines(const uint8_t* edge, int32_t n, int32_t height, int32_t width,
                   int32_t threshold, int32_t min_line_length, int32_t max_line_gap,
                   int32_t max_lines, int32_t* lines, int32_t* counts, void* stream) {
  return dt_hough_lines_ws(edge, n, height, width, threshold, min_line_length, max_line_gap,
                           max_lines, lines, counts, nullptr, 0, stream);
}

static bool line_args_ok(const dt_line_params* p, const uint8_t* bgr, int32_t n, int32_t height,
                         int32_t width, const uint8_t* masks) {
  return p && bgr && masks && n > 0 && height > 0 && width > 0 &&
         (int64_t)height * width <= (int64_t)1 << 30 && p->dilation_kernel_size >= 1 &&
         p->dilation_kernel_size <= 7 && (p->dilation_kernel_size & 1) == 1;
}

size_t dt_line_detect_workspace(int32_t n, int32_t height, int32_t width) {
  if (n <= 0 || height <= 0 || width <= 0 || height * width <= NPIX) return 0;
  return (size_t)n * line_ws_stride(height * width);
}

int dt_line_detect_ws(const dt_line_params* p, const uint8_t* bgr, int32_t n, int32_t height,
                      int32_t width, uint8_t* masks, uint8_t* hsv, void* workspace,
                      size_t workspace_bytes, void* stream) {
  if (!line_args_ok(p, bgr, n, height, width, masks)) return DT_E_ARG;
  if (height * width <= NPIX) {
    hipLaunchKernelGGL(line_detect_kernel, dim3(n), dim3(kThreads), 0, (hipStream_t)stream,
                       to_line_dev(*p), bgr, height, width, masks, hsv);
  } else {
    if (!workspace || workspace_bytes < (size_t)n * line_ws_stride(height * width))
      return DT_E_ARG;
    hipLaunchKernelGGL(line_detect_big_kernel, dim3(n), dim3(kBigThreads), 0, (hipStream_t)stream,
                       to_line_dev(*p), bgr, height, width, masks, hsv,
                       (unsigned char*)workspace);
  }
  return hipGetLastError() == hipSuccess ? DT_OK : DT_E_HIP;
}

int dt_line_detect(const dt_line_params* p, const uint8_t* bgr, int32_t n, int32_t height,
                   int32_t width, uint8_t* masks, uint8_t* hsv, void* stream) {
  return dt_line_detect_ws(p, bgr, n, height, width, masks, hsv, nullptr, 0, stream);
}

}  // extern "C"
