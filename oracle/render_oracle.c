/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of the observation path (config 3).
 *
 * Restates, one image at a time in plain C:
 *   - the build-defined top-down raster (DESIGN.md "Observation path"): tile
 *     background + lane markings drawn with utils/bresenham.py:6-34 semantics;
 *   - skimage rgb2gray on img_as_float (PreliminaryTransformer,
 *     utils/reward_shaping/env_utils.py:48-51);
 *   - features/line_detector1.py LineDetectorHSV.setImage/_colorFilter
 *     (:134-141, :36-57) with OpenCV 8-bit semantics: cvtColor(BGR2HSV)
 *     (RGB2HSV_b fixed point, hsv_shift 12), inRange, dilate with
 *     getStructuringElement(MORPH_ELLIPSE), Canny(apertureSize=3, L1) with a
 *     stack-based hysteresis as OpenCV implements it.
 * cv2 is absent (and unpinned by any reference fixture): HSV is pinned against
 * colorsys to +-1, dilation against scipy.ndimage, bresenham against the
 * reference's golden vectors; Canny is pinned only by this restatement
 * ("parity unpinned" for the edge map).
 * Compiled with -ffp-contract=off -fno-builtin (see Makefile).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dtsim.h"

#define OH DT_OBS_H
#define OW DT_OBS_W
#define ONP (OH * OW)

static const uint8_t PAL[6][3] = {  /* RGB */
    {0, 0, 0}, {72, 132, 52}, {56, 56, 60}, {255, 230, 0}, {250, 250, 250}, {220, 30, 30}};

/* ---- markings ---------------------------------------------------------------- */
typedef struct { float x0, z0, x1, z1; } seg_t;

static void curve_sample(const double* cp, double t, double* x, double* z, double* rx,
                         double* rz) {
  double u = 1.0 - t;
  double c0 = u * u * u, c1 = 3.0 * t * (u * u), c2 = 3.0 * (t * t) * u, c3 = t * t * t;
  double px = c0 * cp[0], pz = c0 * cp[2];
  px = px + c1 * cp[3]; pz = pz + c1 * cp[5];
  px = px + c2 * cp[6]; pz = pz + c2 * cp[8];
  px = px + c3 * cp[9]; pz = pz + c3 * cp[11];
  double a0 = 3.0 * (u * u), a1 = 6.0 * u * t, a2 = 3.0 * (t * t);
  double dx = a0 * (cp[3] - cp[0]), dz = a0 * (cp[5] - cp[2]);
  dx = dx + a1 * (cp[6] - cp[3]); dz = dz + a1 * (cp[8] - cp[5]);
  dx = dx + a2 * (cp[9] - cp[6]); dz = dz + a2 * (cp[11] - cp[8]);
  double n = sqrt(dx * dx + dz * dz);
  *x = px; *z = pz;
  *rx = (0.0 - dz) / n;
  *rz = dx / n;
}

/* returns number of segments written; yellow first (ny), then white */
static int build_marks(const dt_map* m, double ts, seg_t* out, int cap, int* ny) {
  int n = 0;
  /* pass 0: yellow, pass 1: white (same tile order) */
  for (int pass = 0; pass < 2; ++pass) {
    for (int t = 0; t < m->width * m->height; ++t) {
      if (m->kind[t] <= 0 || m->kind[t] > DT_TILE_CURVE_RIGHT) continue;  /* no marks on intersections */
      for (int c = 0; c < 2; ++c) {
        if (pass == 0 && c != 0) continue;
        const double* cp = m->curves + (size_t)(m->curve_start[t] + c) * 12;
        double X[9], Z[9], RX[9], RZ[9];
        for (int k = 0; k <= 8; ++k) curve_sample(cp, (double)k / 8, &X[k], &Z[k], &RX[k], &RZ[k]);
        int wdt = pass == 0 ? 4 : 7;  /* parallel polylines 0.7 px apart */
        double base = pass == 0 ? -0.20 * ts : 0.26 * ts;
        for (int w = 0; w < wdt; ++w) {
          double o = base + (2 * w - (wdt - 1)) * 0.0035;
          for (int k = 0; k < 8; ++k) {
            if (pass == 0 && (k & 1)) continue;
            if (n < cap) {
              out[n].x0 = (float)(X[k] + o * RX[k]);
              out[n].z0 = (float)(Z[k] + o * RZ[k]);
              out[n].x1 = (float)(X[k + 1] + o * RX[k + 1]);
              out[n].z1 = (float)(Z[k + 1] + o * RZ[k + 1]);
            }
            ++n;
          }
        }
      }
    }
    if (pass == 0) *ny = n;
  }
  return n;
}

/* utils/bresenham.py:6-34 */
static void bresenham_draw(uint8_t* img, int x0, int y0, int x1, int y1, uint8_t col) {
  int dx = x1 - x0, dy = y1 - y0;
  int xsign = dx > 0 ? 1 : -1, ysign = dy > 0 ? 1 : -1;
  dx = abs(dx); dy = abs(dy);
  int xx, xy, yx, yy;
  if (dx > dy) { xx = xsign; xy = 0; yx = 0; yy = ysign; }
  else { int t = dx; dx = dy; dy = t; xx = 0; xy = ysign; yx = xsign; yy = 0; }
  int D = 2 * dy - dx, y = 0;
  for (int x = 0; x < dx + 1; ++x) {
    int px = x0 + x * xx + y * yx, py = y0 + x * xy + y * yy;
    if (px >= 0 && px < OW && py >= 0 && py < OH) img[py * OW + px] = col;
    if (D >= 0) { y += 1; D -= 2 * dx; }
    D += 2 * dy;
  }
}

int oracle_bresenham(int x0, int y0, int x1, int y1, int* out, int cap) {
  int dx = x1 - x0, dy = y1 - y0;
  int xsign = dx > 0 ? 1 : -1, ysign = dy > 0 ? 1 : -1;
  dx = abs(dx); dy = abs(dy);
  int xx, xy, yx, yy;
  if (dx > dy) { xx = xsign; xy = 0; yx = 0; yy = ysign; }
  else { int t = dx; dx = dy; dy = t; xx = 0; xy = ysign; yx = xsign; yy = 0; }
  int D = 2 * dy - dx, y = 0, n = 0;
  for (int x = 0; x < dx + 1; ++x) {
    if (n < cap) { out[2 * n] = x0 + x * xx + y * yx; out[2 * n + 1] = y0 + x * xy + y * yy; }
    ++n;
    if (D >= 0) { y += 1; D -= 2 * dx; }
    D += 2 * dy;
  }
  return n;
}

static int to_px(float v) {
  v = floorf(v + 0.5f);
  if (v < -100000.0f) v = -100000.0f;
  if (v > 100000.0f) v = 100000.0f;
  return (int)v;
}

static void raster(const dt_config* cfg, const dt_map* m, const seg_t* segs, int ny, int nseg,
                   double x, double z, double ang, uint8_t* img) {
  double c = cos(ang), s = sin(ang);
  float cx = (float)(x + cfg->camera_forward_dist * c);
  float cz = (float)(z + cfg->camera_forward_dist * (-s));
  float dirx = (float)c, dirz = -(float)s, rx = (float)s, rz = (float)c;
  float inv_ts = (float)(1.0 / cfg->road_tile_size);
  for (int r = 0; r < OH; ++r)
    for (int col = 0; col < OW; ++col) {
      float f = (119.5f - (float)r) * 0.01f;
      float l = ((float)col - 79.5f) * 0.01f;
      float wx = (cx + f * dirx) + l * rx;
      float wz = (cz + f * dirz) + l * rz;
      float fi = floorf(wx * inv_ts), fj = floorf(wz * inv_ts);
      uint8_t v = 0;
      if (fi >= 0.0f && fj >= 0.0f && fi < (float)m->width && fj < (float)m->height) {
        int k = m->kind[(int)fj * m->width + (int)fi];
        v = k > 0 ? 2 : (k == 0 ? 1 : 0);
      }
      img[r * OW + col] = v;
    }
  for (int i = 0; i < nseg; ++i) {
    const seg_t* q = &segs[i];
    float ax = q->x0 - cx, az = q->z0 - cz, bx = q->x1 - cx, bz = q->z1 - cz;
    float fa = ax * dirx + az * dirz, la = ax * rx + az * rz;
    float fb = bx * dirx + bz * dirz, lb = bx * rx + bz * rz;
    int c0 = to_px(la * 100.0f + 79.5f), r0 = to_px(119.5f - fa * 100.0f);
    int c1 = to_px(lb * 100.0f + 79.5f), r1 = to_px(119.5f - fb * 100.0f);
    if ((c0 < 0 && c1 < 0) || (c0 >= OW && c1 >= OW) || (r0 < 0 && r1 < 0) ||
        (r0 >= OH && r1 >= OH))
      continue;
    if (abs(c1 - c0) + abs(r1 - r0) > 400) continue;
    bresenham_draw(img, c0, r0, c1, r1, i < ny ? 3 : 4);
  }
}

/* ---- OpenCV pieces ------------------------------------------------------------- */
static int g_sdiv[256], g_hdiv[256], g_tables = 0;

static void tables(void) {
  if (g_tables) return;
  for (int i = 1; i < 256; ++i) {
    g_sdiv[i] = (int)lrint((double)(255 << 12) / (1.0 * i));
    g_hdiv[i] = (int)lrint((double)(180 << 12) / (6.0 * i));
  }
  g_sdiv[0] = g_hdiv[0] = 0;
  g_tables = 1;
}

/* cvtColor(COLOR_BGR2HSV), 8-bit */
static void hsv_of(int b, int g, int r, int* H, int* S, int* V) {
  int v = b, vmin = b;
  if (g > v) v = g;
  if (r > v) v = r;
  if (g < vmin) vmin = g;
  if (r < vmin) vmin = r;
  int diff = v - vmin;
  int s = (diff * g_sdiv[v] + (1 << 11)) >> 12;
  int h;
  if (v == r) h = g - b;
  else if (v == g) h = b - r + 2 * diff;
  else h = r - g + 4 * diff;
  h = (h * g_hdiv[diff] + (1 << 11)) >> 12;
  if (h < 0) h += 180;
  *H = h; *S = s; *V = v;
}

static int in_range(const uint8_t lo[3], const uint8_t hi[3], int h, int s, int v) {
  return lo[0] <= h && h <= hi[0] && lo[1] <= s && s <= hi[1] && lo[2] <= v && v <= hi[2];
}

/* dilate a 0/1 mask with a MORPH_ELLIPSE k x k element (out-of-image ignored) */
static void dilate(const uint8_t* in, uint8_t* out, int h, int w, int k) {
  int r = k / 2;
  uint8_t el[7][7];
  memset(el, 0, sizeof el);
  if (r == 0) el[0][0] = 1;
  else {
    double inv_r2 = 1.0 / ((double)r * r);
    for (int i = 0; i < k; ++i) {
      int dy = i - r;
      int dx = (int)lrint(r * sqrt((double)(r * r - dy * dy) * inv_r2));
      int j1 = r - dx > 0 ? r - dx : 0, j2 = r + dx + 1 < k ? r + dx + 1 : k;
      for (int j = j1; j < j2; ++j) el[i][j] = 1;
    }
  }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      uint8_t v = 0;
      for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) {
          if (!el[i][j]) continue;
          int yy = y + i - r, xx = x + j - r;
          if (yy < 0 || yy >= h || xx < 0 || xx >= w) continue;
          v |= in[yy * w + xx];
        }
      out[y * w + x] = v;
    }
}

/* Canny(bgr, lo, hi, apertureSize=3, L2gradient=false) on a 3-channel image */
static void canny(const uint8_t* bgr, int h, int w, double lo_t, double hi_t, uint8_t* edges) {
  if (lo_t > hi_t) { double t = lo_t; lo_t = hi_t; hi_t = t; }
  int low = (int)floor(lo_t), high = (int)floor(hi_t);
  int np = h * w;
  int* dxs = malloc(sizeof(int) * np);
  int* dys = malloc(sizeof(int) * np);
  int* mag = malloc(sizeof(int) * np);
  uint8_t* map = malloc(np);
  int* stack = malloc(sizeof(int) * np);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int best = -1, bdx = 0, bdy = 0;
      for (int ch = 0; ch < 3; ++ch) {
#define PIX(yy, xx) ((int)bgr[(((yy) < 0 ? 0 : ((yy) >= h ? h - 1 : (yy))) * w + \
                             ((xx) < 0 ? 0 : ((xx) >= w ? w - 1 : (xx)))) * 3 + ch])
        int gx = (PIX(y - 1, x + 1) + 2 * PIX(y, x + 1) + PIX(y + 1, x + 1)) -
                 (PIX(y - 1, x - 1) + 2 * PIX(y, x - 1) + PIX(y + 1, x - 1));
        int gy = (PIX(y + 1, x - 1) + 2 * PIX(y + 1, x) + PIX(y + 1, x + 1)) -
                 (PIX(y - 1, x - 1) + 2 * PIX(y - 1, x) + PIX(y - 1, x + 1));
#undef PIX
        int m = abs(gx) + abs(gy);
        if (m > best) { best = m; bdx = gx; bdy = gy; }
      }
      dxs[y * w + x] = bdx; dys[y * w + x] = bdy; mag[y * w + x] = best;
    }
#define MAG(yy, xx) (((yy) < 0 || (yy) >= h || (xx) < 0 || (xx) >= w) ? 0 : mag[(yy) * w + (xx)])
  int top = 0;
  /* map: 0 = candidate, 1 = not an edge, 2 = edge (OpenCV's encoding) */
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int j = y * w + x, m = mag[j];
      map[j] = 1;
      if (m <= low) continue;
      int xs = dxs[j], ys = dys[j];
      int ax = abs(xs), ay = abs(ys) << 15;
      int tg22x = ax * 13573;
      int ok;
      if (ay < tg22x) ok = m > MAG(y, x - 1) && m >= MAG(y, x + 1);
      else {
        int tg67x = tg22x + (ax << 16);
        if (ay > tg67x) ok = m > MAG(y - 1, x) && m >= MAG(y + 1, x);
        else {
          int s = (xs ^ ys) < 0 ? -1 : 1;
          ok = m > MAG(y - 1, x - s) && m > MAG(y + 1, x + s);
        }
      }
      if (!ok) continue;
      if (m > high) { map[j] = 2; stack[top++] = j; }
      else map[j] = 0;
    }
#undef MAG
  while (top > 0) {
    int j = stack[--top];
    int y = j / w, x = j % w;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        int yy = y + dy, xx = x + dx;
        if (yy < 0 || yy >= h || xx < 0 || xx >= w) continue;
        int k = yy * w + xx;
        if (map[k] == 0) { map[k] = 2; stack[top++] = k; }
      }
  }
  for (int j = 0; j < np; ++j) edges[j] = map[j] == 2 ? 255 : 0;
  free(dxs); free(dys); free(mag); free(map); free(stack);
}

/* LineDetectorHSV: masks [4, h, w] {white, yellow, red, edges}; hsv optional */
static void line_detect_one(const dt_line_params* p, const uint8_t* bgr, int h, int w,
                            uint8_t* masks, uint8_t* hsv) {
  tables();
  int np = h * w;
  uint8_t* bw = malloc(3 * np);
  for (int j = 0; j < np; ++j) {
    int H, S, V;
    hsv_of(bgr[3 * j], bgr[3 * j + 1], bgr[3 * j + 2], &H, &S, &V);
    if (hsv) { hsv[3 * j] = (uint8_t)H; hsv[3 * j + 1] = (uint8_t)S; hsv[3 * j + 2] = (uint8_t)V; }
    bw[j] = (uint8_t)in_range(p->hsv_white1, p->hsv_white2, H, S, V);
    bw[np + j] = (uint8_t)in_range(p->hsv_yellow1, p->hsv_yellow2, H, S, V);
    bw[2 * np + j] = (uint8_t)(in_range(p->hsv_red1, p->hsv_red2, H, S, V) ||
                               in_range(p->hsv_red3, p->hsv_red4, H, S, V));
  }
  uint8_t* tmp = malloc(np);
  for (int c = 0; c < 3; ++c) {
    dilate(bw + c * np, tmp, h, w, p->dilation_kernel_size);
    for (int j = 0; j < np; ++j) masks[c * np + j] = tmp[j] ? 255 : 0;
  }
  canny(bgr, h, w, p->canny_lo, p->canny_hi, masks + 3 * np);
  free(tmp);
  free(bw);
}

int oracle_line_detect(const dt_line_params* p, const uint8_t* bgr, int n, int h, int w,
                       uint8_t* masks, uint8_t* hsv) {
  for (int e = 0; e < n; ++e)
    line_detect_one(p, bgr + (size_t)e * h * w * 3, h, w, masks + (size_t)e * 4 * h * w,
                    hsv ? hsv + (size_t)e * h * w * 3 : 0);
  return 0;
}

int oracle_render(const dt_config* cfg, const dt_map* map, const dt_line_params* p, int n,
                  const double* x, const double* z, const double* angle, float* gray,
                  uint8_t* masks, uint8_t* rgb) {
  int ny = 0;
  int cap = 64 * 1024;
  seg_t* segs = malloc(sizeof(seg_t) * cap);
  int ns = build_marks(map, cfg->road_tile_size, segs, cap, &ny);
  if (ns > cap) { free(segs); return -1; }
  uint8_t* img = malloc(ONP);
  uint8_t* bgr = malloc(ONP * 3);
  for (int e = 0; e < n; ++e) {
    raster(cfg, map, segs, ny, ns, x[e], z[e], angle[e], img);
    for (int j = 0; j < ONP; ++j) {
      const uint8_t* c = PAL[img[j]];
      bgr[3 * j] = c[2]; bgr[3 * j + 1] = c[1]; bgr[3 * j + 2] = c[0];
      if (rgb) {
        uint8_t* o = rgb + ((size_t)e * ONP + j) * 3;
        o[0] = c[0]; o[1] = c[1]; o[2] = c[2];
      }
      if (gray) {
        double inv = 1.0 / 255.0;
        double rr = c[0] * inv, gg = c[1] * inv, bb = c[2] * inv;
        gray[(size_t)e * ONP + j] = (float)((rr * 0.2125 + gg * 0.7154) + bb * 0.0721);
      }
    }
    if (masks) line_detect_one(p, bgr, OH, OW, masks + (size_t)e * 4 * ONP, 0);
  }
  free(bgr); free(img); free(segs);
  return 0;
}

int oracle_marks(const dt_config* cfg, const dt_map* map, float* out, int cap, int* ny) {
  seg_t* segs = malloc(sizeof(seg_t) * (cap > 0 ? cap : 1));
  int n = build_marks(map, cfg->road_tile_size, segs, cap, ny);
  memcpy(out, segs, sizeof(seg_t) * (n < cap ? n : cap));
  free(segs);
  return n;
}
