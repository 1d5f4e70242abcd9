/* TEST INFRASTRUCTURE ONLY — CPU restatement of cv2.HoughLinesP as
 * features/line_detector1.py:63-70 calls it (rho 1, theta pi/180), for the
 * dt_hough_lines kernel's parity tests.
 *
 * OpenCV is not in /root/reference nor importable here, so
 * this restates OpenCV's published progressive probabilistic Hough transform
 * (imgproc/src/hough.cpp, HoughLinesProbabilistic; Matas, Galambos & Kittler
 * 2000) from its algorithm, not from its code:
 *   - rho and theta are float parameters; numangle = round(pi / theta),
 *     numrho = round(((w + h) * 2 + 1) / rho); trig table
 *     (float)(cos(n * theta) / rho), (float)(sin(n * theta) / rho) in double
 *     then rounded (the caller passes the table: computed once on the host);
 *   - the non-zero pixels are listed in row-major order and visited in the
 *     order of OpenCV's RNG(0xFFFFFFFFFFFFFFFF) (multiply-with-carry,
 *     coefficient 4164903690): idx = next() % count, the visited point
 *     replaced by the last one;
 *   - a visited point still in the mask votes in every angle
 *     (r = round-half-even of the float x * cos + y * sin, offset
 *     (numrho - 1) / 2); the first angle reaching the largest count >=
 *     threshold gives the line;
 *   - from the point the line is walked both ways in 16.16 fixed point along
 *     its major axis until the image border or more than `gap` consecutive
 *     unset pixels; it is kept when either extent is >= min_len; the walk is
 *     repeated clearing the mask (and, for a kept line, taking the points'
 *     votes back) up to the two end points.
 * Parity against OpenCV itself is unpinned (it cannot run here). */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int round_even(float v) { return (int)lrintf(v); }

typedef struct {
  uint64_t state;
} mwc_rng;

static unsigned rng_next(mwc_rng* r) {
  r->state = (uint64_t)(unsigned)r->state * 4164903690u + (unsigned)(r->state >> 32);
  return (unsigned)r->state;
}

/* The trig table of numangle entries (cos, sin pairs), as OpenCV builds it. */
int oracle_hough_table(float rho, float theta, float* tab, int cap) {
  const int numangle = (int)lrint(3.141592653589793 / theta);
  if (numangle > cap) return -1;
  const float irho = 1.0f / rho;
  for (int n = 0; n < numangle; ++n) {
    tab[2 * n] = (float)(cos((double)n * theta) * irho);
    tab[2 * n + 1] = (float)(sin((double)n * theta) * irho);
  }
  return numangle;
}

/* One image (h x w, u8, non-zero = edge) -> up to max_lines segments
 * (x1, y1, x2, y2) in `out`; returns the count. */
int oracle_hough_lines(const uint8_t* img, int h, int w, float rho, const float* tab,
                       int numangle, int threshold, int min_len, int gap, int max_lines,
                       int* out, int* trace) {
  const int numrho = (int)lrintf((float)((w + h) * 2 + 1) / rho);
  int* acc = (int*)calloc((size_t)numangle * numrho, sizeof(int));
  uint8_t* mask = (uint8_t*)malloc((size_t)h * w);
  int* pts = (int*)malloc(sizeof(int) * 2 * (size_t)h * w);
  int count = 0, nlines = 0;
  for (int i = 0; i < h; ++i)
    for (int j = 0; j < w; ++j) {
      mask[i * w + j] = img[i * w + j] ? 1 : 0;
      if (img[i * w + j]) {
        pts[2 * count] = j;
        pts[2 * count + 1] = i;
        ++count;
      }
    }
  mwc_rng rng = {~(uint64_t)0};
  const int shift = 16;
  int it = 0;
  for (; count > 0; count--, ++it) {
    const int idx = (int)(rng_next(&rng) % (unsigned)count);
    const int j = pts[2 * idx], i = pts[2 * idx + 1];
    pts[2 * idx] = pts[2 * (count - 1)];
    pts[2 * idx + 1] = pts[2 * (count - 1) + 1];
    if (!mask[i * w + j]) continue;
    int max_val = threshold - 1, max_n = 0;
    for (int n = 0; n < numangle; ++n) {
      int r = round_even((float)j * tab[2 * n] + (float)i * tab[2 * n + 1]);
      r += (numrho - 1) / 2;
      const int val = ++acc[n * numrho + r];
      if (max_val < val) {
        max_val = val;
        max_n = n;
      }
    }
    if (trace && it < 4096) {   /* diagnostics: the visit order */
      trace[4 * it] = idx;
      trace[4 * it + 1] = i * w + j;
      trace[4 * it + 2] = max_val;
      trace[4 * it + 3] = max_n;
    }
    if (max_val < threshold) continue;
    const float a = -tab[2 * max_n + 1], b = tab[2 * max_n];
    int x0 = j, y0 = i, dx0, dy0, xflag;
    if (fabsf(a) > fabsf(b)) {
      xflag = 1;
      dx0 = a > 0 ? 1 : -1;
      dy0 = round_even(b * (float)(1 << shift) / fabsf(a));
      y0 = (y0 << shift) + (1 << (shift - 1));
    } else {
      xflag = 0;
      dy0 = b > 0 ? 1 : -1;
      dx0 = round_even(a * (float)(1 << shift) / fabsf(b));
      x0 = (x0 << shift) + (1 << (shift - 1));
    }
    int ex[2] = {0, 0}, ey[2] = {0, 0};
    for (int k = 0; k < 2; ++k) {
      int g = 0, x = x0, y = y0, dx = dx0, dy = dy0;
      if (k > 0) dx = -dx, dy = -dy;
      for (;; x += dx, y += dy) {
        int i1, j1;
        if (xflag) {
          j1 = x;
          i1 = y >> shift;
        } else {
          j1 = x >> shift;
          i1 = y;
        }
        if (j1 < 0 || j1 >= w || i1 < 0 || i1 >= h) break;
        if (mask[i1 * w + j1]) {
          g = 0;
          ey[k] = i1;
          ex[k] = j1;
        } else if (++g > gap) {
          break;
        }
      }
    }
    const int good = abs(ex[1] - ex[0]) >= min_len || abs(ey[1] - ey[0]) >= min_len;
    for (int k = 0; k < 2; ++k) {
      int x = x0, y = y0, dx = dx0, dy = dy0;
      if (k > 0) dx = -dx, dy = -dy;
      for (;; x += dx, y += dy) {
        int i1, j1;
        if (xflag) {
          j1 = x;
          i1 = y >> shift;
        } else {
          j1 = x >> shift;
          i1 = y;
        }
        uint8_t* m = mask + i1 * w + j1;
        if (*m) {
          if (good)
            for (int n = 0; n < numangle; ++n) {
              int r = round_even((float)j1 * tab[2 * n] + (float)i1 * tab[2 * n + 1]);
              r += (numrho - 1) / 2;
              acc[n * numrho + r]--;
            }
          *m = 0;
        }
        if (i1 == ey[k] && j1 == ex[k]) break;
      }
    }
    if (good) {
      out[4 * nlines] = ex[0];
      out[4 * nlines + 1] = ey[0];
      out[4 * nlines + 2] = ex[1];
      out[4 * nlines + 3] = ey[1];
      if (++nlines >= max_lines) break;
    }
  }
  free(acc);
  free(mask);
  free(pts);
  return nlines;
}
