// Shared device-side definitions of libdtsim: handle layout, map staging, the
// Philox stream, and the float64 Simulator step math (one wavefront lane per
// environment).  gfx950 only.
//
// Float semantics: every kernel TU is compiled with -ffp-contract=off (and the
// pragma below) so no multiply-add is fused.  The reference (numpy float64)
// never fuses, and the spec demands <=1e-5 on pose/reward and bit-exact
// tile/done; keeping numpy's rounding sequence makes the GPU agree with the
// CPU oracle to the last ulp except where libm and ocml transcendentals differ.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dtsim.h"

namespace dt {

constexpr int kWave = 64;
constexpr int kMaxLdsTiles = 256;             // tiles staged in LDS (kinds: render too)
constexpr size_t kMaxMapLdsBytes = 48 * 1024;  // map image in LDS (dt_create enforces)

constexpr uint32_t kTagTile = 0x54494C45u;    // 'TILE'
constexpr uint32_t kTagSpawnA = 0x53504E41u;  // 'SPNA'
constexpr uint32_t kTagSpawnB = 0x53504E42u;  // 'SPNB'

constexpr uint32_t kErrSpawn = 1u;   // a reset exhausted max_spawn_attempts
constexpr uint32_t kErrNonFinite = 2u;

// SoA environment state, all device pointers (one allocation).
struct State {
  double* x;
  double* z;
  double* angle;
  uint64_t* seed;
  uint32_t* step_count;
  uint32_t* env_step;
  uint32_t* episode;
  uint32_t* err;  // one word, OR of kErr*
  unsigned long long* stats;  // [4] sim steps, decisions, resets, episodes done
  // spawn-ahead: slot k % kSlots of env e holds the reset pose
  // of spawn key k (x, z, angle, lane dist, angle_rad, sin and cos of the
  // angle) when the low word of
  // pre_key[k % kSlots][e] is k (bit 31: the spawn failed); its high word is
  // the launch tick the slot was written in.  want[e] - 1 = the env's episode
  // counter as its last launch left it; the window [want - 1, want - 1 +
  // kSlots) is kept filled.  tick[e] counts the step launches over env e.
  double* pre;                // [kSlots][kSlotRec][n]
  uint64_t* pre_key;          // [kSlots][n]
  uint32_t* want;             // [n]
  uint32_t* tick;             // [n]
};
constexpr uint32_t kKeyFailed = 0x80000000u;
constexpr uint32_t kKeyNone = 0xFFFFFFFFu;
constexpr int kSlots = 8;    // power of two
constexpr int kSlotRec = 7;  // x, z, angle, lane dist, angle_rad, sin, cos

// One atomic per wave: the lane sum of v (0 <= v <= vmax, vmax wave-uniform)
// from one ballot per bit, lane 0 adds.
__device__ inline void wave_count(unsigned long long* p, unsigned v, unsigned vmax) {
  unsigned long long s = 0;
  for (int b = 0; (vmax >> b) != 0u; ++b)
    s += (unsigned long long)__popcll(__ballot((v >> b) & 1u)) << b;
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(p, s);
}


// A lane curve as the step math reads it.  Every map curve lies in the ground
// plane (y = 0 for each control point and heading; dt_create checks), so the
// y terms of bezier_point / bezier_tangent / get_lane_pos2 are exact zeros and
// drop out without changing a result: a term b*b = +0 added to a*a >= +0, and
// 0 * (finite) = +-0 added to a nonzero value, leave the sums unchanged (a
// zero's sign never reaches a comparison or a nonzero output).  Per curve:
//   [0..7]   P0x P0z P1x P1z P2x P2z P3x P3z     control points
//   [8..13]  (P1-P0), (P2-P1), (P3-P2) in x, z  tangent differences (host-made,
//            the same subtractions bezier_tangent does)
//   [14..15] heading x, z                        (P3-P0) / np.linalg.norm quirk
constexpr int kCurveRec = 16;

// Map image in device memory; staged into LDS by each block.
struct MapDev {
  int32_t width, height, n_tiles, n_drivable, n_curves, n_obj, n_spawn_obj;
  const double* curves;     // [C,kCurveRec] ground-plane curve records (CurveRec)
  const double* obj;        // [n_obj, DT_OBJ_STRIDE] collidable static objects
  const double* spawn_obj;  // [n_spawn_obj, 4] x, y, z, spawn radius
  const uint16_t* curve_start;  // [T+1]
  const int8_t* kind;       // [T]
  const int16_t* drivable;  // [n_drivable] tile index of the k-th drivable tile (load order)
};

// LDS view of the map.
struct MapLds {
  const double* curves;
  const double* obj;
  const double* spawn_obj;
  const uint16_t* curve_start;
  const int8_t* kind;
  const int16_t* drivable;
  // per tile, packed for one LDS read: first curve (bits 0-15), curve count
  // (16-23), kind > 0 (bit 24)
  const uint32_t* tinfo;
  int32_t width, height, n_drivable, n_obj, n_spawn_obj;
};

__host__ __device__ inline size_t map_lds_bytes(int n_tiles, int n_drivable, int n_curves,
                                                int n_obj = 0, int n_spawn_obj = 0) {
  size_t b = (size_t)n_curves * kCurveRec * sizeof(double);
  b += ((size_t)n_obj * DT_OBJ_STRIDE + (size_t)n_spawn_obj * 4) * sizeof(double);
  b += ((size_t)(n_tiles + 1) * 2 + 15) & ~(size_t)15;
  b += ((size_t)n_tiles + 15) & ~(size_t)15;
  b += ((size_t)n_drivable * 2 + 15) & ~(size_t)15;
  b += (size_t)n_tiles * 4;
  return b;
}

// Cooperative copy of the map into LDS; every thread of the block calls it.
__device__ inline MapLds stage_map(const MapDev& m, unsigned char* lds) {
  double* cv = reinterpret_cast<double*>(lds);
  double* ob = cv + (size_t)m.n_curves * kCurveRec;
  double* so = ob + (size_t)m.n_obj * DT_OBJ_STRIDE;
  uint16_t* cs = reinterpret_cast<uint16_t*>(so + (size_t)m.n_spawn_obj * 4);
  int8_t* kd = reinterpret_cast<int8_t*>(cs) + (((size_t)(m.n_tiles + 1) * 2 + 15) & ~(size_t)15);
  int16_t* dv = reinterpret_cast<int16_t*>(kd + (((size_t)m.n_tiles + 15) & ~(size_t)15));
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < m.n_curves * kCurveRec; i += nt) cv[i] = m.curves[i];
  for (int i = tid; i < m.n_obj * DT_OBJ_STRIDE; i += nt) ob[i] = m.obj[i];
  for (int i = tid; i < m.n_spawn_obj * 4; i += nt) so[i] = m.spawn_obj[i];
  for (int i = tid; i <= m.n_tiles; i += nt) cs[i] = m.curve_start[i];
  for (int i = tid; i < m.n_tiles; i += nt) kd[i] = m.kind[i];
  for (int i = tid; i < m.n_drivable; i += nt) dv[i] = m.drivable[i];
  uint32_t* ti = reinterpret_cast<uint32_t*>(
      reinterpret_cast<unsigned char*>(dv) + (((size_t)m.n_drivable * 2 + 15) & ~(size_t)15));
  for (int i = tid; i < m.n_tiles; i += nt) {
    const uint32_t k0 = m.curve_start[i], k1 = m.curve_start[i + 1];
    ti[i] = k0 | ((k1 - k0) << 16) | (m.kind[i] > 0 ? (1u << 24) : 0u);
  }
  __syncthreads();
  MapLds r;
  r.curves = cv;
  r.obj = ob;
  r.spawn_obj = so;
  r.curve_start = cs;
  r.kind = kd;
  r.drivable = dv;
  r.tinfo = ti;
  r.width = m.width;
  r.height = m.height;
  r.n_drivable = m.n_drivable;
  r.n_obj = m.n_obj;
  r.n_spawn_obj = m.n_spawn_obj;
  return r;
}

// ---- Philox4x32-10 ----------------------------------------------------------
struct U4 {
  uint32_t a, b, c, d;
};

__device__ inline U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                            uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return U4{c0, c1, c2, c3};
}

__device__ inline double u01(uint32_t a, uint32_t b) {
  return (double)(((((uint64_t)a) << 32) | b) >> 11) * (1.0 / 9007199254740992.0);
}

// ---- wave helpers -------------------------------------------------------------
__device__ inline uint32_t bcast(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ inline double bcast(double v, int lane) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = bcast((uint32_t)u, lane), hi = bcast((uint32_t)(u >> 32), lane);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ inline uint64_t bcast(uint64_t v, int lane) {
  const uint32_t lo = bcast((uint32_t)v, lane), hi = bcast((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// ---- Simulator math -----------------------------------
struct Geo {  // constants hoisted per launch
  double ts, inv_ts, wheel_dist, dt, off, robot_width, front, rad2deg, two_pi, accept_deg,
      reset_safety;
  double robot_speed;
  double robot_length, agent_safety_rad;   // objects: agent box and safety circle
};

// floor(v / ts) exactly as numpy computes it (correctly rounded division, then
// floor), via the reciprocal: RN(v * inv_ts) is within 2 ulp of RN(v / ts), so
// their floors can only differ when the quotient is within a few ulp of an
// integer — only then is the real division done.
// The rare exact paths are out-of-line calls: as inline code the compiler
// speculates them (the division and sqrt are single IR operations) and every
// lane would pay for them on every call.
static __device__ __noinline__ double floor_div_exact(double v, double ts) { return floor(v / ts); }

__device__ inline double floor_div_ts(double v, const Geo& g) {
  const double q = v * g.inv_ts;
  const double f = floor(q);
  const double r = q - f;
  // |q| < 2^9 on any map: a few ulp are < 1e-12; beyond, both floors are off
  // the grid and the tile is -1 either way
  if (r < 1e-9 || r > 1.0 - 1e-9) return floor_div_exact(v, g.ts);
  return f;
}

// get_grid_coords + _get_tile: tile index or -1 (A5)
__device__ inline int tile_of(const MapLds& M, const Geo& g, double x, double z) {
  const double fi = floor_div_ts(x, g), fj = floor_div_ts(z, g);
  if (fi < 0.0 || fj < 0.0 || fi >= (double)M.width || fj >= (double)M.height) return -1;
  return (int)fj * M.width + (int)fi;
}

__device__ inline bool drivable(const MapLds& M, const Geo& g, double x, double z) {
  const int t = tile_of(M, g, x, z);
  return t >= 0 && M.kind[t] > 0;
}

// ---- branch-free fast forms -----------------------------------------------------
// The exact forms above decide their rare cases (a quotient within ulps of a
// tile edge, two distances within ulps) with a divergent branch on every call,
// and the exec-mask juggling of those branches costs more than the float64 math
// around them.  The *_fast forms take the common-case answer unconditionally
// and OR a `near` flag when the exact form could answer differently; a caller
// re-runs the exact form only for lanes with `near` set (one branch per call,
// essentially never taken), so results are identical to the exact forms.
__device__ inline double floor_div_fast(double v, const Geo& g, bool& near) {
  const double q = v * g.inv_ts;
  const double f = floor(q);
  const double r = q - f;
  near |= (r < 1e-9) | (r > 1.0 - 1e-9);
  return f;
}

__device__ inline int tile_of_fast(const MapLds& M, const Geo& g, double x, double z, bool& near) {
  const double fi = floor_div_fast(x, g, near), fj = floor_div_fast(z, g, near);
  const bool in = (fi >= 0.0) & (fj >= 0.0) & (fi < (double)M.width) & (fj < (double)M.height);
  return in ? (int)fj * M.width + (int)fi : -1;
}

__device__ inline bool drivable_fast(const MapLds& M, const Geo& g, double x, double z, bool& near) {
  const int t = tile_of_fast(M, g, x, z, near);
  return ((M.tinfo[t < 0 ? 0 : t] >> 24) & 1u) != 0u && t >= 0;
}

// ---- static objects [upstream collision.py; §8f-3] ---------------------------------
// _collision(get_agent_corners(centre, angle)): separating-axis test of the
// agent's box (ROBOT_WIDTH x ROBOT_LENGTH about the actual centre (px, pz))
// against every collidable object's box.  Axes: the agent's forward / right
// vectors (upstream: generate_norm's eigenvectors of the box, the same axes)
// and each object's two precomputed norms; boxes overlap on an axis when their
// closed projection intervals meet, and collide when they overlap on all four.
__device__ inline bool collide(const MapLds& M, const Geo& g, double px, double pz, double c,
                               double s) {
  if (M.n_obj == 0) return false;
  const double fx = c, fz = -s, rx = s, rz = c;   // get_dir_vec, get_right_vec
  const double hw = g.robot_width * 0.5, hl = g.robot_length * 0.5;
  double ax[4], az[4];   // agent_boundbox corner order
  ax[0] = (px - hw * rx) - hl * fx;
  az[0] = (pz - hw * rz) - hl * fz;
  ax[1] = (px + hw * rx) - hl * fx;
  az[1] = (pz + hw * rz) - hl * fz;
  ax[2] = (px + hw * rx) + hl * fx;
  az[2] = (pz + hw * rz) + hl * fz;
  ax[3] = (px - hw * rx) + hl * fx;
  az[3] = (pz - hw * rz) + hl * fz;
  double amin[2], amax[2];   // the agent on its own axes
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const double nx = a == 0 ? fx : rx, nz = a == 0 ? fz : rz;
    double lo = ax[0] * nx + az[0] * nz, hi = lo;
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const double p = ax[k] * nx + az[k] * nz;
      lo = p < lo ? p : lo;
      hi = p > hi ? p : hi;
    }
    amin[a] = lo;
    amax[a] = hi;
  }
  for (int o = 0; o < M.n_obj; ++o) {
    const double* ob = M.obj + (size_t)o * DT_OBJ_STRIDE;
    bool sep = false;
    // the object's corners on the agent's axes
#pragma unroll
    for (int a = 0; a < 2 && !sep; ++a) {
      const double nx = a == 0 ? fx : rx, nz = a == 0 ? fz : rz;
      double lo = ob[DT_OBJ_CORNERS] * nx + ob[DT_OBJ_CORNERS + 1] * nz, hi = lo;
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const double p = ob[DT_OBJ_CORNERS + 2 * k] * nx + ob[DT_OBJ_CORNERS + 2 * k + 1] * nz;
        lo = p < lo ? p : lo;
        hi = p > hi ? p : hi;
      }
      sep = amax[a] < lo || hi < amin[a];
    }
    // the agent's corners on the object's axes
#pragma unroll
    for (int a = 0; a < 2 && !sep; ++a) {
      const double nx = ob[DT_OBJ_NORMS + 2 * a], nz = ob[DT_OBJ_NORMS + 2 * a + 1];
      double lo = ax[0] * nx + az[0] * nz, hi = lo;
#pragma unroll
      for (int k = 1; k < 4; ++k) {
        const double p = ax[k] * nx + az[k] * nz;
        lo = p < lo ? p : lo;
        hi = p > hi ? p : hi;
      }
      sep = hi < ob[DT_OBJ_PROJ + 2 * a] || ob[DT_OBJ_PROJ + 2 * a + 1] < lo;
    }
    if (!sep) return true;
  }
  return false;
}

// proximity_penalty2 at the actual centre: the sum of the negative
// (|c_o - p| - AGENT_SAFETY_RAD - r_o) over the collidable objects
// (safety_circle_overlap; 0 when no safety circle meets the agent's)
__device__ inline double proximity_penalty(const MapLds& M, const Geo& g, double px, double pz) {
  double pen = 0.0;
  for (int o = 0; o < M.n_obj; ++o) {
    const double* ob = M.obj + (size_t)o * DT_OBJ_STRIDE;
    const double dx = ob[DT_OBJ_CENTER] - px, dy = ob[DT_OBJ_CENTER + 1] - 0.0,
                 dz = ob[DT_OBJ_CENTER + 2] - pz;
    const double d = sqrt((dx * dx + dy * dy) + dz * dz);
    const double sc = (d - g.agent_safety_rad) - ob[DT_OBJ_SAFETY_RAD];
    if (sc < 0.0) pen = pen + sc;
  }
  return pen;
}

// _inconvenient_spawn(propose_pos): within max(max_coords) * 0.5 * scale +
// MIN_SPAWN_OBJ_DIST (precomputed radius) of any object's position
__device__ inline bool inconvenient_spawn(const MapLds& M, double x, double z) {
  for (int o = 0; o < M.n_spawn_obj; ++o) {
    const double* so = M.spawn_obj + 4 * (size_t)o;
    const double dx = so[0] - x, dy = so[1] - 0.0, dz = so[2] - z;
    if (sqrt((dx * dx + dy * dy) + dz * dz) < so[3]) return true;
  }
  return false;
}

// _valid_pose with precomputed (c, s) = (cos, sin)(angle) (A6): the centre and
// both wheels and the front drivable (scaled by safety) and no collision (the
// unscaled agent box)
__device__ inline bool valid_pose(const MapLds& M, const Geo& g, double x, double z, double c,
                                  double s, double safety) {
  const double px = x + g.off * c;
  const double pz = z + g.off * (-s);
  const double kw = (safety * 0.5) * g.robot_width;
  const double kf = (safety * 0.5) * g.front;
  // all four probes evaluated (no short-circuit): they are independent, so
  // their latencies overlap instead of adding up
  const bool d0 = drivable(M, g, px, pz);
  const bool d1 = drivable(M, g, px - kw * s, pz - kw * c);
  const bool d2 = drivable(M, g, px + kw * s, pz + kw * c);
  const bool d3 = drivable(M, g, px + kf * c, pz + kf * (-s));
  const bool ok = d0 & d1 & d2 & d3;
  return ok && !collide(M, g, px, pz, c, s);
}

// valid_pose without the collision test: the four drivable probes (fast form)
__device__ inline bool probes_fast(const MapLds& M, const Geo& g, double x, double z, double c,
                                   double s, double safety, bool& near) {
  const double px = x + g.off * c;
  const double pz = z + g.off * (-s);
  const double kw = (safety * 0.5) * g.robot_width;
  const double kf = (safety * 0.5) * g.front;
  const bool d0 = drivable_fast(M, g, px, pz, near);
  const bool d1 = drivable_fast(M, g, px - kw * s, pz - kw * c, near);
  const bool d2 = drivable_fast(M, g, px + kw * s, pz + kw * c, near);
  const bool d3 = drivable_fast(M, g, px + kf * c, pz + kf * (-s), near);
  return d0 & d1 & d2 & d3;
}

// valid_pose, identical results: the fast probes, the exact form only for a
// lane whose probes came near a tile edge
__device__ inline bool valid_pose_lean(const MapLds& M, const Geo& g, double x, double z, double c,
                                       double s, double safety) {
  bool near = false;
  bool ok = probes_fast(M, g, x, z, c, s, safety, near);
  if (__builtin_expect(near, 0)) return valid_pose(M, g, x, z, c, s, safety);
  if (M.n_obj && ok) ok = !collide(M, g, x + g.off * c, z + g.off * (-s), c, s);
  return ok;
}

// bezier_point (A9) in the ground plane: coefficients are exact dyadics for
// the bisection's t values
__device__ inline void bez_xz(const double* __restrict__ cv, double t, double& ox, double& oz) {
  const double u = 1.0 - t;
  const double c0 = u * u * u, c1 = 3.0 * t * (u * u), c2 = 3.0 * (t * t) * u, c3 = t * t * t;
  double px = c0 * cv[0], pz = c0 * cv[1];
  px = px + c1 * cv[2];
  pz = pz + c1 * cv[3];
  px = px + c2 * cv[4];
  pz = pz + c2 * cv[5];
  px = px + c3 * cv[6];
  pz = pz + c3 * cv[7];
  ox = px;
  oz = pz;
}

// squared distance |B(t) - p|^2, summed as np.linalg.norm's dot (unfused, in order)
__device__ inline double dist2_to(const double* __restrict__ cv, double t, double x, double z) {
  double bx, bz;
  bez_xz(cv, t, bx, bz);
  const double a = bx - x, c = bz - z;
  return a * a + c * c;
}

// the same at an end point: B(0) = P0 and B(1) = P3 exactly (the other terms
// are +-0), so only the distance is left to compute
__device__ inline double dist2_pt(double px, double pz, double x, double z) {
  const double a = px - x, c = pz - z;
  return a * a + c * c;
}

// sqrt(a) < sqrt(b), the comparison bezier_closest makes, decided on the
// squares: sqrt is monotone, so only when a and b are within a few ulp (where
// rounding could make the roots equal) are the roots taken.
static __device__ __noinline__ bool root_less_exact(double a, double b) { return sqrt(a) < sqrt(b); }

__device__ inline bool root_less(double a, double b) {
  const double d = b - a;
  if (fabs(d) > 8.0 * 2.220446049250313e-16 * fmax(a, b)) return a < b;
  return root_less_exact(a, b);
}

// angle_rad = acos(dot_dir), negated right of the tangent (get_lane_pos2);
// lp[2] holds the side value on entry, angle_deg on exit.
__device__ inline void finish_angle(const Geo& g, double lp[4]) {
  double ang = acos(lp[1]);
  if (lp[2] < 0.0) ang = -ang;
  lp[2] = ang * g.rad2deg;
  lp[3] = ang;
}

// get_lane_pos2 (A8-A10), in three parts: the closest curve of the tile
// (nullptr when NotInLane), bezier_closest's parameter, and the lane pose.
__device__ inline const double* closest_curve(const MapLds& M, const Geo& g, double x, double z,
                                              double c, double s) {
  const int t = tile_of(M, g, x, z);
  if (t < 0 || M.kind[t] <= 0) return nullptr;
  const double dx = c, dz = -s;
  // closest curve = np.argmax(curve_headings @ dir): the first of the largest
  const int k0 = M.curve_start[t], k1 = M.curve_start[t + 1];
  int best = k0;
  double bd = 0.0;
  for (int k = k0; k < k1; ++k) {
    const double* hd = M.curves + kCurveRec * k + 14;
    const double d = hd[0] * dx + hd[1] * dz;
    if (k == k0 || d > bd) {
      bd = d;
      best = k;
    }
  }
  return M.curves + kCurveRec * best;
}

// bezier_closest, 8 levels.  One endpoint distance is carried between levels:
// the kept half's end was evaluated at the same t one level earlier, and the
// function is deterministic, so the result is bit-identical to re-evaluating.
// The midpoint is evaluated once, before the comparison: it is the new end
// whichever half is kept (one evaluation, no divergent branches).
__device__ inline double bezier_closest(const double* cv, double x, double z) {
  double tb = 0.0, tt = 1.0;
  double db = dist2_pt(cv[0], cv[1], x, z), dtp = dist2_pt(cv[6], cv[7], x, z);
#pragma unroll
  for (int n = 8; n > 0; --n) {
    const double mid = (tb + tt) * 0.5;
    const double dm = n > 1 ? dist2_to(cv, mid, x, z) : 0.0;
    const bool left = root_less(db, dtp);
    tt = left ? mid : tt;
    dtp = left ? dm : dtp;
    tb = left ? tb : mid;
    db = left ? db : dm;
  }
  return (tb + tt) * 0.5;
}

// bezier_closest with plain comparisons of the squared distances; `near` is
// set when any level compared two values close enough for the roots to round
// equal (where root_less takes the roots), and the caller then re-runs
// bezier_closest.  Same evaluation order as bezier_closest otherwise.
__device__ inline double bezier_closest_fast(const double* cv, double x, double z, bool& near) {
  double tb = 0.0, tt = 1.0;
  double db = dist2_pt(cv[0], cv[1], x, z), dtp = dist2_pt(cv[6], cv[7], x, z);
#pragma unroll
  for (int n = 8; n > 0; --n) {
    const double mid = (tb + tt) * 0.5;
    const double dm = n > 1 ? dist2_to(cv, mid, x, z) : 0.0;
    const double d = dtp - db;
    near |= !(fabs(d) > 8.0 * 2.220446049250313e-16 * fmax(db, dtp));
    const bool left = db < dtp;
    tt = left ? mid : tt;
    dtp = left ? dm : dtp;
    tb = left ? tb : mid;
    db = left ? db : dm;
  }
  return (tb + tt) * 0.5;
}

// lp = {dist, dot_dir, angle_deg, angle_rad} at the curve point tm; without
// kAngle the acos is left out and lp[2] holds the side value for finish_angle.
template <bool kAngle>
__device__ inline void lane_pose_at(const Geo& g, const double* cv, double tm, double x, double z,
                                    double c, double s, double lp[4]) {
  const double dx = c, dz = -s;
  double qx, qz;
  bez_xz(cv, tm, qx, qz);
  const double u = 1.0 - tm;
  const double a0 = 3.0 * (u * u), a1 = 6.0 * u * tm, a2 = 3.0 * (tm * tm);
  double tx = a0 * cv[8], tz = a0 * cv[9];
  tx = tx + a1 * cv[10];
  tz = tz + a1 * cv[11];
  tx = tx + a2 * cv[12];
  tz = tz + a2 * cv[13];
  const double nn = sqrt(tx * tx + tz * tz);
  tx = tx / nn;
  tz = tz / nn;
  double dot = dx * tx + dz * tz;
  dot = dot > 1.0 ? 1.0 : dot;
  dot = dot < -1.0 ? -1.0 : dot;
  const double rx = 0.0 - tz, rz = tx;
  const double px = x - qx, pz = z - qz;
  const double dist = px * rx + pz * rz;
  lp[0] = dist;
  lp[1] = dot;
  lp[2] = (dx * rx + 0.0) + dz * rz;  // side of the tangent (sign of the angle)
  if (kAngle) finish_angle(g, lp);
}

// get_lane_pos2 (A8-A10).  Returns false when NotInLane.
template <bool kAngle = true>
__device__ inline bool lane_pos(const MapLds& M, const Geo& g, double x, double z, double c,
                                double s, double lp[4]) {
  const double* cv = closest_curve(M, g, x, z, c, s);
  if (!cv) return false;
  lane_pose_at<kAngle>(g, cv, bezier_closest(cv, x, z), x, z, c, s, lp);
  return true;
}


// closest_curve with the fast tile lookup and the packed tile word: the
// headings of a tile's first two curves are read together (one LDS round
// trip), the rest (intersection tiles) in the loop
__device__ inline const double* closest_curve_fast(const MapLds& M, const Geo& g, double x,
                                                   double z, double c, double s, bool& near) {
  const int t = tile_of_fast(M, g, x, z, near);
  const uint32_t info = M.tinfo[t < 0 ? 0 : t];
  if (t < 0 || ((info >> 24) & 1u) == 0u) return nullptr;
  const double dx = c, dz = -s;
  const int k0 = (int)(info & 0xFFFFu), nc = (int)((info >> 16) & 0xFFu);
  const double* h0 = M.curves + kCurveRec * k0 + 14;
  const double* h1 = h0 + (nc > 1 ? kCurveRec : 0);
  const double hx0 = h0[0], hz0 = h0[1], hx1 = h1[0], hz1 = h1[1];
  double bd = hx0 * dx + hz0 * dz;
  int best = k0;
  const double d1 = hx1 * dx + hz1 * dz;
  if (nc > 1 && d1 > bd) {
    bd = d1;
    best = k0 + 1;
  }
  for (int k = k0 + 2; k < k0 + nc; ++k) {
    const double* hd = M.curves + kCurveRec * k + 14;
    const double d = hd[0] * dx + hd[1] * dz;
    if (d > bd) {
      bd = d;
      best = k;
    }
  }
  return M.curves + kCurveRec * best;
}

// get_lane_pos2, identical results to lane_pos: the fast forms, and lane_pos
// itself only for a lane that came near a tile edge or a distance tie
template <bool kAngle = true>
__device__ inline bool lane_pos_lean(const MapLds& M, const Geo& g, double x, double z, double c,
                                     double s, double lp[4]) {
  bool near = false;
  const double* cv = closest_curve_fast(M, g, x, z, c, s, near);
  double tm = 0.0;
  if (cv) tm = bezier_closest_fast(cv, x, z, near);
  if (__builtin_expect(near, 0)) return lane_pos<kAngle>(M, g, x, z, c, s, lp);
  if (!cv) return false;
  lane_pose_at<kAngle>(g, cv, tm, x, z, c, s, lp);
  return true;
}

// ---- quad forms: one env on the 4 lanes of a DPP quad -----------------------------
// step_fan_kernel runs every env on the four lanes of a quad (lane & 3 = q);
// the lanes hold the same state and make the same decisions, and split the
// data-parallel parts of the step math: the four drivable probes of
// _valid_pose, the sincos of the decision's rotation and angles, and three
// bisection levels per round of bezier_closest.  Values cross lanes with DPP
// quad_perm moves (no LDS, no waits).
template <int J>
__device__ __forceinline__ int qget(int v) {
  return __builtin_amdgcn_mov_dpp(v, J * 0x55, 0xF, 0xF, true);
}
template <int J>
__device__ __forceinline__ double qget(double v) {
  const long long u = __double_as_longlong(v);
  const int lo = qget<J>((int)(uint32_t)u), hi = qget<J>((int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
// AND / OR of a flag over the quad
__device__ __forceinline__ bool qall(bool b) {
  int v = b ? 1 : 0;
  v &= __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);   // [1,0,3,2]
  v &= __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);   // [2,3,0,1]
  return v != 0;
}
__device__ __forceinline__ bool qany(bool b) {
  int v = b ? 1 : 0;
  v |= __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);
  v |= __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);
  return v != 0;
}

// The drivable probes of _valid_pose at one pose, probe q on lane q: the same
// operands as valid_pose (px - kw*s == px + -(kw*s) exactly).  Returns this
// lane's probe; `near` as floor_div_fast.
__device__ inline bool probe_q(const MapLds& M, const Geo& g, int q, double x, double z, double c,
                               double s, double safety, bool& near) {
  const double px = x + g.off * c;
  const double pz = z + g.off * (-s);
  const double kw = (safety * 0.5) * g.robot_width;
  const double kf = (safety * 0.5) * g.front;
  const double ws = kw * s, wc = kw * c, fc = kf * c, fs = kf * (-s);
  const double ox = q == 1 ? -ws : (q == 2 ? ws : fc);
  const double oz = q == 1 ? -wc : (q == 2 ? wc : fs);
  const double tx = q == 0 ? px : px + ox;
  const double tz = q == 0 ? pz : pz + oz;
  return drivable_fast(M, g, tx, tz, near);
}

// _valid_pose at one pose over a quad, identical to valid_pose (kObj false:
// the caller guarantees a map without collidable objects)
template <bool kObj = true>
__device__ inline bool valid_pose_q(const MapLds& M, const Geo& g, int q, double x, double z,
                                    double c, double s, double safety) {
  bool near = false;
  bool ok = qall(probe_q(M, g, q, x, z, c, s, safety, near));
  if (__builtin_expect(qany(near), 0)) return valid_pose(M, g, x, z, c, s, safety);
  if (kObj && M.n_obj && ok) ok = !collide(M, g, x + g.off * c, z + g.off * (-s), c, s);
  return ok;
}

// bezier_closest over a quad: per round, the first level's comparison is known
// (both end distances are), so the four lanes evaluate the four points the
// next three levels can need -- the midpoint m1, the midpoint m2 of the half
// kept, and both candidate midpoints of m2's halves -- and every lane then
// walks the three levels.  The t values and distances are the ones the
// sequential bisection computes (the same dyadic midpoints, the same
// dist2_to), so the result is identical; `near` as bezier_closest_fast.
__device__ inline double bezier_closest_q(const double* cv, int q, double x, double z,
                                          bool& near) {
  constexpr double kTol = 8.0 * 2.220446049250313e-16;
  double tb = 0.0, tt = 1.0;
  double db = dist2_pt(cv[0], cv[1], x, z), dtp = dist2_pt(cv[6], cv[7], x, z);
  // lane constants (lane 0 takes m1, whose side is known per round)
  const bool q0 = q == 0;
  const double fl = (double)(((0x3010200u >> (8 * q)) & 0xFFu)) * 0.25;   // 1/2, 1/4, 3/4
#pragma unroll
  for (int n = 8; n > 0; n -= 3) {
    // level n (comparison known)
    near |= !(fabs(dtp - db) > kTol * fmax(db, dtp));
    const bool l1 = db < dtp;
    const double m1 = (tb + tt) * 0.5;
    const double lo1 = l1 ? tb : m1, hi1 = l1 ? m1 : tt;
    const double m2 = (lo1 + hi1) * 0.5;
    const double m3a = (lo1 + m2) * 0.5, m3b = (m2 + hi1) * 0.5;
    // this lane's point, lo1 + f * (hi1 - lo1) with f = {m1's side, 1/2, 1/4,
    // 3/4}: every t here is a dyadic rational with at most 10 significant
    // bits, so the product and sum are exact and equal the midpoints above
    // bit for bit (no per-lane branch)
    const double fq = q0 ? (l1 ? 1.0 : 0.0) : fl;
    const double tq = lo1 + fq * (hi1 - lo1);
    const double dq = dist2_to(cv, tq, x, z);
    const double dm1 = qget<0>(dq);
    // level n - 1
    const double e_lo = l1 ? db : dm1, e_hi = l1 ? dm1 : dtp;
    if (n - 1 == 0) {
      tb = lo1;
      tt = hi1;
      break;
    }
    const double dm2 = qget<1>(dq);
    near |= !(fabs(e_hi - e_lo) > kTol * fmax(e_lo, e_hi));
    const bool l2 = e_lo < e_hi;
    const double lo2 = l2 ? lo1 : m2, hi2 = l2 ? m2 : hi1;
    const double d_lo2 = l2 ? e_lo : dm2, d_hi2 = l2 ? dm2 : e_hi;
    if (n - 2 == 0) {
      tb = lo2;
      tt = hi2;
      break;
    }
    // level n - 2
    const double dm3a = qget<2>(dq), dm3b = qget<3>(dq);
    near |= !(fabs(d_hi2 - d_lo2) > kTol * fmax(d_lo2, d_hi2));
    const bool l3 = d_lo2 < d_hi2;
    const double m3 = l2 ? m3a : m3b, dm3 = l2 ? dm3a : dm3b;
    tb = l3 ? lo2 : m3;
    tt = l3 ? m3 : hi2;
    db = l3 ? d_lo2 : dm3;
    dtp = l3 ? dm3 : d_hi2;
  }
  return (tb + tt) * 0.5;
}

// get_lane_pos2 over a quad (every lane returns the full result), identical
// to lane_pos<true>
__device__ inline bool lane_pos_q(const MapLds& M, const Geo& g, int q, double x, double z,
                                  double c, double s, double lp[4]) {
  bool near = false;
  const double* cv = closest_curve_fast(M, g, x, z, c, s, near);
  double tm = 0.0;
  if (cv) tm = bezier_closest_q(cv, q, x, z, near);
  if (__builtin_expect(near, 0)) return lane_pos<true>(M, g, x, z, c, s, lp);
  if (!cv) return false;
  lane_pose_at<true>(g, cv, tm, x, z, c, s, lp);
  return true;
}

// One spawn proposal (A13): returns true if accepted.
__device__ inline bool spawn_try(const MapLds& M, const Geo& g, uint32_t k0, uint32_t k1,
                                 uint32_t env, uint32_t episode, uint32_t k, double fi,
                                 double fj, double& ox, double& oz, double& oa,
                                 double* lp_out = nullptr) {
  const U4 a = philox(k, episode, env, kTagSpawnA, k0, k1);
  const U4 b = philox(k, episode, env, kTagSpawnB, k0, k1);
  const double px = (fi + u01(a.a, a.b)) * g.ts;
  const double pz = (fj + u01(a.c, a.d)) * g.ts;
  const double pa = g.two_pi * u01(b.a, b.b);
  double s, c;
  sincos(pa, &s, &c);
  ox = px;
  oz = pz;
  oa = pa;
  if (inconvenient_spawn(M, px, pz)) return false;
  if (!valid_pose_lean(M, g, px, pz, c, s, g.reset_safety)) return false;
  double lp[4];
  if (!lane_pos_lean<true>(M, g, px, pz, c, s, lp)) return false;
  if (lp_out) {
    lp_out[0] = lp[0];
    lp_out[1] = lp[3];
  }
  return -g.accept_deg < lp[2] && lp[2] < g.accept_deg;
}

// Wave-cooperative Simulator.reset of ONE env (every argument wave-uniform;
// all 64 lanes must call); lp_out (optional) receives the winner's
// (dist, angle_rad).  The 64 lanes test proposals k = 64*round + lane in
// parallel; the lowest accepting lane of the first round with any acceptance
// wins, which is exactly the first accepted k of a sequential rejection loop
// over the same i.i.d. stream — so the spawn distribution is upstream's and the
// result is bit-reproducible by the sequential CPU oracle.  Returns false if
// max_attempts proposals were all rejected (upstream raises).
__device__ inline bool spawn_one(const MapLds& M, const Geo& g, uint32_t max_attempts,
                                 uint32_t env, uint64_t seed, uint32_t episode, double& x,
                                 double& z, double& ang, double* lp_out = nullptr) {
  const int lane = threadIdx.x & 63;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const U4 tw = philox(0u, episode, env, kTagTile, k0, k1);
  int pick = (int)(u01(tw.a, tw.b) * (double)M.n_drivable);
  pick = pick > M.n_drivable - 1 ? M.n_drivable - 1 : pick;
  const int ti = M.drivable[pick];
  const double fi = (double)(ti % M.width), fj = (double)(ti / M.width);
  for (uint32_t base = 0; base < max_attempts; base += kWave) {
    const uint32_t k = base + (uint32_t)lane;
    double px, pz, pa, lpo[2] = {0.0, 0.0};
    const bool ok = (k < max_attempts) && spawn_try(M, g, k0, k1, env, episode, k, fi, fj, px,
                                                    pz, pa, lpo);
    const uint64_t acc = __ballot(ok);
    if (acc) {
      const int w = __ffsll((unsigned long long)acc) - 1;
      x = bcast(px, w);
      z = bcast(pz, w);
      ang = bcast(pa, w);
      if (lp_out) {
        lp_out[0] = bcast(lpo[0], w);
        lp_out[1] = bcast(lpo[1], w);
      }
      return true;
    }
  }
  return false;
}

// The same over a whole workgroup (every thread calls; nthreads = blockDim.x, a
// multiple of 64): proposals k = nthreads*round + tid; per round each wave
// publishes its lowest accepting lane in LDS, and the lowest accepting wave
// wins -- again the first accepted k of the sequential loop.  `scratch` is 48 B
// per wave of LDS.  The winner's lane position (dist, angle_rad) comes back too.
__device__ inline bool spawn_block(const MapLds& M, const Geo& g, uint32_t max_attempts,
                                   uint32_t env, uint64_t seed, uint32_t episode,
                                   double* scratch, double& x, double& z, double& ang,
                                   double& dist, double& angle_rad) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const U4 tw = philox(0u, episode, env, kTagTile, k0, k1);
  int pick = (int)(u01(tw.a, tw.b) * (double)M.n_drivable);
  pick = pick > M.n_drivable - 1 ? M.n_drivable - 1 : pick;
  const int ti = M.drivable[pick];
  const double fi = (double)(ti % M.width), fj = (double)(ti / M.width);
  double* wx = scratch;              // [nw]
  double* wz = scratch + nw;         // [nw]
  double* wa = scratch + 2 * nw;     // [nw]
  double* wd = scratch + 3 * nw;     // [nw] lane dist of the winner
  double* wr = scratch + 4 * nw;     // [nw] lane angle_rad of the winner
  int* flag = reinterpret_cast<int*>(scratch + 5 * nw);  // [nw]
  for (uint32_t base = 0; base < max_attempts; base += blockDim.x) {
    const uint32_t k = base + (uint32_t)tid;
    double px, pz, pa, lpo[2] = {0.0, 0.0};
    const bool ok = (k < max_attempts) && spawn_try(M, g, k0, k1, env, episode, k, fi, fj, px,
                                                    pz, pa, lpo);
    const uint64_t acc = __ballot(ok);
    const int first = acc ? __ffsll((unsigned long long)acc) - 1 : -1;
    if (lane == 0) flag[wave] = first;
    if (first >= 0 && lane == first) {
      wx[wave] = px;
      wz[wave] = pz;
      wa[wave] = pa;
      wd[wave] = lpo[0];
      wr[wave] = lpo[1];
    }
    __syncthreads();
    int win = -1;
    for (int w = 0; w < nw; ++w)
      if (flag[w] >= 0) {
        win = w;
        break;
      }
    if (win >= 0) {
      x = wx[win];
      z = wz[win];
      ang = wa[win];
      dist = wd[win];
      angle_rad = wr[win];
    }
    __syncthreads();
    if (win >= 0) return true;
  }
  return false;
}

}  // namespace dt
