/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle (C restatement).  Linked only by
 * tests/ and bench.py's cpu_baseline leg, never by the product.
 *
 * A plain-C, float64, one-env-at-a-time restatement of oracle/dtsim_ref.py
 * (itself the restatement of gym-duckietown's Simulator step/reset and the
 * reference's EnvironmentWrapper.step, utils/env_wrappers.py:213-253), used to
 * check the HIP kernels at batch sizes the numpy restatement cannot reach in
 * seconds.  Expression order follows dtsim_ref.py; the file must be compiled
 * with -ffp-contract=off so no multiply-add is fused (numpy never fuses them).
 * Citations per function are the SURVEY.md §8(a) rows.
 *
 * Parity status: pinned to dtsim_ref.py by tests/test_oracle_c.py; the
 * Simulator restatement itself is unpinned by reference fixtures (the
 * dependency is absent), see dtsim_ref.py's header.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/dtsim.h"

#define TAG_TILE 0x54494C45u
#define TAG_SPAWN_A 0x53504E41u
#define TAG_SPAWN_B 0x53504E42u

/* ---- Philox4x32-10 (Random123) ------------------------------------------ */
static void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
  }
}

static double u01(uint32_t a, uint32_t b) {
  return (double)((((uint64_t)a << 32) | b) >> 11) * (1.0 / 9007199254740992.0);
}

void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c[4] = {ctr[0], ctr[1], ctr[2], ctr[3]};
  philox(c, key[0], key[1]);
  memcpy(out, c, sizeof c);
}

static double norm3_(double a, double b, double c) { return sqrt((a * a + b * b) + c * c); }

/* ---- map helpers (A5) ---------------------------------------------------- */
typedef struct {
  const dt_config* cfg;
  const dt_map* map;
} ctx_t;

static int tile_index(const ctx_t* C, double x, double z) {
  double ts = C->cfg->road_tile_size;
  double fi = floor(x / ts), fj = floor(z / ts);
  if (fi < 0 || fj < 0 || fi >= C->map->width || fj >= C->map->height) return -1;
  return (int)fj * C->map->width + (int)fi;
}

static int drivable(const ctx_t* C, double x, double z) {
  int t = tile_index(C, x, z);
  return t >= 0 && C->map->kind[t] > 0;
}

/* ---- static objects (dtsim_ref.py _collision /
 * proximity_penalty2 / _inconvenient_spawn over the DT_OBJ_* records) ------- */
static void proj4(const double* xs, const double* zs, int stride, double nx, double nz,
                  double* lo, double* hi) {
  double l = xs[0] * nx + zs[0] * nz, h = l;
  for (int k = 1; k < 4; ++k) {
    double p = xs[k * stride] * nx + zs[k * stride] * nz;
    if (p < l) l = p;
    if (p > h) h = p;
  }
  *lo = l;
  *hi = h;
}

/* agent box at the actual centre (px, pz) vs every collidable object, by
 * separating axes (agent axes: dir / right) */
static int collide(const ctx_t* C, double px, double pz, double c, double s) {
  const dt_map* m = C->map;
  if (m->n_objects <= 0) return 0;
  double fx = c, fz = -s, rx = s, rz = c;
  double hw = C->cfg->robot_width * 0.5, hl = C->cfg->robot_length * 0.5;
  double ax[4], az[4];
  ax[0] = (px - hw * rx) - hl * fx; az[0] = (pz - hw * rz) - hl * fz;
  ax[1] = (px + hw * rx) - hl * fx; az[1] = (pz + hw * rz) - hl * fz;
  ax[2] = (px + hw * rx) + hl * fx; az[2] = (pz + hw * rz) + hl * fz;
  ax[3] = (px - hw * rx) + hl * fx; az[3] = (pz - hw * rz) + hl * fz;
  for (int o = 0; o < m->n_objects; ++o) {
    const double* ob = m->objects + (size_t)o * DT_OBJ_STRIDE;
    const double* cx = ob + DT_OBJ_CORNERS;
    int sep = 0;
    for (int a = 0; a < 2 && !sep; ++a) {
      double nx = a == 0 ? fx : rx, nz = a == 0 ? fz : rz, al, ah, bl, bh;
      proj4(ax, az, 1, nx, nz, &al, &ah);
      proj4(cx, cx + 1, 2, nx, nz, &bl, &bh);
      sep = ah < bl || bh < al;
    }
    for (int a = 0; a < 2 && !sep; ++a) {
      double nx = ob[DT_OBJ_NORMS + 2 * a], nz = ob[DT_OBJ_NORMS + 2 * a + 1], al, ah;
      proj4(ax, az, 1, nx, nz, &al, &ah);
      sep = ah < ob[DT_OBJ_PROJ + 2 * a] || ob[DT_OBJ_PROJ + 2 * a + 1] < al;
    }
    if (!sep) return 1;
  }
  return 0;
}

static double proximity(const ctx_t* C, double px, double pz) {
  const dt_map* m = C->map;
  const dt_config* g = C->cfg;
  double asr = ((g->robot_length > g->robot_width ? g->robot_length : g->robot_width) / 2) *
               g->safety_rad_mult;
  double pen = 0.0;
  for (int o = 0; o < m->n_objects; ++o) {
    const double* ob = m->objects + (size_t)o * DT_OBJ_STRIDE;
    double d = norm3_(ob[0] - px, ob[1] - 0.0, ob[2] - pz);
    double sc = (d - asr) - ob[DT_OBJ_SAFETY_RAD];
    if (sc < 0) pen = pen + sc;
  }
  return pen;
}

static int inconvenient(const ctx_t* C, double x, double z) {
  const dt_map* m = C->map;
  for (int o = 0; o < m->n_spawn_objects; ++o) {
    const double* so = m->spawn_objects + 4 * (size_t)o;
    if (norm3_(so[0] - x, so[1] - 0.0, so[2] - z) < so[3]) return 1;
  }
  return 0;
}

/* _valid_pose (A6) */
static int valid_pose(const ctx_t* C, double x, double z, double angle, double safety) {
  const dt_config* g = C->cfg;
  double c = cos(angle), s = sin(angle);
  double off = g->camera_forward_dist - (g->robot_length / 2);
  double px = x + off * c;
  double pz = z + off * (-s);
  double kw = (safety * 0.5) * g->robot_width;
  double kf = (safety * 0.5) * (g->front_probe_length ? g->robot_length : g->robot_width);
  if (!drivable(C, px, pz)) return 0;
  if (!drivable(C, px - kw * s, pz - kw * c)) return 0;
  if (!drivable(C, px + kw * s, pz + kw * c)) return 0;
  if (!drivable(C, px + kf * c, pz + kf * (-s))) return 0;
  return !collide(C, px, pz, c, s);
}

/* bezier_point (A9) with exact dyadic coefficients */
static void bez_point(const double* cps, double t, double out[3]) {
  double u = 1 - t;
  double c0 = u * u * u, c1 = 3 * t * (u * u), c2 = 3 * (t * t) * u, c3 = t * t * t;
  for (int d = 0; d < 3; ++d) {
    double p = c0 * cps[0 * 3 + d];
    p = p + c1 * cps[1 * 3 + d];
    p = p + c2 * cps[2 * 3 + d];
    p = p + c3 * cps[3 * 3 + d];
    out[d] = p;
  }
}

static double norm3(double a, double b, double c) { return sqrt((a * a + b * b) + c * c); }

/* get_lane_pos2 (A8-A10).  returns 0 if NotInLane */
static int lane_pos(const ctx_t* C, double x, double z, double angle, double lp[4]) {
  int t = tile_index(C, x, z);
  if (t < 0 || C->map->kind[t] <= 0) return 0;
  double c = cos(angle), s = sin(angle);
  double dx = c, dz = -s;
  /* np.argmax(curve_headings @ dir): the first of the largest */
  int k0 = C->map->curve_start[t], k1 = C->map->curve_start[t + 1], ci = k0;
  double best = 0.0;
  for (int k = k0; k < k1; ++k) {
    const double* hd = C->map->headings + (size_t)k * 3;
    double d = (hd[0] * dx + hd[1] * 0.0) + hd[2] * dz;
    if (k == k0 || d > best) { best = d; ci = k; }
  }
  const double* cps = C->map->curves + (size_t)ci * 12;
  double tb = 0.0, tt = 1.0;
  for (int n = 8; n > 0; --n) {
    double mid = (tb + tt) * 0.5;
    double pb[3], pt[3];
    bez_point(cps, tb, pb);
    bez_point(cps, tt, pt);
    double db = norm3(pb[0] - x, pb[1] - 0.0, pb[2] - z);
    double dt = norm3(pt[0] - x, pt[1] - 0.0, pt[2] - z);
    if (db < dt) tt = mid; else tb = mid;
  }
  double tm = (tb + tt) * 0.5;
  double pt[3];
  bez_point(cps, tm, pt);
  /* bezier_tangent */
  double u = 1 - tm;
  double a0 = 3 * (u * u), a1 = 6 * u * tm, a2 = 3 * (tm * tm);
  double tg[3];
  for (int d = 0; d < 3; ++d) {
    double p = a0 * (cps[3 + d] - cps[d]);
    p = p + a1 * (cps[6 + d] - cps[3 + d]);
    p = p + a2 * (cps[9 + d] - cps[6 + d]);
    tg[d] = p;
  }
  double nn = norm3(tg[0], tg[1], tg[2]);
  tg[0] = tg[0] / nn; tg[1] = tg[1] / nn; tg[2] = tg[2] / nn;
  double dot = (dx * tg[0] + 0.0 * tg[1]) + dz * tg[2];
  if (dot > 1) dot = 1;
  if (dot < -1) dot = -1;
  /* rightVec = cross(tangent, [0,1,0]) = (-tz, 0, tx) */
  double rx = 0.0 - tg[2], rz = tg[0];
  double px = x - pt[0], pz = z - pt[2];
  double dist = (px * rx + (0.0 - pt[1]) * 0.0) + pz * rz;
  double ang = acos(dot);
  if ((dx * rx + 0.0) + dz * rz < 0) ang = -ang;
  lp[0] = dist;
  lp[1] = dot;
  lp[2] = ang * C->cfg->rad2deg;
  lp[3] = ang;
  return 1;
}

/* _update_pos (A4) */
static void update_pos(const dt_config* g, double* x, double* z, double* angle, double vl,
                       double vr) {
  double dtm = g->delta_time;
  if (vl == vr) {
    double k = dtm * vl;
    *x = *x + k * cos(*angle);
    *z = *z + k * (-sin(*angle));
    return;
  }
  double l = g->wheel_dist;
  double w = (vr - vl) / l;
  double r = (l * (vl + vr)) / (2 * (vl - vr));
  double rot = w * dtm;
  double px = *x, pz = *z;
  double cx = px + r * sin(*angle);
  double cz = pz + r * cos(*angle);
  double ddx = px - cx, ddz = pz - cz;
  double cr = cos(rot), sr = sin(rot);
  double ndx = ddx * cr + ddz * sr;
  double ndz = ddz * cr - ddx * sr;
  *x = cx + ndx;
  *z = cz + ndz;
  *angle = *angle + rot;
}

static void map_action(const dt_config* g, float a0, float a1, double* vl, double* vr) {
  if (g->action_mode == DT_ACTION_TANH) {
    a0 = a0 / 2.0f; a0 = a0 + 0.5f;
    a1 = a1 / 2.0f; a1 = a1 + 0.5f;
    *vl = a0; *vr = a1;
  } else if (g->action_mode == DT_ACTION_STEERING) {
    double vel = a0, ang = a1;
    double kinv_r = (1.0 + 0.0) / 27.0, kinv_l = (1.0 - 0.0) / 27.0;
    double om_r = (vel + 0.5 * ang * 0.102) / 0.0318;
    double om_l = (vel - 0.5 * ang * 0.102) / 0.0318;
    double ur = om_r * kinv_r, ul = om_l * kinv_l;
    ur = ur < 1.0 ? ur : 1.0; ur = ur > -1.0 ? ur : -1.0;
    ul = ul < 1.0 ? ul : 1.0; ul = ul > -1.0 ? ul : -1.0;
    *vl = ul * 0.8; *vr = ur;
  } else {
    *vl = a0; *vr = a1;
  }
}

static int spawn(const ctx_t* C, uint64_t seed, uint32_t env, uint32_t episode, double* x,
                 double* z, double* angle, int32_t* k_out) {
  const dt_config* g = C->cfg;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  int n_drv = 0;
  for (int t = 0; t < C->map->width * C->map->height; ++t) n_drv += C->map->kind[t] > 0;
  if (n_drv == 0) return DT_E_ARG;
  uint32_t c[4] = {0, episode, env, TAG_TILE};
  philox(c, k0, k1);
  int pick = (int)(u01(c[0], c[1]) * n_drv);
  if (pick > n_drv - 1) pick = n_drv - 1;
  int ti = -1;
  for (int t = 0, m = 0; t < C->map->width * C->map->height; ++t)
    if (C->map->kind[t] > 0 && m++ == pick) { ti = t; break; }
  double fi = ti % C->map->width, fj = ti / C->map->width;
  double M = g->accept_start_angle_deg;
  for (uint32_t k = 0; k < g->max_spawn_attempts; ++k) {
    uint32_t a[4] = {k, episode, env, TAG_SPAWN_A};
    uint32_t b[4] = {k, episode, env, TAG_SPAWN_B};
    philox(a, k0, k1);
    philox(b, k0, k1);
    double px = (fi + u01(a[0], a[1])) * g->road_tile_size;
    double pz = (fj + u01(a[2], a[3])) * g->road_tile_size;
    double pa = g->two_pi * u01(b[0], b[1]);
    if (inconvenient(C, px, pz)) continue;
    if (!valid_pose(C, px, pz, pa, g->reset_safety)) continue;
    double lp[4];
    if (!lane_pos(C, px, pz, pa, lp)) continue;
    if (!(-M < lp[2] && lp[2] < M)) continue;
    *x = px; *z = pz; *angle = pa;
    if (k_out) *k_out = (int32_t)k;
    return 0;
  }
  return DT_E_SPAWN;
}

/* Simulator.reset + EnvironmentWrapper.reset for the masked envs.
 * env_base: global id of env 0 of this batch (keys the Philox stream). */
int oracle_reset(const dt_config* cfg, const dt_map* map, int n, uint32_t env_base,
                 const uint64_t* seed, const uint8_t* mask, double* x, double* z, double* angle,
                 uint32_t* step_count, uint32_t* env_step, uint32_t* episode, int32_t* spawn_k) {
  ctx_t C = {cfg, map};
  int rc = 0;
  for (int e = 0; e < n; ++e) {
    if (mask && !mask[e]) continue;
    int r = spawn(&C, seed[e], env_base + (uint32_t)e, episode[e], &x[e], &z[e], &angle[e],
                  spawn_k ? &spawn_k[e] : 0);
    if (r) { rc = r; continue; }
    step_count[e] = 0;
    env_step[e] = 0;
    episode[e] += 1;
  }
  return rc;
}

/* EnvironmentWrapper.step over repeat_actions Simulator.step calls (A1-A12). */
int oracle_step(const dt_config* cfg, const dt_map* map, int n, uint32_t env_base,
                const uint64_t* seed, const float* actions, double* x, double* z, double* angle,
                uint32_t* step_count, uint32_t* env_step, uint32_t* episode, double* reward,
                double* reward_mod, uint8_t* done, float* obs, double* lanepos, int32_t* tile) {
  ctx_t C = {cfg, map};
  int rc = 0;
  for (int e = 0; e < n; ++e) {
    double vl, vr;
    map_action(cfg, actions[2 * e], actions[2 * e + 1], &vl, &vr);
    if (cfg->clip_action) {
      vl = vl < -1 ? -1 : (vl > 1 ? 1 : vl);
      vr = vr < -1 ? -1 : (vr > 1 ? 1 : vr);
    }
    double wl = vl * cfg->robot_speed * 1, wr = vr * cfg->robot_speed * 1;
    double tr = 0.0, trm = 0.0;
    int dn = 0;
    for (int rep = 0; rep < cfg->repeat_actions; ++rep) {
      double speed = 0;
      for (int f = 0; f < cfg->frame_skip; ++f) {
        double ox = x[e], oz = z[e];
        update_pos(cfg, &x[e], &z[e], &angle[e], wl, wr);
        step_count[e] += 1;
        speed = norm3(x[e] - ox, 0.0, z[e] - oz) / cfg->delta_time;
      }
      double r;
      int sd = 0;
      if (!valid_pose(&C, x[e], z[e], angle[e], 1.0)) {
        r = -1000; sd = 1;
      } else if (step_count[e] >= cfg->max_steps) {
        r = 0; sd = 1;
      } else {
        double lp[4];
        double sp = cfg->reward_speed_measured ? speed : cfg->robot_speed;
        double off = cfg->camera_forward_dist - (cfg->robot_length / 2);
        double pen = map->n_objects > 0 ? proximity(&C, x[e] + off * cos(angle[e]),
                                                     z[e] + off * (-sin(angle[e])))
                                         : 0.0;
        if (lane_pos(&C, x[e], z[e], angle[e], lp)) {
          double ad = lp[0] < 0 ? -lp[0] : lp[0];
          r = ((1.0 * sp) * lp[1] + (-10) * ad) + 40 * pen;
        } else {
          r = 40 * pen;
        }
      }
      double rm = (r == -1000) ? -10 : (r > 0 ? r + 10 : r + 4);
      tr = tr + r;
      trm = trm + rm;
      env_step[e] += 1;
      dn = sd || env_step[e] > cfg->max_env_steps;
      if (dn) break;
    }
    trm = trm * cfg->reward_scale;
    reward[e] = tr;
    reward_mod[e] = trm;
    done[e] = (uint8_t)dn;
    double lp[4];
    int inl = lane_pos(&C, x[e], z[e], angle[e], lp);
    if (lanepos) {
      for (int q = 0; q < 4; ++q) lanepos[4 * e + q] = inl ? lp[q] : NAN;
    }
    if (tile) tile[e] = tile_index(&C, x[e], z[e]);
    if (dn && cfg->auto_reset) {
      int r = spawn(&C, seed[e], env_base + (uint32_t)e, episode[e], &x[e], &z[e], &angle[e], 0);
      if (r) rc = r;
      else {
        step_count[e] = 0;
        env_step[e] = 0;
        episode[e] += 1;
        inl = lane_pos(&C, x[e], z[e], angle[e], lp);
      }
    }
    if (obs) {
      obs[2 * e] = inl ? (float)lp[0] : 0.0f;
      obs[2 * e + 1] = inl ? (float)lp[3] : 0.0f;
    }
  }
  return rc;
}

int oracle_lane_pos(const dt_config* cfg, const dt_map* map, int n, const double* x,
                    const double* z, const double* angle, double* lanepos, int32_t* tile) {
  ctx_t C = {cfg, map};
  for (int e = 0; e < n; ++e) {
    double lp[4];
    int inl = lane_pos(&C, x[e], z[e], angle[e], lp);
    for (int q = 0; q < 4; ++q) lanepos[4 * e + q] = inl ? lp[q] : NAN;
    if (tile) tile[e] = tile_index(&C, x[e], z[e]);
  }
  return 0;
}
