/*
 * dtsim.h — C ABI of libdtsim.so, the MI355X-native batched Duckietown
 * lane-following environment (aido1_amd).
 *
 * The reference (niksaz/aido1) drives ONE gym-duckietown `Simulator` per
 * process through `launch_env()` (duckietown_rl/env.py:4-20) and the
 * `EnvironmentWrapper.step` repeat loop (utils/env_wrappers.py:213-253).
 * This library replaces that per-env Python object with N environments whose
 * state lives in HBM and whose step/reset run as gfx950 kernels.  Every entry
 * point below names the reference call it replaces.
 *
 * Conventions
 *   - Every call returns int: 0 = ok, <0 = error (DT_E_*).  No C++ exception
 *     crosses the ABI.  dt_last_error(h) returns a human-readable message.
 *   - Pointers documented "device" must be device memory of the handle's GPU
 *     (e.g. torch tensors' data_ptr()), contiguous, in the documented layout.
 *     Pointers documented "host" are ordinary host memory.
 *   - All device work is enqueued on the given stream (hipStream_t passed as
 *     void*; NULL = the default stream).  Only dt_get_state / dt_set_state /
 *     dt_seed synchronise.
 *   - One handle per (process, GPU).  Calls on one handle are not thread-safe.
 */
#ifndef AIDO1_AMD_DTSIM_H
#define AIDO1_AMD_DTSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DT_ABI_VERSION 13 /* 2: curves per tile vary (curve_start), intersections;
                             3: static objects in dt_map, safety_rad_mult;
                             4: dt_render_io.pose / list_cap, dt_copy_pose,
                                dt_step_many pose output;
                             5: dtactor.h: dt_conv12 and dt_conv1_bands
                                removed, partials [n, 32, 2];
                             6: dtactor.h: dt_conv1_split / dt_conv32_split
                                (two weight sets in one launch);
                             7: dt_line_detect_ws / dt_hough_lines_ws and
                                their workspace queries (any image size),
                                dt_hough_lines count -2 (max_lines reached);
                             8: dttrain.h non-finite guards: dt_guard_scan, a
                                guard word for dt_bn_leaky_fwd / _bwd / dt_adam;
                                dtactor.h reference-mode partials [n, 32, 3]
                                (mean, M2, centre) with centred activations;
                                dtupd.h (the update's convolutions and the
                                conv trunk's BatchNorm hand-off);
                             9: dtactor.h dt_episode_account (episode sums and
                                the finished-episode ring); dt_render_order;
                            10: palette-index frames: dt_render_io.index,
                                dt_palette_gray, dt_conv1_index_split,
                                dt_frame_gather frame_kind
                            11: dtactor.h dt_conv1x_split / dt_conv32x_split
                                (the float32-accurate convolutions);
                            12: dtupd.h dt_upd_linear_fwd_drop / _dgrad_drop
                                (dropout folded into the linears);
                            13: dtactor.h dt_actor_head_x3_drop,
                                dt_actor_head_f16_drop */

/* error codes */
#define DT_OK 0
#define DT_E_ARG (-1)      /* bad argument (null handle, bad size, bad map) */
#define DT_E_HIP (-2)      /* HIP runtime error (see dt_last_error) */
#define DT_E_SPAWN (-3)    /* reset exhausted max_spawn_attempts (upstream raises) */
#define DT_E_NODEV (-4)    /* no usable gfx950 device */

/* action contracts (how the [N,2] f32 action is turned into wheel velocities) */
#define DT_ACTION_WHEELS 0   /* (left, right) wheel velocities, as the Simulator takes them */
#define DT_ACTION_TANH 1     /* EnvironmentWrapper.step: a = a/2 + 0.5 in f32, in place
                                (utils/env_wrappers.py:214-216, config.json:88 tanh head) */
#define DT_ACTION_STEERING 2 /* (vel, steer) -> SteeringToWheelVelWrapper -> ActionWrapper
                                (duckietown_rl/wrappers.py:138-161, :99-101; order
                                train-ddpg-cnn.py:48-50: the x0.8 lands on the LEFT wheel) */

/* Kinds of a map tile (upstream Simulator._load_map tile dict). */
#define DT_TILE_EMPTY (-1)       /* 'empty' -> no tile; _get_tile returns None */
#define DT_TILE_OFFROAD 0        /* grass / asphalt / floor: drivable False */
#define DT_TILE_STRAIGHT 1
#define DT_TILE_CURVE_LEFT 2
#define DT_TILE_CURVE_RIGHT 3
#define DT_TILE_3WAY_LEFT 4      /* upstream kind.startswith('3way'): 6 lane curves */
#define DT_TILE_3WAY_RIGHT 5
#define DT_TILE_4WAY 6           /* a tile name containing '4' (angle 2): 12 lane curves */

/* Simulator + EnvironmentWrapper constants.  Every value mirrors an upstream
 * gym-duckietown constant or a reference config key; the host fills them from
 * the same Python expressions (aido1_amd/config.py) so the doubles are
 * bit-identical to the ones the reference computes. */
typedef struct dt_config {
  double road_tile_size;      /* ROAD_TILE_SIZE 0.61 */
  double robot_speed;         /* DEFAULT_ROBOT_SPEED 1.20 (wheelVels = a * speed) */
  double wheel_dist;          /* WHEEL_DIST 0.102 */
  double delta_time;          /* 1.0 / DEFAULT_FRAMERATE (30) */
  double robot_width;         /* ROBOT_WIDTH 0.13 + 0.02 */
  double robot_length;        /* ROBOT_LENGTH 0.18 */
  double camera_forward_dist; /* CAMERA_FORWARD_DIST 0.066 */
  double accept_start_angle_deg; /* env.py:14 -> 4 */
  double reset_safety;        /* _valid_pose safety factor in reset: 1.3 */
  double reward_scale;        /* config.json:7 environment.wrapper.reward_scale */
  double two_pi;              /* 2 * math.pi */
  double rad2deg;             /* numpy rad2deg factor 180/pi */
  uint32_t max_steps;         /* Simulator max_steps (env.py:10 -> 500001) */
  uint32_t max_env_steps;     /* config.json:5 wrapper.max_env_steps (2000); done |= env_step > it */
  uint32_t max_spawn_attempts;/* MAX_SPAWN_ATTEMPTS 5000 */
  int32_t repeat_actions;     /* config.json:6 wrapper.repeat_actions (3) */
  int32_t frame_skip;         /* DEFAULT_FRAME_SKIP 1 (update_physics per Simulator.step) */
  int32_t action_mode;        /* DT_ACTION_* */
  int32_t clip_action;        /* 1: Simulator.step clips the action to [-1, 1] */
  int32_t reward_speed_measured; /* 0: compute_reward(.., self.robot_speed); 1: measured |dpos|/dt */
  int32_t front_probe_length; /* 1: _valid_pose front probe uses ROBOT_LENGTH, 0: ROBOT_WIDTH */
  int32_t auto_reset;         /* 1: dt_step resets done envs in the same launch (VectorEnv) */
  double safety_rad_mult;     /* SAFETY_RAD_MULT 1.8: AGENT_SAFETY_RAD =
                                 max(robot_length, robot_width) / 2 * it (objects) */
} dt_config;

/* One collidable static object of dt_map.objects: DT_OBJ_STRIDE doubles
 * (upstream Simulator._load_objects -> collidable_centers / _corners / _norms /
 * _safety_radii, precomputed on the host by aido1_amd/maps.py):
 *   [DT_OBJ_CENTER + 0..2]  world position (x, y, z)
 *   [DT_OBJ_SAFETY_RAD]     safety radius (SAFETY_RAD_MULT * calculate_safety_radius)
 *   [DT_OBJ_CORNERS + 2k]   corner k (x, z), k = 0..3 (generate_corners)
 *   [DT_OBJ_NORMS + 2a]     axis a (x, z), a = 0, 1 (generate_norm)
 *   [DT_OBJ_PROJ + 2a]      (min, max) of the corners projected on axis a */
#define DT_OBJ_CENTER 0
#define DT_OBJ_SAFETY_RAD 3
#define DT_OBJ_CORNERS 4
#define DT_OBJ_NORMS 12
#define DT_OBJ_PROJ 16
#define DT_OBJ_STRIDE 20

/* A tile map.  Tile (i, j) is grid[j * width + i]; i follows +x, j follows +z
 * (upstream get_grid_coords / _get_tile). */
typedef struct dt_map {
  int32_t width;
  int32_t height;
  const int8_t* kind;           /* host [height*width] DT_TILE_* */
  const int32_t* curve_start;   /* host [height*width + 1]: tile t owns curves
                                   curve_start[t] .. curve_start[t+1]-1 (2 for straight /
                                   curve tiles, 6 for 3-way, 12 for 4-way, 0 off-road) */
  const double* curves;         /* host [C, 4, 3] world-frame Bezier control points, C =
                                   curve_start[height*width] (upstream _get_curve: template
                                   * tile_size @ R_y + centre) */
  const double* headings;       /* host [C, 3] curve headings (P3 - P0) divided by the
                                   Frobenius norm of the tile's heading matrix (the
                                   closest_curve_point np.linalg.norm quirk) */
  int32_t n_objects;            /* collidable static objects (0: none; <= 256) */
  const double* objects;        /* host [n_objects, DT_OBJ_STRIDE] or NULL: _collision in
                                   _valid_pose, proximity_penalty2 in the reward */
  int32_t n_spawn_objects;      /* visible objects for _inconvenient_spawn (<= 256) */
  const double* spawn_objects;  /* host [n_spawn_objects, 4] or NULL: (x, y, z, r): a
                                   spawn proposal within r of (x, y, z) is rejected */
} dt_map;

typedef struct dt_handle dt_handle;

/* ---- lifecycle ------------------------------------------------------- */

/* Replaces: Simulator(...) construction in launch_env() (duckietown_rl/env.py:6-17)
 * for n_envs environments on GPU `device`.  Every env is seeded with `seed`
 * (per-env Philox streams are keyed by (seed, env id)) and left un-reset:
 * call dt_reset before the first dt_step. */
int dt_create(const dt_config* cfg, const dt_map* map, uint64_t seed, int32_t n_envs,
              int32_t device, dt_handle** out);
int dt_destroy(dt_handle* h);
int32_t dt_n_envs(const dt_handle* h);
const char* dt_last_error(const dt_handle* h); /* h may be NULL: last create error */
int32_t dt_abi_version(void);

/* Replaces: Simulator.seed(s) / DuckietownEnvironmentWrapper.change_model(seed)
 * (utils/env_wrappers.py:126-130).  seeds: host [n_envs] or NULL (all = base).
 * env_id_base: global id of this handle's env 0 — the spawn stream of env e is
 * Philox(key = seed[e], counter = (k, episode, env_id_base + e, tag)), so shards
 * of one job on different GPUs draw disjoint streams.
 * Also zeroes every env's episode counter.  Synchronous. */
int dt_seed(dt_handle* h, const uint64_t* seeds, uint64_t base, uint32_t env_id_base);

/* Replaces: DuckietownEnvironmentWrapper.change_model(seed) for ONE env of the
 * batch (utils/env_wrappers.py:126-130, one env per pyramid_worker.py port):
 * env's seed = seed, its episode counter = 0; the others are untouched.
 * Synchronous. */
int dt_seed_env(dt_handle* h, int32_t env, uint64_t seed);

/* ---- hot path -------------------------------------------------------- */

/* Replaces: Simulator.reset() (spawn by rejection sampling, MAX_SPAWN_ATTEMPTS,
 * _valid_pose(safety 1.3), |angle_deg| < accept_start_angle_deg) and the
 * EnvironmentWrapper.reset counters (utils/env_wrappers.py:182-204).
 * mask: device [n_envs] u8 (nonzero = reset) or NULL = reset all. */
int dt_reset(dt_handle* h, const uint8_t* mask, void* stream);

/* Replaces: EnvironmentWrapper.step(action) (utils/env_wrappers.py:213-253) ->
 * repeat_actions x Simulator.step (update_physics, _compute_done_reward,
 * compute_reward, get_lane_pos2) -> BaselineAggregationFunction
 * (utils/reward_shaping/aggregation_functions.py:25-32), for all envs at once.
 *   actions    device [n,2] f32 (interpreted per cfg.action_mode)          required
 *   reward     device [n] f64  sum of raw Simulator rewards                required
 *   reward_mod device [n] f64  sum of aggregated rewards * reward_scale    required
 *   done       device [n] u8                                               required
 *   obs        device [n,2] f32 (dist, angle_rad) of the returned pose: the reset
 *              pose for envs that auto-reset; 0 when not in a lane        nullable
 *   lanepos    device [n,4] f64 terminal LanePosition (dist, dot_dir, angle_deg,
 *              angle_rad) before any auto-reset; NaN when not in a lane    nullable
 *   tile       device [n] i32 terminal tile index j*W+i, -1 off the grid   nullable
 */
int dt_step(dt_handle* h, const float* actions, double* reward, double* reward_mod,
            uint8_t* done, float* obs, double* lanepos, int32_t* tile, void* stream);

/* dt_step for the envs where mask (device [n] u8) is nonzero; the others keep
 * their state and their output entries (the env server batches whichever
 * per-env step requests are pending: pyramid_worker.py:25-32). */
int dt_step_masked(dt_handle* h, const uint8_t* mask, const float* actions, double* reward,
                   double* reward_mod, uint8_t* done, float* obs, double* lanepos, int32_t* tile,
                   void* stream);

/* k consecutive dt_step calls in one launch (the spawn-ahead refill blocks run in
 * the same grid): the same results as k dt_step calls over actions[d], with the
 * outputs of decision d at [d * n + env].  The explorer's rollout loop
 * (training/explorers.py) over k actions known ahead, e.g. random ones.
 *   actions    device [k,n,2] f32                                          required
 *   reward, reward_mod  device [k,n] f64; done device [k,n] u8             required
 *   obs        device [k,n,2] f32, as dt_step's                            nullable
 *   pose       device [k,3,n] f64: the pose each decision ends in (x, z, angle
 *              planes; the reset pose after a respawn), i.e. what dt_render of
 *              that decision draws (dt_render_io.pose = pose + 3 n d)  nullable
 * DT_E_ARG for a handle with 3 * 64 * n >= 2^31 (one launch's 32-bit output
 * offsets); step such a handle with dt_step. */
int dt_step_many(dt_handle* h, int32_t k, const float* actions, double* reward,
                 double* reward_mod, uint8_t* done, float* obs, double* pose, void* stream);

/* Replaces: Simulator.get_lane_pos2(cur_pos, cur_angle) for every env (no step).
 * lanepos device [n,4] f64 (NaN if NotInLane); tile device [n] i32 (nullable). */
int dt_lane_pos(dt_handle* h, double* lanepos, int32_t* tile, void* stream);

/* ---- observation path (config 3) --------------------------------------- */

#define DT_OBS_H 120
#define DT_OBS_W 160
#define DT_MASK_WHITE 0
#define DT_MASK_YELLOW 1
#define DT_MASK_RED 2
#define DT_MASK_EDGES 3

/* features/line_detector1.py LineDetectorHSV parameters (dtu.Configurable,
 * :18-34).  The values are not in the reference repo; dt_default_line_params
 * gives the Duckietown defaults (white [0,0,150]-[180,60,255], yellow
 * [25,140,100]-[45,255,255], red [0,140,100]-[15,255,255] U
 * [165,140,100]-[180,255,255], dilation 3, Canny [80,200]).  HSV is OpenCV's
 * 8-bit convention (H in [0,180)). */
typedef struct dt_line_params {
  uint8_t hsv_white1[3], hsv_white2[3];
  uint8_t hsv_yellow1[3], hsv_yellow2[3];
  uint8_t hsv_red1[3], hsv_red2[3], hsv_red3[3], hsv_red4[3];
  int32_t dilation_kernel_size; /* odd, 1..7, MORPH_ELLIPSE */
  double canny_lo, canny_hi;    /* Canny thresholds (apertureSize 3, L1 gradient) */
} dt_line_params;

int dt_default_line_params(dt_line_params* p);

/* Where dt_render writes. */
typedef struct dt_render_io {
  float* gray;          /* device [n, gray_slots, 120, 160] f32 rgb2gray in [0,1], or NULL */
  int32_t gray_slots;   /* frames per env in `gray` (3: a Transformer stack ring; 1: one frame) */
  int32_t gray_slot;    /* slot written by this call */
  const uint8_t* fresh; /* device [n] u8 or NULL: nonzero -> the frame goes to EVERY slot
                           (Transformer.reset fills the stack with copies,
                           utils/reward_shaping/env_utils.py:60-63) */
  uint8_t* masks;       /* device [n, 4, 120, 160] u8 255/0 {white, yellow, red, edges}, or NULL */
  uint8_t* rgb;         /* device [n, 120, 160, 3] u8 RGB raster, or NULL */
  const double* pose;   /* device [3, n] f64 planes (x, z, angle) to render, or NULL = the
                           handle's current state (a dt_copy_pose snapshot lets the next
                           dt_step run on another stream while this render reads it) */
  int32_t list_cap;     /* 0 in production.  > 0 lowers the number of non-uniform words
                           the kernel keeps in LDS, so tests exercise the global-memory
                           overflow path (results are identical either way) */
  uint8_t* index;       /* device [n, gray_slots, 120, 160] u8 palette-index frames, or
                           NULL (not both `gray` and `index`: DT_E_ARG): the frame's
                           palette bytes (0..7), same slots / fresh rules as `gray`.  A quarter of the grey frame's bytes and
                           lossless: gray = dt_palette_gray's table[index] bit for bit
                           (the actor's dt_conv1_index_split and dt_frame_gather read
                           such frames directly) */
} dt_render_io;

/* The 8 grey levels of the renderer's palette bytes (PreliminaryTransformer's
 * rgb2gray of each colour, float64 then float32): gray8[b] is the grey frame's
 * value wherever the index frame holds b.  Host memory. */
int dt_palette_gray(float* gray8);

/* Replaces, per env and fused in one launch (one workgroup per env, the frame
 * kept in LDS): Simulator.render_obs (build-defined 120x160 ego-centric
 * top-down raster: tile background + lane markings drawn as Bresenham
 * polylines, utils/bresenham.py:6-34), PreliminaryTransformer's rgb2gray
 * (utils/reward_shaping/env_utils.py:48-51) and LineDetectorHSV.setImage +
 * _colorFilter (features/line_detector1.py:134-141, :36-57): HSV inRange,
 * ellipse dilation, Canny(bgr, lo, hi, 3).  Renders the CURRENT pose (call it
 * after dt_step), or io->pose.  The envs are dispatched longest measured
 * render first (each launch records every env's cost and orders the next
 * launch's workgroups by it); the order never changes an output. */
int dt_render(dt_handle* h, const dt_render_io* io, void* stream);

/* Two consecutive decisions' renders in one launch (one drain for both):
 * io_a the earlier decision, io_b the later, each with its pose snapshot
 * (dt_step_many's per-decision poses), its ring slot (different slots of one
 * ring), its fresh flags and its own masks buffer; no rgb.  Every output
 * equals dt_render(io_a) followed by dt_render(io_b): io_a's stores that
 * io_b overwrites are not made (io_a never writes io_b's slot; an env io_b
 * refills gets no io_a frame), so the two halves never write one byte. */
int dt_render2(dt_handle* h, const dt_render_io* io_a, const dt_render_io* io_b, void* stream);

/* dt_render2 for three consecutive decisions (three slots of the ring):
 * equals dt_render(io_a), dt_render(io_b), dt_render(io_c) in that order. */
int dt_render3(dt_handle* h, const dt_render_io* io_a, const dt_render_io* io_b,
               const dt_render_io* io_c, void* stream);

/* Diagnostics of that dispatch order (synchronises): launches so far, each
 * env's last recorded cost (shader cycles) and the order the next launch
 * dispatches in (a permutation of 0..n-1).  cost / order: host [n] or NULL. */
int dt_render_order(dt_handle* h, uint32_t* launches, uint32_t* cost, int32_t* order);

/* Enqueue a copy of every env's current pose into pose (device [3, n] f64:
 * x, z, angle planes) on `stream`: the render of decision d can then read the
 * snapshot while dt_step of decision d + 1 runs on another stream. */
int dt_copy_pose(dt_handle* h, double* pose, void* stream);
int dt_set_line_params(dt_handle* h, const dt_line_params* p);

/* LineDetectorHSV on caller images (no environment; features/line_detector1.py
 * :134-141 setImage + _colorFilter :36-57): bgr device [n, height, width, 3]
 * u8; masks device [n, 4, height, width] u8 as above; hsv device [n, height,
 * width, 3] u8 or NULL (cvtColor BGR2HSV).  Images of <= 19200 pixels (e.g.
 * 120x160) run in LDS, one workgroup each; larger ones (e.g. the 640x480
 * camera frame of duckietown_rl/env.py:12-16) need a device workspace of
 * dt_line_detect_workspace(n, height, width) bytes (0 when none is needed) and
 * dt_line_detect_ws.  dt_line_detect is dt_line_detect_ws without one (so it
 * refuses larger images with DT_E_ARG).  Runs on the current device. */
size_t dt_line_detect_workspace(int32_t n, int32_t height, int32_t width);
int dt_line_detect_ws(const dt_line_params* p, const uint8_t* bgr, int32_t n, int32_t height,
                      int32_t width, uint8_t* masks, uint8_t* hsv, void* workspace,
                      size_t workspace_bytes, void* stream);
int dt_line_detect(const dt_line_params* p, const uint8_t* bgr, int32_t n, int32_t height,
                   int32_t width, uint8_t* masks, uint8_t* hsv, void* stream);

/* LineDetectorHSV._HoughLine (features/line_detector1.py:63-70):
 * cv2.HoughLinesP(edge, rho 1, theta pi/180, threshold, min_line_length,
 * max_line_gap) on n u8 images (non-zero = edge), e.g. a dt_render mask
 * plane (edge_color = the colour mask AND the edge mask, :55).  edge device
 * [n, height, width] u8; lines device [n, max_lines, 4] i32 (x1, y1, x2, y2)
 * in OpenCV's order; counts device [n] i32 = lines found, or
 *   -1: the image had more edge pixels than the LDS point list holds (~16k
 *       points at 120x160, of its 19,200 pixels), its lines are not valid;
 *   -2: max_lines lines were found with edge points still unvisited, so
 *       OpenCV (which has no cap) may find more: the max_lines rows are the
 *       first ones, the list is cut short.
 * dt_hough_lines runs in LDS (height*width <= 65536 and the accumulator +
 * image within 160 KB: 120x160 fits).  dt_hough_lines_ws with a workspace of
 * dt_hough_workspace(n, height, width) bytes keeps the accumulator, mask and
 * point list there instead: any image size, never -1.  One wave per image;
 * runs on the current device. */
int dt_hough_lines(const uint8_t* edge, int32_t n, int32_t height, int32_t width,
                   int32_t threshold, int32_t min_line_length, int32_t max_line_gap,
                   int32_t max_lines, int32_t* lines, int32_t* counts, void* stream);
size_t dt_hough_workspace(int32_t n, int32_t height, int32_t width);
int dt_hough_lines_ws(const uint8_t* edge, int32_t n, int32_t height, int32_t width,
                      int32_t threshold, int32_t min_line_length, int32_t max_line_gap,
                      int32_t max_lines, int32_t* lines, int32_t* counts, void* workspace,
                      size_t workspace_bytes, void* stream);

/* ---- state access (parity injection; synchronous) ---------------------- */
/* x, z, angle: host [n] f64; step_count (Simulator), env_step (wrapper),
 * episode (resets so far, keys the Philox spawn stream): host [n] u32.
 * Any pointer may be NULL (that field is skipped). */
int dt_get_state(dt_handle* h, double* x, double* z, double* angle, uint32_t* step_count,
                 uint32_t* env_step, uint32_t* episode);
int dt_set_state(dt_handle* h, const double* x, const double* z, const double* angle,
                 const uint32_t* step_count, const uint32_t* env_step, const uint32_t* episode);

/* Counters accumulated on the device since dt_create (synchronous read):
 * out[0] Simulator steps executed (each repeat that ran, x frame_skip = 1 env-step),
 * out[1] EnvironmentWrapper steps (agent decisions x envs), out[2] resets done,
 * out[3] episodes finished (done flags raised).  reset != 0 zeroes them after reading.
 * Replaces the "step per second" bookkeeping of training/explorers.py:215-240. */
int dt_stats(dt_handle* h, uint64_t out[4], int32_t reset);

/* Device-side error word (DT_E_SPAWN bit etc.) accumulated by kernels since the
 * last call; synchronous; clears it. */
int dt_check(dt_handle* h, uint32_t* flags);

#ifdef __cplusplus
}
#endif
#endif
