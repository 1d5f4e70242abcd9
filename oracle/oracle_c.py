"""TEST INFRASTRUCTURE ONLY — ctypes front-end of oracle/_build/liboracle.so
(the C restatement, dtsim_oracle.c).  Used by tests/ and bench.py's
cpu_baseline leg; never by the product.

The oracle takes the same ``dt_config`` / ``dt_map`` structs as the product's
ABI (include/dtsim.h) — they are the contract's data, not its implementation —
but builds them itself from the map rows and its own constants.
"""
import ctypes
import math
import os
import subprocess

import numpy as np

from oracle import dtsim_ref as R

HERE = os.path.dirname(os.path.abspath(__file__))
# DTSIM_ORACLE_LIB: another build of the same sources, loaded as is (the
# sanitizer build of `make asan`, tests/test_asan.py)
SO = os.environ.get('DTSIM_ORACLE_LIB') or os.path.join(HERE, '_build', 'liboracle.so')


def build():
    r = subprocess.run(['make', '-s', '-C', HERE], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('oracle build failed:\n' + r.stdout + r.stderr)
    return SO


class _Cfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        'road_tile_size', 'robot_speed', 'wheel_dist', 'delta_time', 'robot_width',
        'robot_length', 'camera_forward_dist', 'accept_start_angle_deg', 'reset_safety',
        'reward_scale', 'two_pi', 'rad2deg')] + \
        [(n, ctypes.c_uint32) for n in ('max_steps', 'max_env_steps', 'max_spawn_attempts')] + \
        [(n, ctypes.c_int32) for n in ('repeat_actions', 'frame_skip', 'action_mode',
                                       'clip_action', 'reward_speed_measured',
                                       'front_probe_length', 'auto_reset')] + \
        [('safety_rad_mult', ctypes.c_double)]


class _LineParams(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint8 * 3) for k in (
        'hsv_white1', 'hsv_white2', 'hsv_yellow1', 'hsv_yellow2', 'hsv_red1', 'hsv_red2',
        'hsv_red3', 'hsv_red4')] + [('dilation_kernel_size', ctypes.c_int32),
                                    ('canny_lo', ctypes.c_double), ('canny_hi', ctypes.c_double)]


class _Map(ctypes.Structure):
    _fields_ = [('width', ctypes.c_int32), ('height', ctypes.c_int32),
                ('kind', ctypes.c_void_p), ('curve_start', ctypes.c_void_p),
                ('curves', ctypes.c_void_p), ('headings', ctypes.c_void_p),
                ('n_objects', ctypes.c_int32), ('objects', ctypes.c_void_p),
                ('n_spawn_objects', ctypes.c_int32), ('spawn_objects', ctypes.c_void_p)]


_MODES = {'wheels': 0, 'tanh': 1, 'steering': 2}
_KINDS = {'straight': 1, 'curve_left': 2, 'curve_right': 3, '3way_left': 4, '3way_right': 5,
          '4way': 6}


def make_cfg(sc: 'R.SimConfig', auto_reset=True):
    c = _Cfg()
    c.road_tile_size = sc.road_tile_size
    c.robot_speed = sc.robot_speed
    c.wheel_dist = R.WHEEL_DIST
    c.delta_time = 1.0 / sc.frame_rate
    c.robot_width = R.ROBOT_WIDTH
    c.robot_length = R.ROBOT_LENGTH
    c.camera_forward_dist = R.CAMERA_FORWARD_DIST
    c.accept_start_angle_deg = sc.accept_start_angle_deg
    c.reset_safety = sc.reset_safety
    c.reward_scale = sc.reward_scale
    c.two_pi = 2 * math.pi
    c.rad2deg = float(np.rad2deg(1.0))
    c.max_steps = sc.max_steps
    c.max_env_steps = sc.max_env_steps
    c.max_spawn_attempts = sc.max_spawn_attempts
    c.repeat_actions = sc.repeat_actions
    c.frame_skip = sc.frame_skip
    c.action_mode = _MODES[sc.action_mode]
    c.clip_action = int(sc.clip_action)
    c.reward_speed_measured = int(sc.reward_speed_measured)
    c.front_probe_length = int(sc.front_probe_length)
    c.auto_reset = int(auto_reset)
    c.safety_rad_mult = R.SAFETY_RAD_MULT
    return c


class OracleMap:
    """Map arrays built by the oracle's own MapRef (restated _load_map/_get_curve)."""

    def __init__(self, rows, road_tile_size=R.ROAD_TILE_SIZE, objects=()):
        m = R.MapRef(rows, road_tile_size, objects)
        T = m.grid_width * m.grid_height
        self.width, self.height = m.grid_width, m.grid_height
        self.kind = np.full(T, -1, np.int8)
        per_tile = [None] * T
        for t, tile in enumerate(m.grid):
            if tile is None:
                continue
            if tile['drivable']:
                self.kind[t] = _KINDS[tile['kind']]
                per_tile[t] = tile['curves']
            else:
                self.kind[t] = 0
        self.curve_start = np.zeros(T + 1, np.int32)
        self.curve_start[1:] = np.cumsum([0 if c is None else len(c) for c in per_tile])
        C = int(self.curve_start[-1])
        self.curves = np.zeros((C, 4, 3))
        self.headings = np.zeros((C, 3))
        for t, cv in enumerate(per_tile):
            if cv is not None:
                a, b = self.curve_start[t], self.curve_start[t + 1]
                self.curves[a:b] = cv
                self.headings[a:b] = R.tile_headings(cv)
        # objects in the ABI layout (include/dtsim.h DT_OBJ_*), from the oracle's MapRef
        recs = []
        for pos, c, nv, r in zip(m.collidable_centers, m.collidable_corners,
                                 m.collidable_norms, m.collidable_safety_radii):
            rec = np.zeros(20)
            rec[0:3] = pos
            rec[3] = r
            rec[4:12] = np.asarray(c).reshape(-1)
            rec[12:16] = np.asarray(nv).reshape(-1)
            for a in range(2):
                p = np.asarray(c) @ np.asarray(nv)[a]
                rec[16 + 2 * a], rec[17 + 2 * a] = p.min(), p.max()
            recs.append(rec)
        self.objects = np.ascontiguousarray(np.array(recs).reshape(-1, 20))
        self.spawn_objects = np.ascontiguousarray(np.array(
            [np.r_[o['pos'], max(o['max_coords']) * 0.5 * o['scale'] + R.MIN_SPAWN_OBJ_DIST]
             for o in m.objects]).reshape(-1, 4))
        self.c = _Map(self.width, self.height, self.kind.ctypes.data, self.curve_start.ctypes.data,
                      self.curves.ctypes.data, self.headings.ctypes.data,
                      len(self.objects), self.objects.ctypes.data,
                      len(self.spawn_objects), self.spawn_objects.ctypes.data)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


class OracleBatch:
    """N envs stepped by the C oracle with the product's batch semantics."""

    def __init__(self, rows, n, seed=123, sim_config=None, auto_reset=True, env_base=0,
                 objects=()):
        if not os.path.exists(SO) or os.path.getmtime(SO) < max(
                os.path.getmtime(os.path.join(HERE, f)) for f in os.listdir(HERE)
                if f.endswith('.c')):
            build()
        self.L = ctypes.CDLL(SO)
        self.sc = sim_config or R.SimConfig()
        self.cfg = make_cfg(self.sc, auto_reset)
        self.map = OracleMap(rows, self.sc.road_tile_size, objects)
        self.n = n
        self.env_base = env_base
        self.seed = np.full(n, seed, np.uint64)
        self.x = np.zeros(n)
        self.z = np.zeros(n)
        self.angle = np.zeros(n)
        self.step_count = np.zeros(n, np.uint32)
        self.env_step = np.zeros(n, np.uint32)
        self.episode = np.zeros(n, np.uint32)
        self.spawn_k = np.full(n, -1, np.int32)

    def _state(self):
        return [_p(a) for a in (self.x, self.z, self.angle, self.step_count, self.env_step,
                                self.episode)]

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        rc = self.L.oracle_reset(ctypes.byref(self.cfg), ctypes.byref(self.map.c), self.n,
                                 ctypes.c_uint32(self.env_base), _p(self.seed), _p(m),
                                 *self._state(), _p(self.spawn_k))
        if rc:
            raise R.SpawnError('oracle_reset rc=%d' % rc)

    def step(self, actions):
        a = np.ascontiguousarray(actions, np.float32)
        assert a.shape == (self.n, 2)
        out = dict(reward=np.zeros(self.n), reward_mod=np.zeros(self.n),
                   done=np.zeros(self.n, np.uint8), obs=np.zeros((self.n, 2), np.float32),
                   lanepos=np.zeros((self.n, 4)), tile=np.zeros(self.n, np.int32))
        rc = self.L.oracle_step(ctypes.byref(self.cfg), ctypes.byref(self.map.c), self.n,
                                ctypes.c_uint32(self.env_base), _p(self.seed), _p(a),
                                *self._state(), _p(out['reward']), _p(out['reward_mod']),
                                _p(out['done']), _p(out['obs']), _p(out['lanepos']),
                                _p(out['tile']))
        if rc:
            raise R.SpawnError('oracle_step rc=%d' % rc)
        return out

    def lane_pos(self):
        lp = np.zeros((self.n, 4))
        tile = np.zeros(self.n, np.int32)
        self.L.oracle_lane_pos(ctypes.byref(self.cfg), ctypes.byref(self.map.c), self.n,
                               _p(self.x), _p(self.z), _p(self.angle), _p(lp), _p(tile))
        return lp, tile

    def state(self):
        return dict(x=self.x.copy(), z=self.z.copy(), angle=self.angle.copy(),
                    step_count=self.step_count.copy(), env_step=self.env_step.copy(),
                    episode=self.episode.copy())

    def set_state(self, **kw):
        for k, v in kw.items():
            getattr(self, k)[...] = v


def philox(ctr, key):
    if not os.path.exists(SO):
        build()
    L = ctypes.CDLL(SO)
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    L.oracle_philox(c, k, o)
    return tuple(o)


def line_params_default():
    """Duckietown defaults (same values as dt_default_line_params)."""
    p = _LineParams()
    vals = [(0, 0, 150), (180, 60, 255), (25, 140, 100), (45, 255, 255), (0, 140, 100),
            (15, 255, 255), (165, 140, 100), (180, 255, 255)]
    for k, v in zip(('hsv_white1', 'hsv_white2', 'hsv_yellow1', 'hsv_yellow2', 'hsv_red1',
                     'hsv_red2', 'hsv_red3', 'hsv_red4'), vals):
        getattr(p, k)[:] = v
    p.dilation_kernel_size = 3
    p.canny_lo, p.canny_hi = 80.0, 200.0
    return p


class OracleRender:
    """Observation-path oracle (render_oracle.c)."""

    def __init__(self, rows, sim_config=None, params=None):
        if not os.path.exists(SO):
            build()
        self.L = ctypes.CDLL(SO)
        self.sc = sim_config or R.SimConfig()
        self.cfg = make_cfg(self.sc)
        self.map = OracleMap(rows, self.sc.road_tile_size)
        self.params = params or line_params_default()

    def render(self, x, z, angle):
        x, z, angle = (np.ascontiguousarray(v, np.float64) for v in (x, z, angle))
        n = len(x)
        gray = np.zeros((n, 120, 160), np.float32)
        masks = np.zeros((n, 4, 120, 160), np.uint8)
        rgb = np.zeros((n, 120, 160, 3), np.uint8)
        rc = self.L.oracle_render(ctypes.byref(self.cfg), ctypes.byref(self.map.c),
                                  ctypes.byref(self.params), n, _p(x), _p(z), _p(angle),
                                  _p(gray), _p(masks), _p(rgb))
        assert rc == 0
        return gray, masks, rgb

    def marks(self):
        cap = 1 << 16
        out = np.zeros((cap, 4), np.float32)
        ny = ctypes.c_int(0)
        n = self.L.oracle_marks(ctypes.byref(self.cfg), ctypes.byref(self.map.c), _p(out), cap,
                                ctypes.byref(ny))
        return out[:n], ny.value

    def line_detect(self, bgr, hsv=False):
        bgr = np.ascontiguousarray(bgr, np.uint8)
        n, h, w, _ = bgr.shape
        masks = np.zeros((n, 4, h, w), np.uint8)
        hs = np.zeros((n, h, w, 3), np.uint8) if hsv else None
        self.L.oracle_line_detect(ctypes.byref(self.params), _p(bgr), n, h, w, _p(masks), _p(hs))
        return (masks, hs) if hsv else masks


def bresenham(x0, y0, x1, y1):
    if not os.path.exists(SO):
        build()
    L = ctypes.CDLL(SO)
    cap = 4096
    buf = (ctypes.c_int * (2 * cap))()
    n = L.oracle_bresenham(x0, y0, x1, y1, buf, cap)
    return [(buf[2 * i], buf[2 * i + 1]) for i in range(min(n, cap))]
