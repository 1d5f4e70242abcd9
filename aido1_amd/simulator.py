"""Simulator — the per-environment, gym-shaped drop-in for gym-duckietown's
``Simulator`` as the reference constructs it (duckietown_rl/env.py:4-20) and
drives it (utils/env_wrappers.py:103-134, train-ddpg-cnn.py:40-57,
duckietown_rl/utils.py:60-77).

It is a view of a one-env VecEnv handle: ``step`` is one Simulator step
(repeat 1, no wrapper cap, no auto-reset — the wrappers above it own those),
followed by a render of the new pose.  Surface used by the reference:

  step(action) -> (obs HxWx3 uint8, reward float, done bool, info dict)
  reset() -> obs;  seed(s);  render(mode);  close()
  observation_space (Box uint8, .low[0,0,0] / .high[0,0,0] read by
  ResizeWrapper, duckietown_rl/wrappers.py:12-13)
  action_space (.shape[0], .high[0], .low, .sample(): train-ddpg-cnn.py:56-57,110,118)
  cur_pos, cur_angle, step_count, get_lane_pos2()

The observation is the build's 120x160 ego-centric top-down raster (the
reference's OpenGL 640x480 camera frame does not exist here; the reference's
wrappers resize every frame to 120x160 anyway, ResizeWrapper /
PreliminaryTransformer, so camera_width/height are accepted and ignored).
"""
import numpy as np
import torch

from aido1_amd.config import EnvConfig, REWARD_INVALID_POSE  # noqa: F401
from aido1_amd.render import H, W, RenderOutput

U32_MAX = 0xFFFFFFFF


class Box:
    """Minimal gym.spaces.Box (gym is not a dependency)."""

    def __init__(self, low, high, shape, dtype, seed=None):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, self.dtype)
        self.high = np.full(self.shape, high, self.dtype)
        self._rng = np.random.default_rng(seed)

    def sample(self):
        if self.dtype.kind == 'f':
            return self._rng.uniform(self.low, self.high).astype(self.dtype)
        return self._rng.integers(self.low, self.high.astype(np.int64) + 1).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high)

    def __repr__(self):
        return 'Box(%s, %s)' % (self.shape, self.dtype)


LanePosition = __import__('collections').namedtuple('LanePosition',
                                                    'dist dot_dir angle_deg angle_rad')


class NotInLane(Exception):
    pass


class Simulator:
    """gym-duckietown Simulator constructor surface (aido1 era) on libdtsim."""

    metadata = {'render.modes': ['rgb_array', 'human']}
    reward_range = (-1000, 1000)

    def __init__(self, seed=None, map_name='loop_empty', max_steps=500001, domain_rand=False,
                 camera_width=640, camera_height=480, accept_start_angle_deg=60,
                 full_transparency=False, distortion=False, frame_skip=1, draw_curve=False,
                 draw_bbox=False, robot_speed=None, frame_rate=30, device=None, env_id=0,
                 **unsupported):
        if domain_rand:
            raise NotImplementedError('domain randomisation is not on the hot path '
                                      '(launch_env passes domain_rand=0, env.py:11)')
        if unsupported:
            raise TypeError('unsupported Simulator arguments: %s' % sorted(unsupported))
        from aido1_amd.vec_env import VecEnv
        cfg = EnvConfig(map_name=map_name, max_steps=max_steps,
                        accept_start_angle_deg=accept_start_angle_deg, frame_skip=frame_skip,
                        frame_rate=frame_rate, repeat_actions=1, max_env_steps=U32_MAX,
                        action_mode='wheels', auto_reset=False)
        if robot_speed is not None:
            cfg = cfg.replace(robot_speed=robot_speed)
        self.config = cfg
        self._seed = 0 if seed is None else int(seed)
        self._env = VecEnv(1, seed=self._seed, device=device, config=cfg, env_id_base=env_id)
        self._dev = self._env.device
        self._out = RenderOutput(1, self._dev, slots=1, rgb=True, masks=False)
        self._act = torch.zeros(1, 2, dtype=torch.float32, device=self._dev)
        self.map_name = map_name
        self.camera_width, self.camera_height = camera_width, camera_height
        self.observation_space = Box(0, 255, (H, W, 3), np.uint8)
        self.action_space = Box(-1, 1, (2,), np.float32, seed=self._seed)
        self.reward_range = (-1000, 1000)
        self._obs = None
        self._reset_done = False

    # ---- gym API ---------------------------------------------------------------
    def seed(self, seed=None):
        self._seed = 0 if seed is None else int(seed)
        self._env.seed(self._seed)
        self.action_space = Box(-1, 1, (2,), np.float32, seed=self._seed)
        return [self._seed]

    def reset(self):
        self._env.reset()
        self._reset_done = True
        return self._render()

    def step(self, action):
        if not self._reset_done:
            raise RuntimeError('call reset() before step()')
        a = np.asarray(action, dtype=np.float64).reshape(2)
        self._act.copy_(torch.from_numpy(a.astype(np.float32)).view(1, 2))
        out = self._env.step_into(self._act)
        obs = self._render()
        reward = float(out.reward.item())
        done = bool(out.done.item())
        lp = out.lanepos[0].cpu().numpy()
        info = {'Simulator': {
            'action': a.tolist(), 'cur_pos': self.cur_pos.tolist(), 'cur_angle': self.cur_angle,
            'step_count': self.step_count, 'tile': int(out.tile.item()),
            'lane_position': None if np.isnan(lp).any() else
            dict(zip(LanePosition._fields, (float(v) for v in lp))),
            'msg': ('Stopping the simulator because we are at an invalid pose.'
                    if done and reward == REWARD_INVALID_POSE else
                    'Stopping the simulator because we reached max_steps = %d' % self.config.max_steps
                    if done else '')}}
        return obs, reward, done, info

    def render(self, mode='human', close=False):
        if close:
            return None
        return self._obs.copy() if self._obs is not None else self._render()

    def close(self):
        self._env.close()

    # ---- state ---------------------------------------------------------------------
    @property
    def _state(self):
        return self._env.get_state()

    @property
    def cur_pos(self):
        s = self._state
        return np.array([s['x'][0], 0.0, s['z'][0]])

    @property
    def cur_angle(self):
        return float(self._state['angle'][0])

    @property
    def step_count(self):
        return int(self._state['step_count'][0])

    def get_lane_pos2(self, pos=None, angle=None):
        """LanePosition of the current pose (pos/angle, if given, must be it)."""
        lp, _ = self._env.lane_pos()
        v = lp[0].cpu().numpy()
        if np.isnan(v).any():
            raise NotInLane('Point not in lane: %s' % self.cur_pos)
        return LanePosition(*(float(x) for x in v))

    def _render(self):
        self._out.restart()
        self._env.render_into(self._out)
        self._obs = self._out.rgb[0].cpu().numpy()
        return self._obs
