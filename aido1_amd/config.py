"""Simulator / EnvironmentWrapper configuration -> the C ABI's ``dt_config``.

Every constant is computed from the same Python expression gym-duckietown (aido1
era) or the reference uses, so the float64 handed to the kernels is
bit-identical to the one the reference computes:

  - Simulator constants: ROAD_TILE_SIZE, WHEEL_DIST, ROBOT_WIDTH = 0.13 + 0.02,
    ROBOT_LENGTH, CAMERA_FORWARD_DIST, DEFAULT_ROBOT_SPEED, DEFAULT_FRAMERATE,
    MAX_SPAWN_ATTEMPTS (upstream simulator.py, un-vendored).
  - launch_env kwargs: max_steps=500001, accept_start_angle_deg=4
    (duckietown_rl/env.py:7-17).
  - EnvironmentWrapper keys: max_env_steps, repeat_actions, reward_scale
    (config.json:3-16, read at utils/env_wrappers.py:166-168).
"""
import ctypes
import math
from dataclasses import dataclass, field, fields

ACTION_MODES = {'wheels': 0, 'tanh': 1, 'steering': 2}

# upstream Simulator constants
ROAD_TILE_SIZE = 0.61
WHEEL_DIST = 0.102
ROBOT_WIDTH = 0.13 + 0.02
ROBOT_LENGTH = 0.18
CAMERA_FORWARD_DIST = 0.066
DEFAULT_ROBOT_SPEED = 1.20
DEFAULT_FRAMERATE = 30
DEFAULT_FRAME_SKIP = 1
MAX_SPAWN_ATTEMPTS = 5000
SAFETY_RAD_MULT = 1.8      # [upstream] objects: safety circles (AGENT_SAFETY_RAD, radii)
MIN_SPAWN_OBJ_DIST = 0.25  # [upstream] _inconvenient_spawn margin
REWARD_INVALID_POSE = -1000


class DtConfig(ctypes.Structure):
    """Mirror of ``dt_config`` in include/dtsim.h (field order matters)."""
    _fields_ = [
        ('road_tile_size', ctypes.c_double),
        ('robot_speed', ctypes.c_double),
        ('wheel_dist', ctypes.c_double),
        ('delta_time', ctypes.c_double),
        ('robot_width', ctypes.c_double),
        ('robot_length', ctypes.c_double),
        ('camera_forward_dist', ctypes.c_double),
        ('accept_start_angle_deg', ctypes.c_double),
        ('reset_safety', ctypes.c_double),
        ('reward_scale', ctypes.c_double),
        ('two_pi', ctypes.c_double),
        ('rad2deg', ctypes.c_double),
        ('max_steps', ctypes.c_uint32),
        ('max_env_steps', ctypes.c_uint32),
        ('max_spawn_attempts', ctypes.c_uint32),
        ('repeat_actions', ctypes.c_int32),
        ('frame_skip', ctypes.c_int32),
        ('action_mode', ctypes.c_int32),
        ('clip_action', ctypes.c_int32),
        ('reward_speed_measured', ctypes.c_int32),
        ('front_probe_length', ctypes.c_int32),
        ('auto_reset', ctypes.c_int32),
        ('safety_rad_mult', ctypes.c_double),
    ]


@dataclass
class EnvConfig:
    """Constructor arguments of the reference's Simulator (env.py:7-17) plus the
    EnvironmentWrapper section of config.json, plus flags that pin choices the
    un-vendored upstream leaves uncertain (DESIGN.md "Upstream-spec
    uncertainty")."""
    map_name: str = 'loop_empty'
    max_steps: int = 500001
    accept_start_angle_deg: float = 4
    frame_skip: int = DEFAULT_FRAME_SKIP
    robot_speed: float = DEFAULT_ROBOT_SPEED
    frame_rate: int = DEFAULT_FRAMERATE
    road_tile_size: float = ROAD_TILE_SIZE
    max_env_steps: int = 2000
    repeat_actions: int = 3
    reward_scale: float = 1.0
    action_mode: str = 'wheels'
    clip_action: bool = True
    reward_speed_measured: bool = False
    front_probe_length: bool = True
    reset_safety: float = 1.3
    max_spawn_attempts: int = MAX_SPAWN_ATTEMPTS
    auto_reset: bool = True

    @classmethod
    def from_reference_config(cls, config, **overrides):
        """Build from the reference's config.json dict (utils/util.py:107-110)."""
        w = config['environment']['wrapper']
        head = config['model']['actor'][-1]['modules'][-1][-1]['name']
        kw = dict(max_env_steps=w['max_env_steps'], repeat_actions=w['repeat_actions'],
                  reward_scale=w['reward_scale'],
                  action_mode='tanh' if head == 'tanh' else 'wheels')
        kw.update(overrides)
        return cls(**kw)

    def to_c(self) -> DtConfig:
        if self.action_mode not in ACTION_MODES:
            raise ValueError('action_mode must be one of %s' % sorted(ACTION_MODES))
        c = DtConfig()
        c.road_tile_size = self.road_tile_size
        c.robot_speed = self.robot_speed
        c.wheel_dist = WHEEL_DIST
        c.delta_time = 1.0 / self.frame_rate
        c.robot_width = ROBOT_WIDTH
        c.robot_length = ROBOT_LENGTH
        c.camera_forward_dist = CAMERA_FORWARD_DIST
        c.accept_start_angle_deg = self.accept_start_angle_deg
        c.reset_safety = self.reset_safety
        c.reward_scale = self.reward_scale
        c.two_pi = 2 * math.pi
        c.rad2deg = 180.0 / math.pi
        c.max_steps = self.max_steps
        c.max_env_steps = self.max_env_steps
        c.max_spawn_attempts = self.max_spawn_attempts
        c.repeat_actions = self.repeat_actions
        c.frame_skip = self.frame_skip
        c.action_mode = ACTION_MODES[self.action_mode]
        c.clip_action = int(self.clip_action)
        c.reward_speed_measured = int(self.reward_speed_measured)
        c.front_probe_length = int(self.front_probe_length)
        c.auto_reset = int(self.auto_reset)
        c.safety_rad_mult = SAFETY_RAD_MULT
        return c

    def replace(self, **kw):
        d = {f.name: getattr(self, f.name) for f in fields(self)}
        d.update(kw)
        return EnvConfig(**d)
