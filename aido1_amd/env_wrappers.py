"""Batched mirror of the reference's environment-wrapper contract
(utils/env_wrappers.py): ``create_env(config, internal_env_args, transfer)``
and an EnvironmentWrapper with the same methods (step, reset, change_model,
collect_garbage, get_observation) whose arguments and results carry a leading
env dimension and live on the GPU.

EnvironmentWrapper.step (utils/env_wrappers.py:213-253) semantics kept:
  - tanh actor head (config.json:88): action/2 + 0.5 in float32 (in-kernel),
    and, as the reference's ``action /= 2; action += 0.5``, the caller's
    action array is left holding the mapped values (what the explorer then
    stores in its replay, explorers.py:209);
  - repeat_actions Simulator steps, break on done (per env);
  - reward = sum of raw rewards, reward_mod = sum of BaselineAggregation
    rewards x reward_scale;
  - done |= env_step > max_env_steps;
  - observation: the Transformer's 3-frame stack, oldest first
    (env_utils.py:54-70), of PreliminaryTransformer grey frames
    (env_utils.py:41-51) — or, with obs='lane', the (dist, angle_rad) lane pose.
Finished envs respawn inside the same launch (VectorEnv auto-reset); their
stack restarts with three copies of the first frame (Transformer.reset) and
``terminal`` in the info holds the lane pose they finished in.
``total_reward`` holds a finished env's episode return until its next step
(the reference's sum lives until reset(), env_wrappers.py:197,251).
"""
import torch

from aido1_amd.config import EnvConfig
from aido1_amd.render import RenderOutput
from aido1_amd.vec_env import VecEnv


def create_env(config, internal_env_args=None, transfer=False, **kw):
    """utils/env_wrappers.py:16-18 for the batched GPU environment."""
    if transfer:
        raise NotImplementedError('transfer (cut_off_leg) belongs to the prosthetics project')
    args = dict((internal_env_args or {}).get('env_init_args', {}))
    args.update(kw)
    env = EnvironmentWrapper(config, **args)
    seed = (internal_env_args or {}).get('env_config', {}).get('seed')
    if seed is not None:
        env.change_model(seed)
    return env


def map_tanh_in_place(action):
    """utils/env_wrappers.py:214-216 on the caller's array (float32 ops, the
    values the kernel used).  Stream-ordered after the step that read it."""
    if isinstance(action, torch.Tensor):
        action.div_(2).add_(0.5)
    else:
        action /= 2
        action += 0.5


class EnvironmentWrapper:
    def __init__(self, config, n_envs=4096, device=None, seed=123, map_name='loop_empty',
                 obs='render', env_id_base=0, **env_overrides):
        self.config = config
        ec = EnvConfig.from_reference_config(config, map_name=map_name, **env_overrides)
        self.env = VecEnv(n_envs, seed=seed, device=device, config=ec, env_id_base=env_id_base)
        self.n = n_envs
        self.obs_mode = obs
        self.render = RenderOutput(n_envs, self.env.device, slots=3) if obs == 'render' else None
        self.seed = None
        self.total_reward = torch.zeros(n_envs, dtype=torch.float64, device=self.env.device)
        self._restart = torch.zeros(n_envs, dtype=torch.bool, device=self.env.device)
        self.observation_transformed = None

    # ---- reference API -----------------------------------------------------------
    def change_model(self, seed):
        """Seed every env (utils/env_wrappers.py:208-211: only the first call counts)."""
        if self.seed is None:
            self.env.seed(seed)
            self.seed = seed

    def collect_garbage(self):
        """The reference re-creates its leaking OpenGL env every 128 episodes
        (explorers.py:107-108); nothing leaks here."""

    def reset(self):
        obs = self.env.reset()
        self.total_reward.zero_()
        self._restart.zero_()
        if self.render is not None:
            self.render.restart()
            self.env.render_into(self.render)
            obs = self.render.stack_view()
        self.observation_transformed = obs
        return obs

    def step(self, action):
        out = self.env.step_into(self._actions(action))
        if self.env.config.action_mode == 'tanh':
            map_tanh_in_place(action)
        if self.render is not None:
            self.env.render_into(self.render, fresh=out.done)
            obs = self.render.stack_view()
        else:
            obs = out.obs
        # the reference keeps total_reward until the next reset()
        # (utils/env_wrappers.py:197,251); a finished env's auto-reset is
        # that reset, so its sum restarts at the env's next step and the
        # finished episode's return stays readable until then
        self.total_reward.masked_fill_(self._restart, 0.0)
        self.total_reward += out.reward
        self._restart = out.done.bool()
        self.observation_transformed = obs
        info = {'terminal': out.lanepos, 'tile': out.tile}
        return obs, (out.reward, out.reward_mod), out.done.bool(), info

    def get_observation(self):
        return self.observation_transformed

    # ---- helpers -----------------------------------------------------------------
    def _actions(self, action):
        a = torch.as_tensor(action, dtype=torch.float32, device=self.env.device)
        return a.reshape(self.n, 2).contiguous()

    def ring(self):
        """(ring [n,3,120,160], oldest->newest slot order) for zero-copy consumers."""
        return self.render.ring, self.render.order()
