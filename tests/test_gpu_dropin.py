"""The drop-in surfaces on the GPU: the gym-shaped Simulator behind launch_env
(duckietown_rl/env.py:4-20) and the batched EnvironmentWrapper mirror
(utils/env_wrappers.py:137-263), checked against the oracle."""
import math

import numpy as np
import pytest
import torch

from conftest import golden, map_rows
from oracle import dtsim_ref as R

pytestmark = pytest.mark.gpu


def test_launch_env_simulator_matches_oracle(gpu):
    from aido1_amd.env import launch_env
    env = launch_env()
    assert env.observation_space.shape == (120, 160, 3)
    assert env.action_space.shape == (2,) and env.action_space.high[0] == 1.0
    obs = env.reset()
    assert obs.shape == (120, 160, 3) and obs.dtype == np.uint8
    sim = R.SimulatorRef(map_rows('loop_empty'), seed=123, env_id=0,
                         cfg=R.SimConfig(max_env_steps=2**32 - 1, repeat_actions=1))
    sim.reset()
    assert np.allclose(env.cur_pos, sim.cur_pos, atol=0, rtol=0)
    assert env.cur_angle == sim.cur_angle
    rng = np.random.default_rng(0)
    for t in range(200):
        a = rng.uniform(0, 1, 2)
        obs, r, d, info = env.step(a)
        _, rr, dd, _ = sim.step(a.astype(np.float32).astype(np.float64))
        assert d == dd and abs(r - rr) <= 1e-9
        assert abs(env.cur_angle - sim.cur_angle) <= 1e-9
        assert np.max(np.abs(env.cur_pos - sim.cur_pos)) <= 1e-9
        assert obs.shape == (120, 160, 3)
        if d:
            assert info['Simulator']['msg']
            env.reset()
            sim.reset()
    lp = env.get_lane_pos2()
    assert -1.0 <= lp.dot_dir <= 1.0


def test_simulator_with_reference_wrapper_stack(gpu):
    """duckietown_rl/wrappers.py's stack semantics on the drop-in: steering
    action through the ×0.8-left-wheel quirk (golden vectors)."""
    from aido1_amd.env import launch_env
    env = launch_env()
    env.reset()
    fx = [c for c in golden('steering.json') if 'action' in c][:20]
    s0 = env.cur_pos.copy()
    for c in fx:
        wheels = np.array(c['sim_action'])
        env.step(wheels)
    assert not np.allclose(env.cur_pos, s0)


def test_env_wrappers_batched(gpu):
    from aido1_amd.env_wrappers import create_env
    cfg = golden('reference_config.json')
    env = create_env(cfg, {'env_init_args': {'n_envs': 256, 'device': 0},
                           'env_config': {'seed': 42}})
    obs = env.reset()
    assert obs.shape == (256, 3, 120, 160) and obs.dtype == torch.float32
    assert torch.equal(obs[:, 0], obs[:, 2])            # reset: three copies
    rng = np.random.default_rng(1)
    prev_newest = obs[:, 2].clone()
    for t in range(20):
        a = torch.from_numpy(rng.uniform(-1, 1, (256, 2)).astype(np.float32))
        a0 = a.clone()
        obs, (r, rm), done, info = env.step(a)
        assert torch.equal(a, a0 / 2 + 0.5)             # env_wrappers.py:214-216, in place
        keep = ~done
        # the previous newest frame is now the middle one (Transformer shift)
        assert torch.equal(obs[keep, 1], prev_newest[keep])
        if done.any():
            d = done
            assert torch.equal(obs[d, 0], obs[d, 2])    # respawned: stack refilled
        prev_newest = obs[:, 2].clone()
        assert torch.isfinite(r).all() and torch.isfinite(rm).all()
