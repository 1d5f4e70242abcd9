"""launch_env — drop-in for duckietown_rl/env.py:4-20.

The reference builds one gym-duckietown Simulator per process; this returns the
libdtsim-backed Simulator view built from the same constructor arguments, so
DuckietownEnvironmentWrapper (utils/env_wrappers.py:103-134),
train-ddpg-cnn.py and test-ddpg-cnn.py run on it unchanged once their import
points here.  Batched consumers use aido1_amd.vec_env.VecEnv.
"""
from aido1_amd.simulator import Simulator

# duckietown_rl/env.py:7-17 — the reference's Simulator arguments
REFERENCE_SIMULATOR_KWARGS = dict(
    seed=123, map_name='loop_empty', max_steps=500001, domain_rand=0, camera_width=640,
    camera_height=480, accept_start_angle_deg=4, full_transparency=True, distortion=True)


def launch_env(id=None, device=None, **overrides):
    if id is not None:
        raise NotImplementedError('gym.make(%r): only the Duckietown Simulator is provided' % id)
    kw = dict(REFERENCE_SIMULATOR_KWARGS)
    kw.update(overrides)
    return Simulator(device=device, **kw)
