"""aido1_amd — MI355X-native batched Duckietown lane-following environment.

The hot path of niksaz/aido1 (gym-duckietown Simulator.step/reset behind
duckietown_rl/env.py:launch_env and utils/env_wrappers.py:EnvironmentWrapper)
as gfx950 HIP kernels behind a C ABI (include/dtsim.h, libdtsim.so), driven
from Python via ctypes.  See DESIGN.md.
"""
__version__ = '0.1.0'
