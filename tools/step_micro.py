"""Diagnostic: shader cycles of one wave per call of each step-math piece
(-DDTSIM_STAMPS build, dt_diag_micro), on 64 envs' current poses."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd import _lib  # noqa: E402
from aido1_amd.vec_env import VecEnv  # noqa: E402

NAMES = ['lane_pos', 'valid_pose', 'sincos', 'bezier_closest', 'closest_curve', 'tile_of',
         'lane_pose_at', 'drivable', 'lane_pos_lean', 'valid_pose_lean', 'bezier_closest_fast',
         'tile_of_fast', 'closest_curve_fast', 'lane_pos_q', 'bezier_closest_q',
         'lane_pose_at<true>', 'valid_pose_q', 'lane_pose_at<false> (t varies)', 'sqrt chain',
         'div chain', '14 dep fp64 ops', 'tangent+sqrt+2div', 'bez_xz', 'acos']


def main():
    env = VecEnv(4096, seed=1234, device=0)
    env.reset()
    a = torch.rand(5, 4096, 2, device='cuda')
    for i in range(5):
        env.step_into(a[i])
    torch.cuda.synchronize()
    L = _lib.lib()
    L.dt_diag_micro.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    out = np.zeros(1, np.uint64)
    for w, nm in enumerate(NAMES):
        r = []
        for iters in (100, 200):
            L.dt_diag_micro(env._h, iters, w, out.ctypes.data_as(ctypes.c_void_p))
            r.append(int(out[0]))
        print('%-16s %7.1f cycles per call' % (nm, (r[1] - r[0]) / 100.0))


if __name__ == '__main__':
    main()
