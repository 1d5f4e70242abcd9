"""Diagnostic: where a step_pair_kernel decision spends its time, from the
shader-clock stamps of a -DDTSIM_STAMPS build (tools/step_stamps.sh builds
aido1_amd/libdtsim_stamps.so; run with DTSIM_DIAG_LIB pointing at it).
Per decision d < 8, lane 0 of both waves (role 0 = _valid_pose, role 1 =
get_lane_pos2) of the first 64 blocks: 0 start, per sim step r: 1+3r pose
updated, 2+3r role work done (before the exchange barrier), 3+3r past the
barrier; 10 sim_decision returned, 11 decision end (spawn, stores).  Point 15:
real time (100 MHz) at entry/exit and shader clock at entry/exit, giving the
shader clock rate."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd import _lib  # noqa: E402
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402


def main():
    n = int(os.environ.get('ENVS', '4096'))
    k = int(os.environ.get('K', '20'))
    dev = torch.device('cuda', 0)
    env = VecEnv(n, seed=1234, device=0)
    acts = torch.rand(20 * k, n, 2, device=dev)
    out = StepOutput(k * n, dev, lanepos=False, tile=False)
    env.reset()
    L = _lib.lib()
    L.dt_diag_pstamps.argtypes = [ctypes.c_void_p]
    buf = np.zeros((64, 2, 8, 16), np.uint64)
    nb = min(64, (n + 63) // 64)
    recs = []
    for it in range(20):
        env.step_many_into(acts[it * k:(it + 1) * k], out)
        torch.cuda.synchronize()
        if it < 5:
            continue
        L.dt_diag_pstamps(buf.ctypes.data_as(ctypes.c_void_p))
        recs.append(buf[:nb].astype(np.int64).copy())
    b = np.stack(recs)          # [launch, block, role, dec, 16]
    real = (b[:, :, 0, 1, 15] - b[:, :, 0, 0, 15]) / 100e6
    cyc = b[:, :, 0, 2, 15] - b[:, :, 0, 3, 15]
    clk = np.median(cyc / real) / 1e9
    print('launches %d, blocks %d, k %d; kernel body median %.2f us; shader clock %.3f GHz'
          % (b.shape[0], nb, k, np.median(real) * 1e6, clk))
    names = ['pose 1', 'work 1', 'barrier 1', 'pose 2', 'work 2', 'barrier 2', 'pose 3', 'work 3',
             'barrier 3', 'decision tail', 'spawn+stores']
    for role in (0, 1):
        d = b[:, :, role, 1:8, :]   # decisions 1..7 (0 pays the map staging)
        seg = np.diff(d[..., 0:12], axis=-1)
        print('role %d (cycles, median over launches x blocks x decisions 1-7):' % role)
        for i, nm in enumerate(names):
            print('   %-14s %7.0f  (p90 %7.0f)' % (nm, np.median(seg[..., i]),
                                                  np.percentile(seg[..., i], 90)))
        tot = d[..., 11] - d[..., 0]
        print('   %-14s %7.0f  (p90 %7.0f) = %.2f us' % ('decision', np.median(tot),
                                                        np.percentile(tot, 90),
                                                        np.median(tot) / clk / 1e3))
    for role in (0, 1):
        d = b[:, :, role, 1:8, :]
        print('role %d rep 2: barrier 1 -> top of rep %.0f, top -> before sincos %.0f, sincos %.0f, '
              'after sincos -> pose stamp %.0f' % (
                  role, np.median(d[..., 12] - d[..., 3]), np.median(d[..., 13] - d[..., 12]),
                  np.median(d[..., 14] - d[..., 13]), np.median(d[..., 4] - d[..., 14])))
    # decision to decision, including any gap
    dd = np.diff(b[:, :, 0, :8, 0], axis=-1)
    print('decision start to start (role 0): median %.0f cycles' % np.median(dd))


if __name__ == '__main__':
    main()
