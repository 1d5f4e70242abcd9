"""Diagnostic: where a dt_step launch spends its time, from shader-clock stamps
of a -DDTSIM_STAMPS build (tools/step_stamps.sh builds
aido1_amd/libdtsim_stamps.so; run with DTSIM_DIAG_LIB pointing at it).
Stamps (wave 0 of each step block): 0 entry, 1 map staged, 2 state loaded,
3-5 after each sim step, 6 terminal lane pose, 7 before the counters,
8 after the stores; 9/10 entry/exit on the 100 MHz real-time clock."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd import _lib  # noqa: E402
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402

NAMES = ['map staged', 'state loaded', 'sim step 1', 'sim step 2', 'sim step 3',
         'terminal lane pose', 'to counters', 'counters+stores']


def main():
    n = 4096
    dev = torch.device('cuda', 0)
    env = VecEnv(n, seed=1234, device=0)
    out = StepOutput(n, dev, lanepos=False, tile=False)
    acts = torch.rand(60, n, 2, device=dev)
    env.reset()
    for i in range(40):
        env.step_into(acts[i], out)
    L = _lib.lib()
    L.dt_diag_stamps.argtypes = [ctypes.c_void_p]
    buf = np.zeros((64, 16), np.uint64)
    nb = (n + 255) // 256
    deltas, real, stamps_mid = [], [], []
    L.dt_diag_rstamps.argtypes = [ctypes.c_void_p]
    rbuf = np.zeros((4096, 4), np.uint64)
    nr = (n + 7) // 8   # refill groups of kRefillEnvs = 8
    rinfo = []
    prev_exit = None
    sg = env.capture(acts[40:60], out)
    for k in range(20):
        # one launch at a time so that the stamps are this launch's
        env.step_into(acts[40 + k], out)
        torch.cuda.synchronize()
        L.dt_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p))
        b = buf[:nb].astype(np.int64)
        deltas.append(np.diff(b[:, 0:9], axis=1))
        stamps_mid.append(b.copy())
        L.dt_diag_rstamps(rbuf.ctypes.data_as(ctypes.c_void_p))
        r = rbuf[:nr].astype(np.int64)
        t0 = min(b[:, 9].min(), r[:, 0].min())
        busy = r[:, 2] > 0
        rinfo.append(((b[:, 10].max() - t0) / 100.0, (r[:, 1].max() - t0) / 100.0,
                      (r[:, 0].max() - t0) / 100.0, busy.sum(), r[:, 2].max(),
                      np.median((r[busy, 1] - r[busy, 0])) / 100.0 if busy.any() else 0,
                      ((r[busy, 1] - r[busy, 0]).max()) / 100.0 if busy.any() else 0))
        real.append((b[:, 10] - b[:, 9]) * 10.0)   # ns
    d = np.concatenate(deltas)
    bb = np.concatenate([x for x in stamps_mid])
    print('inside sim step 2 (cycles, median): pose update %.0f, valid_pose %.0f, lane_pos %.0f' % (
        np.median(bb[:, 11] - bb[:, 3]), np.median(bb[:, 12] - bb[:, 11]),
        np.median(bb[:, 13] - bb[:, 12])))
    print('per wave-0 of %d step blocks, 20 launches: cycles (median / max over blocks)' % nb)
    for i, nm in enumerate(NAMES):
        print('  %-20s %8.0f %8.0f' % (nm, np.median(d[:, i]), np.max(d[:, i])))
    print('  total cycles       %8.0f' % np.median(d.sum(1)))
    ri = np.array(rinfo)
    print('launch timeline (us from first block entry, median of 20): step blocks done %.2f, '
          'refill blocks done %.2f, last refill block entered %.2f; busy refill blocks %.0f, '
          'max items %.0f; busy block duration median %.2f max %.2f' % tuple(np.median(ri, 0)))
    r = np.concatenate(real)
    print('  entry->exit real time: median %.2f us, max %.2f us' % (np.median(r) / 1e3,
                                                                  np.max(r) / 1e3))
    # inside a graph: spread of block entry times and gap between launches
    sg.replay()
    torch.cuda.synchronize()
    L.dt_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p))
    b = buf[:nb].astype(np.int64)
    print('  last graph launch: block entry spread %.2f us, exit spread %.2f us' % (
        (b[:, 9].max() - b[:, 9].min()) / 100.0, (b[:, 10].max() - b[:, 10].min()) / 100.0))


if __name__ == '__main__':
    main()
