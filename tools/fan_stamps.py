"""Diagnostic: where a step_fan_kernel decision spends its time (shader-clock
stamps of the -DDTSIM_STAMPS build, tools/step_stamps.sh; run with
DTSIM_DIAG_LIB pointing at aido1_amd/libdtsim_stamps.so).  Per decision d < 8,
lane 0 of each of the 4 waves of the first 64 blocks: 0 start (slot loads
issued), 1 pose chain done, 2 step math done (before the barrier), 3 past the
barrier, 4 reward chain done, 5 decision end (spawn, stores)."""
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
    buf = np.zeros((64, 4, 8, 16), np.uint64)
    nb = min(64, (n + 15) // 16)
    recs = []
    L.dt_diag_bstamps.argtypes = [ctypes.c_void_p]
    bst = np.zeros((4096, 4), np.uint64)
    nstep = (n + 15) // 16
    nref = (n + 7) // 8
    blk = []
    for it in range(20):
        env.step_many_into(acts[it * k:(it + 1) * k], out)
        torch.cuda.synchronize()
        if it < 5:
            continue
        L.dt_diag_pstamps(buf.ctypes.data_as(ctypes.c_void_p))
        recs.append(buf[:nb].astype(np.int64).copy())
        L.dt_diag_bstamps(bst.ctypes.data_as(ctypes.c_void_p))
        blk.append(bst[:nstep + nref].astype(np.int64).copy())
    b = np.stack(recs)          # [launch, block, wave, dec, 16]
    real = (b[:, :, 0, 1, 15] - b[:, :, 0, 0, 15]) / 100e6
    cyc = b[:, :, 0, 2, 15] - b[:, :, 0, 3, 15]
    clk = np.median(cyc / real) / 1e9
    print('launches %d, blocks %d, k %d; kernel body median %.2f us; shader clock %.3f GHz'
          % (b.shape[0], nb, k, np.median(real) * 1e6, clk))
    names = ['pose chain', 'step math', 'barrier', 'reward chain', 'spawn+stores']
    for w in range(4):
        d = b[:, :, w, 1:8, :]
        seg = np.diff(d[..., 0:6], axis=-1)
        print('wave %d (cycles, median / p90 over launches x blocks x decisions 1-7):' % w)
        for i, nm in enumerate(names):
            print('   %-14s %7.0f  %7.0f' % (nm, np.median(seg[..., i]), np.percentile(seg[..., i], 90)))
        nxt = np.diff(b[:, :, w, 1:8, 0], axis=-1)
        print('   %-14s %7.0f  (start to start %.0f) = %.2f us' % (
            'decision', np.median(d[..., 5] - d[..., 0]), np.median(nxt), np.median(nxt) / clk / 1e3))


    bb = blk[-1]
    t0 = bb[:, 0].min()
    st_ = bb[:nstep]
    rf = bb[nstep:]
    dur = (st_[:, 1] - st_[:, 0]) / 100.0
    print('step blocks: entry spread %.2f us, duration median %.2f min %.2f max %.2f us; '
          'last exit %.2f us' % ((st_[:, 0].max() - t0) / 100.0, np.median(dur), dur.min(),
                                 dur.max(), (st_[:, 1].max() - t0) / 100.0))
    print('refill blocks: entry first %.2f last %.2f us, exit last %.2f us, duration median %.2f max %.2f'
          % ((rf[:, 0].min() - t0) / 100.0, (rf[:, 0].max() - t0) / 100.0,
             (rf[:, 1].max() - t0) / 100.0, np.median(rf[:, 1] - rf[:, 0]) / 100.0,
             (rf[:, 1] - rf[:, 0]).max() / 100.0))
    hw = st_[:, 2]
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = st_[:, 3] & 0xF
    ids = xcc * 1000 + se * 100 + sh * 16 + cu
    u, cnt = np.unique(ids, return_counts=True)
    print('step blocks on %d distinct CUs; blocks per CU histogram %s' % (
        len(u), dict(zip(*np.unique(cnt, return_counts=True)))))
    slow = dur > 1.5 * np.median(dur)
    print('slow step blocks (>1.5x median): %d; of those sharing a CU with another step block: %d'
          % (slow.sum(), sum(1 for i in np.where(slow)[0] if cnt[np.searchsorted(u, ids[i])] > 1)))
    order = np.argsort(st_[:, 0])
    print('first 16 step blocks by entry: id, start us, dur us, xcc, se, cu:')
    for i in order[:8]:
        print('  ', i, (st_[i, 0] - t0) / 100.0, dur[i], xcc[i], se[i], cu[i])
    print('durations by block id (every 16th):', np.round(dur[::16], 1).tolist())


if __name__ == '__main__':
    main()
