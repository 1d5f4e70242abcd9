"""Diagnostic: where a render_kernel workgroup spends its time (shader-clock
stamps of the -DDTSIM_STAMPS build, tools/step_stamps.sh; run with
DTSIM_DIAG_LIB=aido1_amd/libdtsim_stamps.so).  Thread 0 of every workgroup
stamps after each phase's barrier: 4 entry, 5 prologue (palette, tiles, view),
6 background, 7 markings, 8 uniformity + grey stores, 9 Sobel, 10 NMS,
11 hysteresis, 13 masks; [0]/[1] real time at entry/exit, [2] HW_ID,
[3] XCC_ID, [12] nlist | nweak << 32."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd import _lib  # noqa: E402
from aido1_amd.config import EnvConfig  # noqa: E402
from aido1_amd.render import RenderOutput  # noqa: E402
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402


def main():
    n = int(os.environ.get('ENVS', '4096'))
    dev = torch.device('cuda', 0)
    env = VecEnv(n, seed=1234, device=0, config=EnvConfig(map_name=os.environ.get('MAP', 'loop_empty')))
    out = StepOutput(n, dev, lanepos=False, tile=False)
    ro = RenderOutput(n, dev)
    env.reset()
    L = _lib.lib()
    L.dt_diag_renstamps.argtypes = [ctypes.c_void_p]
    buf = np.zeros((4096, 24), np.uint64)
    recs = []
    acts = torch.rand(40, n, 2, device=dev)
    for it in range(40):
        env.step_into(acts[it], out)
        env.render_into(ro, fresh=out.done)
        torch.cuda.synchronize()
        if it < 10:
            continue
        L.dt_diag_renstamps(buf.ctypes.data_as(ctypes.c_void_p))
        recs.append(buf[:min(n, 4096)].astype(np.int64).copy())
    b = np.stack(recs)                     # [launch, wg, 16]
    real = (b[..., 1] - b[..., 0]) / 100.0  # us (100 MHz real-time clock)
    cyc = b[..., 13] - b[..., 4]
    clk = np.median(cyc / (real * 1e3))
    names = ['prologue', 'background', 'markings', 'uniform+grey', 'sobel', 'nms', 'hysteresis',
             'masks']
    pts = [4, 5, 6, 7, 8, 9, 10, 11, 13]
    seg = np.stack([b[..., pts[i + 1]] - b[..., pts[i]] for i in range(len(names))], -1)
    print('launches %d, workgroups %d; workgroup life median %.2f us (p10 %.2f, p90 %.2f); '
          'shader clock %.2f GHz' % (b.shape[0], b.shape[1], np.median(real),
                                     np.percentile(real, 10), np.percentile(real, 90), clk))
    tot = np.median(seg.sum(-1))
    for i, nm in enumerate(names):
        print('  %-13s median %7.0f cyc  mean %7.0f  p90 %7.0f  (%4.1f %% of the median life)'
              % (nm, np.median(seg[..., i]), seg[..., i].mean(), np.percentile(seg[..., i], 90),
                 100 * np.median(seg[..., i]) / tot))
    wpush = b[..., 14] - b[..., 6]
    print('  markings split: to the lists ready %.0f cyc, drawing %.0f cyc; visible '
          'segments median %d (p90 %d)' % (np.median(wpush), np.median(b[..., 7] - b[..., 14]),
                                          np.median(b[..., 15]), np.percentile(b[..., 15], 90)))
    print('  wave 0 in the markings: projection %.0f, list slots %.0f, records + barrier %.0f, '
          'yellow draw %.0f, white draw %.0f cyc' % (
              np.median(b[..., 16] - b[..., 6]), np.median(b[..., 17] - b[..., 16]),
              np.median(b[..., 14] - b[..., 17]), np.median(b[..., 18] - b[..., 14]),
              np.median(b[..., 7] - b[..., 18])))
    nl = b[..., 12] & 0xFFFFFFFF
    nw = b[..., 12] >> 32
    print('  nlist median %d (p90 %d, max %d) of 4800 words; nweak median %d max %d'
          % (np.median(nl), np.percentile(nl, 90), nl.max(), np.median(nw), nw.max()))
    # launch span and concurrency
    last = b[-1]
    t0 = last[:, 0].min()
    span = (last[:, 1].max() - t0) / 100.0
    hw = last[:, 2]
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = last[:, 3] & 0xF
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    ev = np.concatenate([np.stack([last[:, 0], np.ones(len(last))], 1),
                         np.stack([last[:, 1], -np.ones(len(last))], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    print('last launch: span %.1f us, distinct CUs %d, workgroups per CU %.1f, max concurrent '
          'workgroups %d (%.2f per CU)' % (span, len(np.unique(key)), len(last) / len(np.unique(key)),
                                           conc.max(), conc.max() / len(np.unique(key))))
    env.close()


if __name__ == '__main__':
    main()
