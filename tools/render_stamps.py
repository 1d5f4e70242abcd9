"""Diagnostic: where a render_kernel workgroup spends its time (shader-clock
stamps of the -DDTSIM_STAMPS build, tools/step_stamps.sh; run with
DTSIM_DIAG_LIB=aido1_amd/libdtsim_stamps.so).  Thread 0 of every workgroup
stamps after each phase's barrier: 16 kernel entry (17 its real time), 4 after the
prologue (palette, tiles, view), 5 background spans + segment
projection, 6 span fix-up + markings, 8 uniformity + grey + uniform masks,
9 Sobel, 10 NMS, 11/13 hysteresis, 14 outputs (grey + masks); [0]/[1] real time at
entry/exit, [2] HW_ID, [3] XCC_ID, [12] nlist | nweak << 32, [15] visible
segments (yellow | white << 16).
With TIME_ONLY=1 (production library): mean dt_render time of 4096 envs
alone, back to back, from HIP events."""
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


def time_only(n):
    dev = torch.device('cuda', 0)
    env = VecEnv(n, seed=1234, device=0, config=EnvConfig(map_name=os.environ.get('MAP', 'loop_empty')))
    out = StepOutput(n, dev, lanepos=False, tile=False)
    ro = RenderOutput(n, dev)
    env.reset()
    acts = torch.rand(30, n, 2, device=dev)
    for it in range(10):
        env.step_into(acts[it], out)
        env.render_into(ro, fresh=out.done)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(20)]
    for a, b in ev:
        a.record()
        env.render_into(ro)
        b.record()
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ev]
    print('render alone, %d envs: mean %.4f ms, min %.4f ms -> %.1f %% of 8 TB/s'
          % (n, np.mean(ms), np.min(ms), 100 * 153624 * n / (np.mean(ms) * 1e-3) / 8e12))
    env.close()


def main():
    n = int(os.environ.get('ENVS', '4096'))
    if os.environ.get('TIME_ONLY'):
        return time_only(n)
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
    real = (b[..., 1] - b[..., 17]) / 100.0  # us (100 MHz real-time clock), from kernel entry
    cyc = b[..., 14] - b[..., 16]
    clk = np.median(cyc / (real * 1e3))
    names = ['prologue', 'spans+proj', 'fixup+marks', 'uniformity', 'sobel', 'nms',
             'hysteresis', 'output']
    pts = [16, 4, 5, 6, 8, 9, 10, 13, 14]
    seg = np.stack([b[..., pts[i + 1]] - b[..., pts[i]] for i in range(len(names))], -1)
    print('launches %d, workgroups %d; workgroup life median %.2f us (p10 %.2f, p90 %.2f); '
          'shader clock %.2f GHz' % (b.shape[0], b.shape[1], np.median(real),
                                     np.percentile(real, 10), np.percentile(real, 90), clk))
    tot = np.median(seg.sum(-1))
    for i, nm in enumerate(names):
        print('  %-13s median %7.0f cyc  mean %7.0f  p90 %7.0f  (%4.1f %% of the median life)'
              % (nm, np.median(seg[..., i]), seg[..., i].mean(), np.percentile(seg[..., i], 90),
                 100 * np.median(seg[..., i]) / tot))
    print('  spans+proj split: spans %.0f, projection + lists %.0f cyc (medians)'
          % (np.median(b[..., 18] - b[..., 4]), np.median(b[..., 5] - b[..., 18])))
    segs = b[..., 15] & 0xFFFFFFFF
    vis = (segs & 0xFFFF) + (segs >> 16)
    print('  visible segments median %d (p90 %d)' % (np.median(vis), np.percentile(vis, 90)))
    nl = b[..., 12] & 0xFFFFFFFF
    nw = b[..., 12] >> 32
    print('  nlist median %d (p90 %d, max %d) of 4800 words; nweak median %d max %d'
          % (np.median(nl), np.percentile(nl, 90), nl.max(), np.median(nw), nw.max()))
    # launch span and concurrency
    last = b[-1]
    t0 = last[:, 17].min()
    span = (last[:, 1].max() - t0) / 100.0
    hw = last[:, 2]
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = last[:, 3] & 0xF
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    ev = np.concatenate([np.stack([last[:, 17], np.ones(len(last))], 1),
                         np.stack([last[:, 1], -np.ones(len(last))], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    print('last launch: span %.1f us, distinct CUs %d, workgroups per CU %.1f, max concurrent '
          'workgroups %d (%.2f per CU)' % (span, len(np.unique(key)), len(last) / len(np.unique(key)),
                                           conc.max(), conc.max() / len(np.unique(key))))
    # per-CU timelines of the last launch: when each CU's first workgroup
    # starts and its last ends, how many of its slots are busy on average over
    # that span, and the gap from a workgroup's end to the next start on the CU
    t_start = (last[:, 17] - t0) / 100.0
    t_end = (last[:, 1] - t0) / 100.0
    firsts, lasts, occ, gaps = [], [], [], []
    for k in np.unique(key):
        sel = key == k
        st, en = np.sort(t_start[sel]), np.sort(t_end[sel])
        firsts.append(st[0])
        lasts.append(en[-1])
        occ.append((en - st).sum() if False else (t_end[sel] - t_start[sel]).sum() / (en[-1] - st[0]))
        # each start after the first 4 follows some end: the latest end before it
        for s0 in st[4:]:
            prev = en[en <= s0 + 1e-9]
            if len(prev):
                gaps.append(s0 - prev[-1])
    firsts, lasts, occ = np.array(firsts), np.array(lasts), np.array(occ)
    print('per CU: first start median %.1f us (max %.1f), last end median %.1f us (min %.1f, '
          'max %.1f), busy slots over its span mean %.2f' % (np.median(firsts), firsts.max(),
                                                              np.median(lasts), lasts.min(),
                                                              lasts.max(), occ.mean()))
    if gaps:
        g = np.array(gaps)
        print('end -> next start on a CU: median %.2f us, p90 %.2f us, max %.2f us'
              % (np.median(g), np.percentile(g, 90), g.max()))
    # the waves' ends: thread 0's [1] against waves 1, 3, 5, 7 ([19..22])
    wend = b[..., 19:23]
    ok = (wend > 0).all(-1)
    if ok.any():
        lastw = np.maximum(wend.max(-1), b[..., 1])[ok]
        print('wave ends after thread 0\'s: median %.2f us, p90 %.2f us; the last wave is '
              'wave 0 in %.0f %% of the workgroups'
              % (np.median((lastw - b[..., 1][ok]) / 100.0),
                 np.percentile((lastw - b[..., 1][ok]) / 100.0, 90),
                 100 * np.mean(b[..., 1][ok] >= wend.max(-1)[ok])))
    hist = np.histogram(t_start, bins=10, range=(0, span))[0]
    print('workgroup starts per tenth of the span:', hist.tolist())
    env.close()


if __name__ == '__main__':
    main()
