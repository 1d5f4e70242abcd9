"""Diagnostic: fixed cost around one timed config-2 launch (K decisions): wall
time of graph replay + synchronize vs an eager dt_step_many + synchronize vs
synchronize alone, and the HIP-event time of the kernel, medians of 30."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402


def main():
    n, K = 4096, int(os.environ.get('K', '20'))
    dev = torch.device('cuda', 0)
    env = VecEnv(n, seed=1234, device=0)
    acts = torch.rand(K, n, 2, device=dev)
    out = StepOutput(K * n, dev, lanepos=False, tile=False)
    env.reset()
    for _ in range(5):
        env.step_many_into(acts, out)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        env.step_many_into(acts, out)
    torch.cuda.synchronize()
    res = {'graph': [], 'eager': [], 'sync_only': [], 'graph_events': [], 'eager_events': [],
           'graph_call': [], 'eager_call': []}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(30):
        for mode in ('graph', 'eager'):
            torch.cuda.synchronize()
            time.sleep(0.002)
            t0 = time.perf_counter()
            e0.record()
            if mode == 'graph':
                g.replay()
            else:
                env.step_many_into(acts, out)
            t1 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            res[mode].append((t2 - t0) * 1e6)
            res[mode + '_call'].append((t1 - t0) * 1e6)
            res[mode + '_events'].append(e0.elapsed_time(e1) * 1e3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        res['sync_only'].append((time.perf_counter() - t0) * 1e6)
    for k, v in res.items():
        print('%-14s median %8.1f us  min %8.1f' % (k, np.median(v), np.min(v)))
    # back to back: 10 launches then one sync
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        env.step_many_into(acts, out)
    torch.cuda.synchronize()
    print('10 eager launches back to back: %.1f us each' % ((time.perf_counter() - t0) * 1e5))


if __name__ == '__main__':
    main()
