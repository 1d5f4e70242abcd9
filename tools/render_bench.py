"""Diagnostic: render_kernel on realistic inputs with no host in the way.

Records K decisions of a config-3 rollout first (pose snapshots via
dt_copy_pose and the done flags of every step), then times K back-to-back
dt_render launches over those snapshots with fresh = that decision's done
flags, the way bench.py's loop feeds the kernel.  Prints the mean kernel time
from HIP events, the same with fresh disabled, and the host's enqueue time of
bench.py's ObsLoop (a host-bound loop would show enqueue ~= wall)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.config import EnvConfig  # noqa: E402
from aido1_amd.render import RenderOutput  # noqa: E402
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402


def timed(fn, k):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(k)]
    for i, (a, b) in enumerate(ev):
        a.record()
        fn(i)
        b.record()
    torch.cuda.synchronize()
    return np.array([a.elapsed_time(b) for a, b in ev])


def main():
    n = int(os.environ.get('ENVS', '4096'))
    K = int(os.environ.get('K', '40'))
    dev = torch.device('cuda', 0)
    env = VecEnv(n, seed=1234, device=0, config=EnvConfig(map_name=os.environ.get('MAP', 'loop_empty')))
    env.reset()
    acts = torch.rand(K + 10, n, 2, device=dev)
    outs = [StepOutput(n, dev, lanepos=False, tile=False) for _ in range(K + 10)]
    poses = [torch.empty(3, n, dtype=torch.float64, device=dev) for _ in range(K + 10)]
    for d in range(K + 10):
        env.step_into(acts[d], outs[d])
        env.copy_pose(poses[d])
    torch.cuda.synchronize()
    ro = RenderOutput(n, dev)
    for d in range(10):
        env.render_into(ro, fresh=outs[d].done, pose=poses[d])
    torch.cuda.synchronize()
    fr = float(np.mean([o.done.float().mean().item() for o in outs[10:]]))
    ms = timed(lambda i: env.render_into(ro, fresh=outs[10 + i].done, pose=poses[10 + i]), K)
    ms0 = timed(lambda i: env.render_into(ro, pose=poses[10 + i]), K)
    ms1 = timed(lambda i: env.render_into(ro, pose=poses[10]), K)
    byt = 153624 * n
    print('render, %d envs, %d recorded decisions (fresh %.1f %%):' % (n, K, 100 * fr))
    for name, m in (('fresh = done', ms), ('no fresh', ms0), ('one pose, no fresh', ms1)):
        print('  %-20s mean %.4f ms  min %.4f  max %.4f  -> %.1f %% of 8 TB/s (single-slot bytes)'
              % (name, m.mean(), m.min(), m.max(), 100 * byt / (m.mean() * 1e-3) / 8e12))
    # host enqueue rate of bench.py's loop
    import bench
    big = StepOutput(K * n, dev, lanepos=False, tile=False)
    for mode in ('many', 'serial', 'pipe'):
        loop = bench.ObsLoop(env, ro, torch, mode)
        ev = loop.events(K)
        calls = loop.bind(acts[10:10 + K], big)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.run(calls, ev)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print('  ObsLoop %-6s host enqueue %.1f us/decision, wall %.1f us/decision'
              % (mode, (t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6))
    env.close()


if __name__ == '__main__':
    main()
