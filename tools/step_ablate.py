"""Diagnostic: dt_step launch time (HIP events, mean of 200 launches) under
config variants, to split the step kernel's time into its parts.
Run on the GPU box: python tools/step_ablate.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.config import EnvConfig  # noqa: E402
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402


def run(name, n=4096, steps=200, warm=20, straight=False, graph=0, **kw):
    dev = torch.device('cuda', 0)
    env = VecEnv(n, seed=1234, device=0, config=EnvConfig(**kw))
    out = StepOutput(n, dev, lanepos=False, tile=False)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    acts = torch.rand(warm + steps, n, 2, generator=g, device=dev)
    if straight:
        acts[..., 1] = acts[..., 0]
    env.reset()
    for i in range(warm):
        env.step_into(acts[i], out)
    torch.cuda.synchronize()
    if graph:
        sg = env.capture(acts[warm:warm + graph], out)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps // graph)]
        for e0, e1 in ev:
            e0.record()
            sg.replay()
            e1.record()
        torch.cuda.synchronize()
        ts = sorted(a.elapsed_time(b) * 1e3 / graph for a, b in ev)
    else:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        for k in range(steps):
            ev[k][0].record()
            env.step_into(acts[warm + k], out)
            ev[k][1].record()
        torch.cuda.synchronize()
        ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    print('%-34s mean %7.2f us  median %7.2f us  min %7.2f' % (
        name, sum(ts) / len(ts), ts[len(ts) // 2], ts[0]), flush=True)
    env.close()


def empty_kernel():
    x = torch.zeros(64, device='cuda')
    for _ in range(20):
        x.add_(1.0)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(200)]
    for e0, e1 in ev:
        e0.record()
        x.add_(1.0)
        e1.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    print('%-34s median %7.2f us' % ('tiny torch kernel (event floor)', ts[len(ts) // 2]))


if __name__ == '__main__':
    empty_kernel()
    run('default')
    run('default, graph of 20', graph=20)
    run('no auto-reset, graph of 20', graph=20, auto_reset=False)
    run('repeat 1, no auto-reset, graph 20', graph=20, repeat_actions=1, auto_reset=False)
    run('no auto-reset', auto_reset=False)
    run('repeat 1', repeat_actions=1)
    run('repeat 1, no auto-reset', repeat_actions=1, auto_reset=False)
    run('straight actions', straight=True)
    run('64 envs', n=64)
    run('64 envs, no auto-reset', n=64, auto_reset=False)
    run('64 envs, repeat 1, no auto-reset', n=64, repeat_actions=1, auto_reset=False)
    run('1024 envs', n=1024)
    run('16384 envs', n=16384)
