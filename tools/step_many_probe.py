"""Decision throughput of dt_step_many for several k against HIP graphs of
dt_step (config 2: 4096 envs, loop_empty, U[0,1)^2 actions).

  python tools/step_many_probe.py [--decisions 480]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--decisions', type=int, default=480)
    p.add_argument('--ks', default='1,4,8,16,30,60,120')
    args = p.parse_args()
    import torch
    from aido1_amd.config import EnvConfig
    from aido1_amd.vec_env import StepOutput, VecEnv
    dev = torch.device('cuda', 0)
    n, D = 4096, args.decisions
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    acts = torch.rand(D + 30, n, 2, generator=g, device=dev)
    res = {}
    for k in [int(v) for v in args.ks.split(',')]:
        env = VecEnv(n, seed=1234, device=0, config=EnvConfig(map_name='loop_empty'))
        env.reset()
        out = StepOutput(k * n, dev, lanepos=False, tile=False)
        for i in range(30):
            env.step_into(acts[i])
        torch.cuda.synchronize()
        env.stats(reset=True)
        t0 = time.perf_counter()
        for c in range(D // k):
            env.step_many_into(acts[30 + c * k:30 + (c + 1) * k], out)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st = env.stats()
        env.check()
        res['many_k%d' % k] = dict(us_per_decision=dt / (D // k * k) * 1e6,
                                   env_steps_per_s=st['sim_steps'] / dt,
                                   resets_per_decision=st['resets'] / max(1, st['decisions']) * n)
        env.close()
    env = VecEnv(n, seed=1234, device=0, config=EnvConfig(map_name='loop_empty'))
    env.reset()
    out = StepOutput(n, dev, lanepos=False, tile=False)
    graphs = [env.capture(acts[30 + c * 30:30 + (c + 1) * 30], out) for c in range(D // 30)]
    torch.cuda.synchronize()
    env.stats(reset=True)
    t0 = time.perf_counter()
    for gr in graphs:
        gr.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = env.stats()
    env.check()
    res['graph30'] = dict(us_per_decision=dt / (D // 30 * 30) * 1e6,
                          env_steps_per_s=st['sim_steps'] / dt)
    print(json.dumps(res, indent=1), flush=True)


if __name__ == '__main__':
    main()
