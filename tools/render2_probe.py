"""Diagnostic: config 3's renders one decision a launch (dt_render) against two
decisions a launch (dt_render2), 4096 envs on loop_empty, the poses and done
flags of dt_step_many chunks of 20 decisions; HIP events around each chunk's
renders.  Prints ms per decision for both forms (alternating, R rounds)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.config import EnvConfig  # noqa: E402
from aido1_amd.render import RenderOutput, bind_render, bind_render2  # noqa: E402
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402

n, k, R = 4096, 20, int(os.environ.get('R', '5'))
dev = torch.device('cuda', 0)
env = VecEnv(n, seed=1234, device=0, config=EnvConfig(map_name='loop_empty'))
env.reset()
ro = RenderOutput(n, dev)
masks_b = torch.zeros_like(ro.masks)
g = torch.Generator(device=dev)
g.manual_seed(3)
s = torch.cuda.current_stream(dev)
res = {'single': [], 'pair': []}
for r in range(R + 1):
    for form in ('single', 'pair'):
        acts = torch.rand(k, n, 2, generator=g, device=dev)
        out = StepOutput(k * n, dev, lanepos=False, tile=False)
        pose = torch.empty(k, 3, n, dtype=torch.float64, device=dev)
        env.step_many_into(acts, out, pose=pose)
        done = out.done.view(k, n)
        if form == 'single':
            calls = [bind_render(env, ro, s, fresh=done[d], pose=pose[d]) for d in range(k)]
        else:
            calls = [bind_render2(env, ro, s, masks_b, done[d], pose[d], done[d + 1], pose[d + 1])
                     for d in range(0, k, 2)]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = 0
        for c in calls:
            rc |= c()
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if r:
            res[form].append(e0.elapsed_time(e1) / k)
for form, v in res.items():
    print('%-6s ms per decision: %s  mean %.4f' % (form, ' '.join('%.4f' % x for x in v),
                                                  sum(v) / len(v)))
