"""Diagnostic: config 3's renders one decision a launch (dt_render) against two
and three decisions a launch (dt_render2 / dt_render3), 4096 envs on
loop_empty, the poses and done flags of dt_step_many chunks of 18 decisions;
HIP events around each chunk's renders.  Prints ms per decision for each form
(alternating, R rounds)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.config import EnvConfig  # noqa: E402
from aido1_amd.render import RenderOutput, bind_render, bind_render_group  # noqa: E402
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402

n, k, R = 4096, 18, int(os.environ.get('R', '5'))
dev = torch.device('cuda', 0)
env = VecEnv(n, seed=1234, device=0, config=EnvConfig(map_name='loop_empty'))
env.reset()
ro = RenderOutput(n, dev)
extra = [torch.zeros_like(ro.masks) for _ in range(2)]
g = torch.Generator(device=dev)
g.manual_seed(3)
s = torch.cuda.current_stream(dev)
res = {1: [], 2: [], 3: []}
for r in range(R + 1):
    for form in (1, 2, 3):
        acts = torch.rand(k, n, 2, generator=g, device=dev)
        out = StepOutput(k * n, dev, lanepos=False, tile=False)
        pose = torch.empty(k, 3, n, dtype=torch.float64, device=dev)
        env.step_many_into(acts, out, pose=pose)
        done = out.done.view(k, n)
        if form == 1:
            calls = [bind_render(env, ro, s, fresh=done[d], pose=pose[d]) for d in range(k)]
        else:
            calls = [bind_render_group(env, ro, s, extra[:form - 1],
                                       [done[d + i] for i in range(form)],
                                       [pose[d + i] for i in range(form)])
                     for d in range(0, k, form)]
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
    print('%d a launch, ms per decision: %s  mean %.4f' % (form, ' '.join('%.4f' % x for x in v),
                                                  sum(v) / len(v)))
