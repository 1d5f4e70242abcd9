"""Diagnostic: detect_lines time on 4096 rendered envs (white and yellow)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.render import RenderOutput, detect_lines, hough_lines, MASK_EDGES, COLOR_PLANE  # noqa: E402
from aido1_amd.vec_env import StepOutput, VecEnv  # noqa: E402

n = 4096
gpu = torch.device('cuda', 0)
env = VecEnv(n, seed=3, device=0)
env.reset()
out = StepOutput(n, gpu, lanepos=False, tile=False)
ro = RenderOutput(n, gpu)
for _ in range(5):
    env.step_into(torch.rand(n, 2, device=gpu), out)
    env.render_into(ro, fresh=out.done)
torch.cuda.synchronize()
for color in ('white', 'yellow'):
    ec = (ro.masks[:, COLOR_PLANE[color]] & ro.masks[:, MASK_EDGES]).contiguous()
    hough_lines(ec)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lines, counts = hough_lines(ec)
    e1.record()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    det = detect_lines(ro.masks, color)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    px = (ec != 0).sum(dim=(1, 2)).float()
    print('%s: hough kernel %.3f ms for %d images (edge px mean %.0f max %.0f, lines mean %.1f '
          'max %d); detect_lines wall %.3f ms' % (color, e0.elapsed_time(e1), n, px.mean(),
                                                    px.max(), counts.float().mean(),
                                                    counts.max(), (t1 - t0) * 1e3))
env.close()
