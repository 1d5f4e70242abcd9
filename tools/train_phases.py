"""Diagnostic: per-phase GPU time of one TrainLoop decision (config 5):
rollout, add_batch_ring, sample, update, priorities, actor refresh.
Run on the GPU box: python tools/train_phases.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.train_loop import TrainLoop  # noqa: E402


def main():
    if os.environ.get('TP_CUDNN_BENCH'):   # MIOpen Find-mode algorithm search (experiment)
        torch.backends.cudnn.benchmark = True
    with open(os.path.join(os.path.dirname(__file__), '..', 'aido1_amd', 'configs',
                           'reference_config.json')) as f:
        cfg = json.load(f)
    loop = TrainLoop(cfg, 4096, device=0, buffer_size=131072)
    loop.reset()
    for _ in range(6):
        loop.step()
    torch.cuda.synchronize()
    names = ['rollout', 'add_batch_ring', 'sample', 'update', 'priorities', 'refresh']
    acc = {k: [] for k in names}
    for _ in range(20):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
        ev[0].record()
        r, rm, done = loop.rollout.step()
        ev[1].record()
        loop.obs = loop.replay.add_batch_ring(loop.obs, loop.rollout.actions, rm,
                                              loop.rollout.ring, loop.rollout.order(), done)
        ev[2].record()
        obs, act, rew, nx, dn, _w, idx = loop.replay.sample(loop.batch_size, loop.beta)
        ev[3].record()
        loop.metrics, info = loop.trainer.update((obs, act, rew, nx, dn))
        ev[4].record()
        pr = info['td_error'].detach().abs().reshape(-1).double() + 1e-6
        loop.replay.update_priorities(idx, pr)
        ev[5].record()
        loop._refresh()
        ev[6].record()
        torch.cuda.synchronize()
        for i, k in enumerate(names):
            acc[k].append(ev[i].elapsed_time(ev[i + 1]))
    for k in names:
        print('%-12s %.3f ms' % (k, float(np.median(acc[k]))))


if __name__ == '__main__':
    main()
