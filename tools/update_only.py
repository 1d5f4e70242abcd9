"""Diagnostic (GPU): the DDPG update alone (config.json networks with their
dropout, batch 64, graph mode) on one synthetic batch, for a per-update kernel
profile: rocprofv3 --kernel-trace --stats -- python3 tools/update_only.py
Prints the median update time over the timed updates."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.actor import ConfigActor, ConfigCritic  # noqa: E402
from aido1_amd.trainer import DDPGTrainer  # noqa: E402


def main():
    n_up = int(os.environ.get('UPDATES', '50'))
    with open(os.path.join(os.path.dirname(__file__), '..', 'aido1_amd', 'configs',
                           'reference_config.json')) as f:
        cfg = json.load(f)
    torch.manual_seed(0)
    dev = torch.device('cuda', 0)
    tr = DDPGTrainer(cfg, ConfigActor(cfg['model']['actor']), ConfigCritic(cfg['model']['critic']),
                     device=dev, graph=True)
    for kv in filter(None, os.environ.get('TR_SET', '').split(',')):   # attr=0/1 on the trainer
        k, v = kv.split('=')
        setattr(tr, k, bool(int(v)))
    b = 64
    g = torch.Generator(device=dev).manual_seed(1)
    batch = (torch.rand(b, 3, 120, 160, device=dev, generator=g),
             torch.rand(b, 2, device=dev, generator=g) * 2 - 1,
             torch.rand(b, device=dev, generator=g),
             torch.rand(b, 3, 120, 160, device=dev, generator=g),
             torch.zeros(b, dtype=torch.bool, device=dev))
    for _ in range(5):
        tr.update(batch)
    torch.cuda.synchronize()
    def timed(fn):
        times = []
        for _ in range(n_up):
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            times.append(a.elapsed_time(e))
        return float(np.median(times))
    ab = os.environ.get('AB_ATTR')       # e.g. split_target: A/B of a trainer switch, one box
    if ab:
        tr2 = DDPGTrainer(cfg, ConfigActor(cfg['model']['actor']),
                          ConfigCritic(cfg['model']['critic']), device=dev, graph=True)
        setattr(tr2, ab, not getattr(tr, ab))
        for _ in range(5):
            tr2.update(batch)
        res = {True: [], False: []}
        for _ in range(5):
            for t in (tr, tr2):
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(n_up):
                    t.update_prepared()
                e.record()
                torch.cuda.synchronize()
                res[bool(getattr(t, ab))].append(a.elapsed_time(e) / n_up)
        for v in (True, False):
            print('%s=%s back to back: %s ms (median %.3f)'
                  % (ab, v, ' '.join('%.3f' % x for x in res[v]), float(np.median(res[v]))))
    t_full = timed(lambda: tr.update(batch))
    # the inputs already in the static buffers (TrainLoop: dt_frame_gather)
    t_prep = timed(tr.update_prepared)
    # back to back, as the training loop issues them (the host runs ahead of
    # the GPU, so its launch latency is hidden): mean over n_up updates
    b2b, host = [], []
    for _ in range(5):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        h0 = time.perf_counter()
        for _ in range(n_up):
            tr.update_prepared()
        host.append((time.perf_counter() - h0) * 1e3 / n_up)
        e.record()
        torch.cuda.synchronize()
        b2b.append(a.elapsed_time(e) / n_up)
    t_b2b = float(np.median(b2b))
    print('back to back, 5 runs of %d: %s ms' % (n_up, ' '.join('%.3f' % v for v in b2b)))
    print('host time a call (graph replay enqueue), same runs: %s ms'
          % ' '.join('%.3f' % v for v in host))
    tr.check()
    print('update %.3f ms with the input conversion + copies, %.3f ms on prepared inputs '
          '(medians of %d, each synchronised); %.3f ms back to back (median of 5 means of %d, '
          'host ahead)'
          % (t_full, t_prep, n_up, t_b2b, n_up))


if __name__ == '__main__':
    main()
