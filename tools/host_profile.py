"""Host-side cost of one training-loop decision (GPU): cProfile over K
TrainLoop.step calls after warm-up, without extra synchronisation, so the
listed times are what the Python host spends issuing work (the GPU idles
whenever the host falls behind it).  usage: python tools/host_profile.py [K]"""
import cProfile
import json
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.train_loop import TrainLoop  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    with open(os.path.join(os.path.dirname(__file__), '..', 'aido1_amd', 'configs',
                           'reference_config.json')) as f:
        cfg = json.load(f)
    loop = TrainLoop(cfg, 4096, device=0, seed=1234, buffer_size=131072)
    loop.reset()
    for _ in range(8):
        loop.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        loop.step()
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print('host issue %.3f ms / decision, wall %.3f ms / decision' % (1e3 * host / k,
                                                                   1e3 * wall / k))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(k):
        loop.step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats('cumulative').print_stats(45)
    st.sort_stats('tottime').print_stats(30)


if __name__ == '__main__':
    main()
