"""The batched env server on the GPU: four concurrent clients speaking the
reference's VirtualEnvironment protocol, each checked step for step against a
standalone Simulator of the same env id and seed — masked batching must not
change any env's trajectory."""
import threading

import numpy as np
import pytest

from test_env_server import Client, _free_base

pytestmark = pytest.mark.gpu


def _gray(rgb):   # PreliminaryTransformer on the Simulator's raster
    return ((rgb.astype(np.float64) / 255.0) @ np.array([0.2125, 0.7154, 0.0721]))[None]


def test_server_matches_standalone_simulators(gpu):
    from aido1_amd.env_server import EnvServer, GpuBatch
    from aido1_amd.simulator import Simulator
    n, steps = 4, 25
    base = _free_base(n)
    srv = EnvServer(GpuBatch(n, device=0), port_start=base, window_s=0.01).start()
    logs = [None] * n
    barrier = threading.Barrier(n)

    def client(i):
        c = Client(base + i)
        rng = np.random.default_rng(100 + i)
        c.change_model(1000 + i)
        log = [('reset', np.asarray(c.reset()))]
        barrier.wait()
        for _ in range(steps):
            a = rng.uniform(0, 1, 2).tolist()
            obs, r, d, info = c.step(a)
            log.append(('step', a, np.asarray(obs), r, d))
            if d:
                log.append(('reset', np.asarray(c.reset())))
        logs[i] = log

    ts = [threading.Thread(target=client, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    srv.stop()
    for i in range(n):
        assert logs[i] is not None, i
        sim = Simulator(seed=1000 + i, env_id=i, device=0, accept_start_angle_deg=4)
        for entry in logs[i]:
            if entry[0] == 'reset':
                assert np.array_equal(entry[1], _gray(sim.reset())), i
            else:
                _, a, obs, r, d = entry
                o2, r2, d2, _ = sim.step(np.asarray(a, np.float32))
                assert r == r2 and d == d2, (i, r, r2)
                assert np.array_equal(obs, _gray(o2)), i
        sim.close()
