"""HTTP env-server compatibility (aido1_amd/env_server.py) on CPU with a stand-in
batch: routes, the reference client's double-encoded bodies
(utils/env_wrappers.py:70-100, pyramid_worker.py:25-52), replies, and that
concurrent requests are served as one batch."""
import json
import socket
import threading

import numpy as np
import pytest
import requests

from aido1_amd.env_server import EnvServer


class FakeBatch:
    def __init__(self, n):
        self.n = n
        self.pos = np.zeros(n)
        self.seeds = [None] * n
        self.step_batches = []

    def seed(self, env, seed):
        self.seeds[env] = seed

    def reset(self, envs):
        for e in envs:
            self.pos[e] = 0.0

    def step(self, envs, actions):
        self.step_batches.append(sorted(envs))
        out = []
        for e, a in zip(envs, actions):
            self.pos[e] += float(a[0] + a[1])
            out.append((float(self.pos[e]), self.pos[e] > 3.0, {'Simulator': {'env': e}}))
        return out

    def observations(self, envs):
        return [[[[float(self.pos[e])]]] for e in envs]


def _free_base(n):
    for base in range(23000, 60000, 97):
        socks = []
        try:
            for i in range(n):
                s = socket.socket()
                s.bind(('127.0.0.1', base + i))
                socks.append(s)
            return base
        except OSError:
            continue
        finally:
            for s in socks:
                s.close()
    raise RuntimeError('no free ports')


class Client:
    """The request side of the reference's VirtualEnvironment."""

    def __init__(self, port):
        self.url = 'http://127.0.0.1:%d/%%s/' % port

    def step(self, action):
        res = requests.post(self.url % 'post_step_request',
                            json=json.dumps({'action': list(action)})).json()
        return res['observation'], res['reward'], res['done'], res['info']

    def reset(self):
        return requests.post(self.url % 'post_reset_request', json={}).json()['observation']

    def change_model(self, seed):
        return requests.post(self.url % 'post_change_model_request',
                             json=json.dumps({'seed': seed})).json()

    def collect_garbage(self):
        return requests.post(self.url % 'post_collect_garbage_request', json={}).json()


@pytest.fixture
def server():
    fb = FakeBatch(4)
    base = _free_base(4)
    srv = EnvServer(fb, port_start=base, window_s=0.05).start()
    yield fb, base
    srv.stop()


def test_routes_and_replies(server):
    fb, base = server
    c = Client(base + 2)
    assert c.change_model(7) == {'success': True} and fb.seeds[2] == 7
    assert c.reset() == [[[0.0]]]
    obs, r, d, info = c.step([0.5, 1.0])
    assert obs == [[[1.5]]] and r == 1.5 and d is False and info == {'Simulator': {'env': 2}}
    obs, r, d, info = c.step([1.0, 1.0])
    assert r == 3.5 and d is True
    assert json.loads(c.collect_garbage()) == {'success': True}   # double-encoded reply
    assert requests.post('http://127.0.0.1:%d/nope/' % base, json={}).status_code == 404


def test_concurrent_steps_are_batched(server):
    fb, base = server
    clients = [Client(base + i) for i in range(4)]
    barrier = threading.Barrier(4)
    out = [None] * 4

    def run(i):
        barrier.wait()
        out[i] = clients[i].step([0.1 * i, 0.0])

    ts = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    assert [o[1] for o in out] == pytest.approx([0.0, 0.1, 0.2, 0.3])
    assert max(len(b) for b in fb.step_batches) >= 2      # served together
