"""The N>1 path on CPU: world_size-2 gloo processes exercise the run
reduction, the episode-return gather and the bucketed gradient all-reduce
(the same code runs over RCCL on the GPUs)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        from aido1_amd import distributed as D
        assert D.env_id_base(rank, 4096) == rank * 4096
        counts, el = D.reduce_run({'env_steps': 100 * (rank + 1), 'resets': rank}, 1.0 + rank)
        ret = D.gather_returns(torch.arange(rank + 1, dtype=torch.float64) + 10 * rank)
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 2))
        x = torch.full((4, 8), float(rank + 1))
        model(x).sum().backward()
        local = [p.grad.clone() for p in model.parameters()]
        D.GradAllReduce(model.parameters(), bucket_mb=0.0001)()
        q.put((rank, counts, el, ret.tolist(), [g.tolist() for g in local],
               [p.grad.tolist() for p in model.parameters()]))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo():
    ws = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(ws)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, counts, el, ret, local, red in res:
        assert counts == {'env_steps': 300.0, 'resets': 1.0}
        assert el == 2.0
        assert ret == [0.0, 10.0, 11.0]
    # all-reduced grads = mean of the two ranks' local grads, identical on both
    l0, l1 = res[0][4], res[1][4]
    for a, b, g0, g1 in zip(l0, l1, res[0][5], res[1][5]):
        ta, tb = torch.tensor(a), torch.tensor(b)
        assert torch.allclose(torch.tensor(g0), (ta + tb) / 2)
        assert torch.equal(torch.tensor(g0), torch.tensor(g1))


def _trainer_worker(rank, ws, port, q):
    """Data-parallel DDPG update: each rank its own batch, gradients
    all-reduced before every optimiser step (trainer.py; RCCL on the GPUs)."""
    import sys
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, here)
        sys.path.insert(0, os.path.join(here, 'golden'))
        from formulas import formula_batch
        from test_trainer import make_trainer
        import numpy as np
        tr = make_trainer('cpu')
        assert tr.sync_actor is not None and tr.sync_critic is not None
        obs, act, rew, nxt, done = formula_batch(8)
        # rank-specific batch: different rewards and actions
        batch = (obs, np.roll(act, rank, 0), rew + 3.0 * rank, nxt, np.roll(done, rank))
        for _ in range(2):
            m, info = tr.update(batch)
        q.put((rank, float(m['critic_loss']),        # numpy: pickled by value
               [p.detach().numpy().copy() for p in tr.actor.parameters()],
               [p.detach().numpy().copy() for p in tr.target_critic.parameters()]))
    finally:
        dist.destroy_process_group()


def test_two_rank_trainer_replicas_stay_identical():
    ws = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trainer_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(ws)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, l0, a0, t0), (_, l1, a1, t1) = res
    assert l0 != l1                                   # different local batches ...
    for x, y in zip(a0 + t0, a1 + t1):
        assert (x == y).all()                         # ... identical replicas
