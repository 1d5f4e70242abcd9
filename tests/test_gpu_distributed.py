"""The data-parallel DDPG update on the GPU with two ranks (config 5's N > 1
path): two processes on cuda:0 joined by a gloo process group
(one box has one GPU; RCCL needs distinct devices), each with its own batch,
the update captured as three HIP graphs with the bucketed gradient
all-reduce (GradAllReduce) between them.  After three updates both replicas
must hold bit-identical parameters, different from an update on either
rank's batch alone."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rank):
    sys.path.insert(0, os.path.join(HERE, 'golden'))
    from formulas import formula_batch
    obs, act, rew, nxt, done = formula_batch(16)
    return obs + 0.05 * rank, act, rew + rank, nxt, done


def _flat(tr):
    return torch.cat([p.detach().reshape(-1).double().cpu() for m in (tr.actor, tr.critic)
                      for p in m.parameters()])


def _worker(rank, ws, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        from test_trainer import make_trainer
        tr = make_trainer(torch.device('cuda', 0), graph=True, warmup=1)
        assert tr.sync_actor is not None and tr.sync_critic is not None
        for _ in range(3):
            tr.update(_batch(rank))
        torch.cuda.synchronize()
        assert tr._graphs is not None and len(tr._graphs) == 3
        try:
            tr.check()          # names the first stage that produced NaN / Inf
            q.put((rank, _flat(tr).numpy()))
        except Exception as e:  # noqa: BLE001 -- reported by the parent
            q.put((rank, 'rank %d: %s' % (rank, e)))
            raise
    finally:
        dist.destroy_process_group()


def test_two_rank_update_replicas_identical(gpu):
    ws = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(ws))
    errs = [v for v in res.values() if isinstance(v, str)]
    assert not errs, errs
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(res[0], res[1])
    # a single-rank run on rank 0's batch alone ends elsewhere
    from test_trainer import make_trainer
    solo = make_trainer(gpu, graph=True, warmup=1)
    for _ in range(3):
        solo.update(_batch(0))
    torch.cuda.synchronize()
    assert not np.array_equal(_flat(solo).numpy(), res[0])
