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


def _loop_worker(rank, ws, port, save_dir, q):
    """Two real TrainLoops (envs [rank * 64, (rank + 1) * 64)) whose finished
    episodes are gathered by poll_episodes over the process group."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        from aido1_amd.train_loop import TrainLoop
        from test_gpu_episodes import short_episode_config
        loop = TrainLoop(short_episode_config(), n_envs=64, device=0, seed=5,
                         env_id_base=rank * 64, buffer_size=512, batch_size=32,
                         save_dir=save_dir)
        loop.reset()
        for _ in range(8):
            loop.step()
        loop.check()
        tab = loop.poll_episodes()
        q.put((rank, {k: v.tolist() for k, v in tab.items()}, loop.book.exploiter.saved))
    except Exception as e:  # noqa: BLE001 -- reported by the parent
        q.put((rank, 'rank %d: %s' % (rank, e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_train_loops_gather_episodes(gpu, tmp_path):
    ws = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    save_dir = str(tmp_path / 'saved')
    procs = [ctx.Process(target=_loop_worker, args=(r, ws, port, save_dir, q))
             for r in range(ws)]
    for p in procs:
        p.start()
    res = {r: (t, s) for r, t, s in (q.get(timeout=300) for _ in range(ws))}
    errs = [t for t, _ in res.values() if isinstance(t, str)]
    assert not errs, errs
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    t0, t1 = res[0][0], res[1][0]
    assert t0 == t1 and set(t0['rank']) == {0, 1}
    keys = list(zip(t0['tick'], t0['rank'], t0['env']))
    assert keys == sorted(keys) and len(keys) >= 64     # every env finishes within 4 decisions
    assert res[0][1] and all(d is None for _, _, d in res[1][1])   # rank 0 writes
    for _, _, d in res[0][1]:
        assert os.path.exists(os.path.join(d, 'actor_state_dict.pth'))
