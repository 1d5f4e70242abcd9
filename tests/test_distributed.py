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


def _oracle_episodes(rank, n=64, decisions=30):
    """One rank's finished-episode records: the C oracle's EnvironmentWrapper
    (envs [rank * n, (rank + 1) * n)) under random wheel actions, accounted
    as dt_episode_account does (test_episodes.account)."""
    import sys
    import numpy as np
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    from conftest import map_rows
    from oracle import oracle_c as OC
    from test_episodes import account
    ob = OC.OracleBatch(map_rows('loop_empty'), n, seed=1234, env_base=rank * n)
    ob.reset()
    rng = np.random.default_rng(100 + rank)
    rs, rms, ds = [], [], []
    for _ in range(decisions):
        o = ob.step(rng.uniform(0, 1, (n, 2)).astype(np.float32))
        rs.append(o['reward'])
        rms.append(o['reward_mod'])
        ds.append(o['done'])
    return account(np.stack(rs), np.stack(rms), np.stack(ds))[0]


EP_CONFIG = {'environment': {'wrapper': {'reward_scale': 1.0, 'repeat_actions': 3}},
             'training': {'saving_reward_tolerance': 1, 'save_every_episode': 7}}


def _episode_worker(rank, ws, port, q):
    """TrainLoop.poll_episodes' host side (episodes.EpisodeBook) on two ranks:
    each polls its own oracle episodes twice; both must see every rank's."""
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        from aido1_amd.episodes import EpisodeBook
        recs = _oracle_episodes(rank)
        saved = []
        book = EpisodeBook(EP_CONFIG, 'cpu', n_explore=56, save=lambda c, r: saved.append((c, r)))
        half = recs['tick'] <= 15
        tabs = [book.poll(recs[half]), book.poll(recs[~half])]
        q.put((rank, [{k: v.tolist() for k, v in t.items()} for t in tabs], saved,
               book.exploiter.counter, book.exploiter.best, book.episodes_done))
    finally:
        dist.destroy_process_group()


def test_two_rank_episode_gather_and_exploiter_saves():
    import numpy as np
    from test_episodes import _explorer_saves
    ws = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_episode_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(ws)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, tabs0, saved0, c0, b0, n0), (_, tabs1, saved1, c1, b1, n1) = res
    assert tabs0 == tabs1 and (c0, b0, n0) == (c1, b1, n1)
    assert saved1 == []                                   # rank 0 saves
    recs = [_oracle_episodes(r) for r in range(ws)]
    rewards = []
    for part in (0, 1):
        rows = []
        for r in range(ws):
            sel = (recs[r]['tick'] <= 15) if part == 0 else (recs[r]['tick'] > 15)
            for x in recs[r][sel]:
                rows.append((int(x['tick']), r, int(x['env']), float(x['reward']),
                             int(x['decisions']) * 3))
        rows.sort()
        t = tabs0[part]
        assert list(zip(t['tick'], t['rank'], t['env'], t['reward'], t['step'])) == rows
        assert set(t['rank']) == {0, 1}
        rewards.append([x[3] for x in rows if x[2] >= 56])
    saves, best = _explorer_saves(np.array(rewards[0] + rewards[1]), 1, 7)
    assert c0 == len(rewards[0]) + len(rewards[1]) and b0 == best
    per_poll = []
    for lo, hi in ((0, len(rewards[0])), (len(rewards[0]), c0)):
        inside = [s for s in saves if lo < s[0] <= hi]
        if inside:
            per_poll.append(inside[-1])
    assert [tuple(s) for s in saved0] == per_poll and per_poll
