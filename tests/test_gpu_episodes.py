"""Episode accounting on the GPU (training/explorers.py:118-154, 202-204;
utils/env_wrappers.py:197,251).

* dt_episode_account's records at 4096 envs, one decision a launch and
  dt_step_many chunks of 20, against the reference explorer's sums over the C
  oracle's EnvironmentWrapper rewards: (env, episode, tick, length) and done
  exact, returns within the pose/reward bar; bit for bit against the same
  sums over the kernel's own per-decision outputs.
* EnvironmentWrapper.total_reward keeps a finished episode's return.
* TrainLoop: the rollout's episodes polled, the exploiters' checkpoints
  written on a new best / every save_every_episode."""
import copy
import os

import numpy as np
import pytest
import torch

from conftest import golden
from test_episodes import account
from test_gpu_step import TOL_SPEC, make_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('k', [1, 20])
def test_episode_records_match_oracle(gpu, k):
    from aido1_amd.episodes import EpisodeTracker
    from aido1_amd.vec_env import StepOutput
    n, decisions = 4096, 60
    env, ob = make_pair(n)
    env.reset()
    ob.reset()
    tr = EpisodeTracker(n, gpu)
    out = StepOutput(k * n, gpu, lanepos=False, tile=False)
    rng = np.random.default_rng(5 + k)
    g_r, g_m, g_d, o_r, o_m, o_d, recs = [], [], [], [], [], [], []
    for launch in range(decisions // k):
        a = rng.uniform(0, 1, (k, n, 2)).astype(np.float32)
        if k == 1:
            o = env.step_into(torch.from_numpy(a[0]).to(gpu), out)
        else:
            o = env.step_many_into(torch.from_numpy(a).to(gpu), out)
        tr.account(o.reward, o.reward_mod, o.done)
        g_r.append(o.reward.view(k, n).cpu().numpy())
        g_m.append(o.reward_mod.view(k, n).cpu().numpy())
        g_d.append(o.done.view(k, n).cpu().numpy())
        for d in range(k):
            ref = ob.step(a[d])
            o_r.append(ref['reward'])
            o_m.append(ref['reward_mod'])
            o_d.append(ref['done'])
        if launch % 2:
            recs.append(tr.drain())          # drains between launches
    recs.append(tr.drain())
    got = np.concatenate(recs)
    got = got[np.lexsort((got['env'], got['tick']))]
    g_d, o_d = np.concatenate(g_d), np.stack(o_d)
    assert np.array_equal(g_d, o_d)
    mine, (run_r, run_m, run_len) = account(np.concatenate(g_r), np.concatenate(g_m), g_d)
    ref, _ = account(np.stack(o_r), np.stack(o_m), o_d)
    assert len(got) == len(ref) > n // 2 and tr.lost == 0
    for f in ('env', 'tick', 'episode', 'decisions'):
        assert np.array_equal(got[f], ref[f]), f
    for f in ('reward', 'reward_modified'):
        assert np.array_equal(got[f], mine[f]), f                 # the kernel's sums, bitwise
        assert np.max(np.abs(got[f] - ref[f])) <= TOL_SPEC, f     # vs the oracle
    cr, cm, cl = tr.current()
    assert np.array_equal(cr.cpu().numpy(), run_r) and np.array_equal(cm.cpu().numpy(), run_m)
    assert np.array_equal(cl.cpu().numpy(), run_len)
    if k > 1:   # envs that finish more than once inside one chunk: one record each
        launch_of = (got['tick'] - 1) // k
        key = got['env'].astype(np.int64) * 1000 + launch_of
        assert (np.unique(key, return_counts=True)[1] > 1).any()


def test_episode_ring_overflow_counts_lost(gpu):
    from aido1_amd.episodes import EpisodeTracker
    n = 4096
    env, _ = make_pair(n)
    env.reset()
    tr = EpisodeTracker(n, gpu, capacity=100)
    total = 0
    for _ in range(20):
        o = env.step_into(torch.rand(n, 2, device=gpu))
        tr.account(o.reward, o.reward_mod, o.done)
        total += int(o.done.sum())
    recs = tr.drain()
    assert total > 100 and len(recs) == 100 and tr.lost == total - 100
    assert len(tr.drain()) == 0


def test_env_wrapper_total_reward_survives_done(gpu):
    """total_reward = the episode's running sum; a finished env's sum stays
    readable after the step that finished it and restarts at its next step."""
    from aido1_amd.env_wrappers import EnvironmentWrapper
    n = 512
    w = EnvironmentWrapper(golden('reference_config.json'), n_envs=n, obs='lane', seed=7)
    w.reset()
    run = np.zeros(n)
    finished = 0
    for _ in range(30):
        a = torch.rand(n, 2, device=gpu) * 2 - 1            # tanh head: mapped in place
        _, (r, _), done, _ = w.step(a)
        run = run + r.cpu().numpy()
        assert np.array_equal(w.total_reward.cpu().numpy(), run)
        d = done.cpu().numpy()
        finished += int(d.sum())
        run[d] = 0.0
    assert finished > 0


def _loop(cfg, tmp_path, **kw):
    from aido1_amd.train_loop import TrainLoop
    return TrainLoop(cfg, n_envs=128, device=0, seed=5, buffer_size=1024, batch_size=32,
                     save_dir=str(tmp_path / 'saved'), log_dir=str(tmp_path / 'logs'), **kw)


def short_episode_config():
    cfg = copy.deepcopy(golden('reference_config.json'))
    cfg['environment']['wrapper']['max_env_steps'] = 9      # every episode <= 4 decisions
    cfg['training']['saving_reward_tolerance'] = 1
    cfg['training']['save_every_episode'] = 50
    return cfg


def test_train_loop_episodes_and_exploiter_checkpoints(gpu, tmp_path):
    from aido1_amd.checkpoint import load
    from aido1_amd.actor import ConfigActor, ConfigCritic
    cfg = short_episode_config()
    loop = _loop(cfg, tmp_path, poll_every=4, check_every=8)
    loop.reset()
    rs, rms, ds = [], [], []
    for _ in range(16):
        r, rm, d = loop.step()
        rs.append(r.cpu().numpy())
        rms.append(rm.cpu().numpy())
        ds.append(d.cpu().numpy())
    last = loop.poll_episodes()                 # nothing new since the poll at 16
    assert len(last['reward']) == 0
    book = loop.book
    expect, _ = account(np.stack(rs), np.stack(rms), np.stack(ds))
    assert book.episodes_done == len(expect) >= 128
    ne = loop.rollout.n_explore
    assert ne == 112                                          # 7 exploring : 1 exploiting
    ex = expect[expect['env'] >= ne]
    assert book.exploiter.counter == len(ex) > 0
    assert book.exploiter.best == pytest.approx(float(ex['reward'].max()), abs=0)
    # the first exploiter episode beats -inf: at least one save, each in the
    # reference's layout and loadable
    assert book.exploiter.saved
    base = os.path.join(str(tmp_path / 'saved'), 'exploiting_virtual_thread_0')
    for c, r, d in book.exploiter.saved:
        assert d == os.path.join(base, 'episode_{}_reward_{:.2f}'.format(c, r))
        for f in ('config.json', 'actor_state_dict.pth', 'critic_state_dict.pth'):
            assert os.path.exists(os.path.join(d, f))
    a, c = ConfigActor(cfg['model']['actor']), ConfigCritic(cfg['model']['critic'])
    load(book.exploiter.saved[-1][2], a, c)
    tags = [json_row['tag'] for json_row in book.log.rows]
    assert 'exploiting/reward' in tags and 'step per second' in tags
    assert os.path.getsize(str(tmp_path / 'logs' / 'scalars.jsonl')) > 0
