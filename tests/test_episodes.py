"""Episode accounting host logic (aido1_amd/episodes.py) on CPU: the explorers'
per-episode units (training/explorers.py:134-140), the exploiter checkpoint
rule (:142-152), the record layout against include/dtactor.h, and the
restatement of dt_episode_account the GPU tests and the gloo test use."""
import os
import re

import numpy as np

from conftest import REPO
from aido1_amd.episodes import COLUMNS, RECORD, EpisodeBook, ExploiterSaver, ScalarLog, metrics


def account(rews, rewms, dones):
    """dt_episode_account restated over [D, n] per-decision arrays: the
    explorer's `episode_metrics[...] += ...` per env in decision order, one
    record per done (explorers.py:118-123, 202-204).  Returns a RECORD array
    ordered by (tick, env) and the running sums."""
    D, n = dones.shape
    r, m = np.zeros(n), np.zeros(n)
    length, ep = np.zeros(n, np.int64), np.zeros(n, np.int64)
    out = []
    for d in range(D):
        r = r + rews[d]
        m = m + rewms[d]
        length += 1
        for i in np.nonzero(dones[d])[0]:
            out.append((r[i], m[i], d + 1, ep[i], i, length[i]))
        f = dones[d].astype(bool)
        r[f], m[f], length[f] = 0.0, 0.0, 0
        ep += f
    return np.array(out, RECORD), (r, m, length)


def test_record_layout_matches_header():
    src = open(os.path.join(REPO, 'include', 'dtactor.h')).read()
    body = re.search(r'typedef struct DtEpisodeRecord \{(.*?)\} DtEpisodeRecord;', src, re.S)
    fields = re.findall(r'(double|int64_t|int32_t)\s+(\w+);', body.group(1))
    kinds = {'double': '<f8', 'int64_t': '<i8', 'int32_t': '<i4'}
    assert [(n, kinds[t]) for t, n in fields] == [(n, RECORD[n].str) for n in RECORD.names]
    assert RECORD.itemsize == 40


def test_metrics_units():
    recs = np.zeros(2, RECORD)
    recs['reward'] = [3.0, -7.5]
    recs['reward_modified'] = [1.5, 2.25]
    recs['decisions'] = [4, 11]
    m = metrics(recs, reward_scale=0.5, repeat_actions=3)
    assert m['reward'].tolist() == [6.0, -15.0]
    assert m['reward_modified'].tolist() == [3.0, 4.5]
    assert m['step'].tolist() == [12, 33]


def _explorer_saves(rewards, tol, every):
    """explorers.py:142-152 one episode at a time: (counter, reward) saved."""
    best, saves = -np.inf, []
    for c, r in enumerate(rewards, 1):
        cond = r > best + tol
        if cond:
            best = r
        if c % every == 0 or cond:
            saves.append((c, r))
    return saves, best


def test_exploiter_saver_follows_explorer_rule():
    rng = np.random.default_rng(3)
    rewards = np.cumsum(rng.normal(0.2, 2.0, 400))
    cfg = {'training': {'saving_reward_tolerance': 1, 'save_every_episode': 50}}
    got = []
    sv = ExploiterSaver(cfg, lambda c, r, best: got.append((c, r, best)) or 'dir')
    polls = np.split(rewards, [7, 8, 60, 61, 150, 333])
    for p in polls:
        sv(p)
    saves, best = _explorer_saves(rewards, 1, 50)
    assert sv.counter == 400 and sv.best == best
    # a poll saves once per trigger kind: its last best-reward episode and its
    # last periodic one, each a (counter, reward) the reference saves under
    expect = []
    bounds = np.cumsum([0] + [len(p) for p in polls])
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        b = [s for s in saves if lo < s[0] <= hi and _is_best(rewards, s[0], 1)]
        e = [s for s in saves if lo < s[0] <= hi and s[0] % 50 == 0]
        trig = sorted({t for t in (b[-1:] + e[-1:])})
        expect += [t + (bool(b) and t == b[-1],) for t in trig]
    assert got == expect
    assert [s[:2] for s in sv.saved] == [t[:2] for t in expect]
    assert all(s in saves for s in [t[:2] for t in expect])
    assert sum(t[2] for t in expect) >= 2 and any(not t[2] for t in expect)


def _is_best(rewards, c, tol):
    """Episode c (1-based) meets explorers.py:142's saving_best_cond."""
    return rewards[c - 1] > max([-np.inf] + list(_running_best(rewards[:c - 1], tol))) + tol \
        if c > 1 else True


def _running_best(rewards, tol):
    best = -np.inf
    for r in rewards:
        if r > best + tol:
            best = r
        yield best


def test_episode_book_single_rank(tmp_path):
    """ws = 1: the table in the explorers' units, exploiters = envs >= n_explore,
    scalars written with the reference's tag names."""
    rng = np.random.default_rng(4)
    D, n = 40, 16
    dones = rng.random((D, n)) < 0.2
    recs, _ = account(rng.normal(size=(D, n)), rng.normal(size=(D, n)), dones)
    cfg = {'environment': {'wrapper': {'reward_scale': 2.0, 'repeat_actions': 3}},
           'training': {'saving_reward_tolerance': 0.5, 'save_every_episode': 5}}
    saved = []
    book = EpisodeBook(cfg, 'cpu', n_explore=12, save=lambda c, r: saved.append((c, r)),
                       log_dir=str(tmp_path))
    out = book.poll(recs)
    assert set(out) == set(COLUMNS) | {'exploiting'}
    assert np.array_equal(out['env'], recs['env']) and np.array_equal(out['tick'], recs['tick'])
    assert np.array_equal(out['reward'], recs['reward'] / 2.0)
    assert np.array_equal(out['step'], recs['decisions'] * 3)
    assert np.array_equal(out['exploiting'], recs['env'] >= 12)
    rew = out['reward'][out['exploiting']]
    saves, best = _explorer_saves(rew, 0.5, 5)
    b = [s for s in saves if _is_best(rew, s[0], 0.5)]
    e = [s for s in saves if s[0] % 5 == 0]
    assert saved == sorted({t for t in (b[-1:] + e[-1:])}) and book.exploiter.best == best
    assert [r['value'] for r in book.log.rows if r['tag'] == 'best reward'] == [b[-1][1]]
    tags = {r['tag'] for r in book.log.rows}
    assert {'exploring/reward', 'exploiting/reward', 'step per second', 'episode per minute',
            'best reward'} <= tags
    assert os.path.exists(os.path.join(tmp_path, 'scalars.jsonl'))
    assert len(book.poll(np.zeros(0, RECORD))['reward']) == 0


def test_scalar_log_in_memory():
    log = ScalarLog(None, keep=3)
    for i in range(5):
        log.scalar_summary('reward', i, i)
    assert [r['value'] for r in log.rows] == [2.0, 3.0, 4.0]
