"""Per-episode accounting on the batched path, and what the reference's
explorers do with it (training/explorers.py).

Each of the reference's explorer processes sums its episode's rewards in
Python floats (explorers.py:118-123, 202-204), then per finished episode
divides the sums by reward_scale and multiplies the decision count by
repeat_actions (:134-140), tracks the best reward and saves the exploiter's
model on a new best (plus saving_reward_tolerance) or every
save_every_episode episodes (:142-152), and logs reward, modified reward,
steps, epsilon, episodes per minute and steps per second (:215-240).

Here thousands of envs a GPU finish episodes inside one launch:

  EpisodeTracker   device accumulators + a ring of finished-episode records
                   (dt_episode_account, include/dtactor.h), fed with every
                   decision's [k, n] reward / reward_mod / done (k = 1 after
                   dt_step, k decisions after dt_step_many); drain() reads
                   the records written since the last drain, ordered by
                   (tick, env): the order the per-env explorers would have
                   finished them in
  metrics()        the explorer's per-episode numbers from records
  ExploiterSaver   explorers.py:142-152 over the exploiting envs' episodes
  ScalarLog        utils/logger.py's scalar_summary(tag, value, step) as JSON
                   lines (tensorboardX is absent here)
  EpisodeBook      per poll: one rank's records -> all ranks' (gathered over
                   torch.distributed) -> ExploiterSaver and the explorers'
                   scalars (TrainLoop.poll_episodes)
"""
import ctypes
import json
import os
import time

import numpy as np
import torch

from aido1_amd import _lib
from aido1_amd import distributed as D

RECORD = np.dtype([('reward', '<f8'), ('reward_modified', '<f8'), ('tick', '<i8'),
                   ('episode', '<i8'), ('env', '<i4'), ('decisions', '<i4')])
assert RECORD.itemsize == 40     # sizeof(DtEpisodeRecord)


class EpisodeTracker:
    """Episode sums of n envs on one GPU (see the module docstring).

    capacity: records the device ring keeps between drains (older ones are
    overwritten and counted in `lost`)."""

    def __init__(self, n, device, capacity=None):
        self.n = int(n)
        self.device = torch.device(device)
        self.capacity = int(capacity or max(16 * self.n, 1 << 16))
        kw = dict(device=self.device)
        self.reward = torch.zeros(self.n, dtype=torch.float64, **kw)
        self.reward_modified = torch.zeros(self.n, dtype=torch.float64, **kw)
        self.tick = torch.zeros(self.n, dtype=torch.int64, **kw)
        self.episode = torch.zeros(self.n, dtype=torch.int64, **kw)
        self.decisions = torch.zeros(self.n, dtype=torch.int32, **kw)
        self.count = torch.zeros(1, dtype=torch.int64, **kw)     # uint64 on the device side
        self.ring = torch.zeros(self.capacity, RECORD.itemsize, dtype=torch.uint8, **kw)
        self.state = _lib.DtEpisodeState(
            self.reward.data_ptr(), self.reward_modified.data_ptr(), self.tick.data_ptr(),
            self.episode.data_ptr(), self.decisions.data_ptr(), self.count.data_ptr(),
            self.ring.data_ptr(), self.capacity)
        self.read = 0        # records drained so far
        self.lost = 0        # records overwritten before a drain
        self._L = _lib.lib()

    def account(self, reward, reward_mod, done, stream=None):
        """Enqueue one dt_episode_account over k = reward.numel() / n decisions."""
        m = reward.numel()
        for t, dt in ((reward, torch.float64), (reward_mod, torch.float64), (done, torch.uint8)):
            if (t.dtype != dt or t.device != self.device or not t.is_contiguous()
                    or t.numel() != m):
                raise ValueError('reward / reward_mod (f64) and done (u8) must be contiguous '
                                 '[k, %d] tensors on %s' % (self.n, self.device))
        if m == 0 or m % self.n:
            raise ValueError('%d entries is not k * %d' % (m, self.n))
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = self._L.dt_episode_account(self.n, m // self.n, reward.data_ptr(),
                                        reward_mod.data_ptr(), done.data_ptr(),
                                        ctypes.byref(self.state), ctypes.c_void_p(st.cuda_stream))
        if rc != 0:
            raise _lib.DtError('dt_episode_account failed (%d)' % rc)

    def reset(self):
        """Every env starts a new episode (an explicit reset): the running sums
        restart; records not yet drained stay."""
        for t in (self.reward, self.reward_modified, self.decisions):
            t.zero_()

    def drain(self):
        """Synchronise the device and return the records written since the last
        drain as a RECORD array ordered by (tick, env)."""
        torch.cuda.synchronize(self.device)
        count = int(self.count.item())
        new = count - self.read
        if new > self.capacity:
            self.lost += new - self.capacity
            self.read = count - self.capacity
        if count == self.read:
            return np.zeros(0, RECORD)
        idx = torch.arange(self.read, count, device=self.device) % self.capacity
        recs = self.ring[idx].cpu().numpy().reshape(-1).view(RECORD).copy()
        self.read = count
        return recs[np.lexsort((recs['env'], recs['tick']))]

    def current(self):
        """The running (reward, reward_modified, decisions) of every env's
        unfinished episode (device tensors, no copy)."""
        return self.reward, self.reward_modified, self.decisions


def metrics(recs, reward_scale=1.0, repeat_actions=3):
    """explorers.py:134-140 for every record: reward and reward_modified over
    reward_scale, step = decisions * repeat_actions (float64, as the Python
    floats)."""
    return {'reward': recs['reward'] / float(reward_scale),
            'reward_modified': recs['reward_modified'] / float(reward_scale),
            'step': recs['decisions'].astype(np.int64) * int(repeat_actions)}


class ScalarLog:
    """utils/logger.py Logger.scalar_summary as JSON lines in log_dir/scalars.jsonl
    (None: keep them in memory only, `self.rows`)."""

    def __init__(self, log_dir=None, keep=10000):
        self.path = None
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
            self.path = os.path.join(log_dir, 'scalars.jsonl')
        self.rows = []
        self.keep = keep

    def scalar_summary(self, tag, value, step):
        row = {'tag': tag, 'value': float(value), 'step': int(step), 'wall': time.time()}
        self.rows.append(row)
        del self.rows[:-self.keep]
        if self.path:
            with open(self.path, 'a') as f:
                f.write(json.dumps(row) + '\n')


class ExploiterSaver:
    """explorers.py:142-152 for the exploiting envs' finished episodes, taken
    in (tick, rank, env) order as one exploiter's episode sequence:
      counter += 1
      saving_best_cond = reward > saving_best_reward + saving_reward_tolerance
      (then saving_best_reward = reward)
      save if counter % save_every_episode == 0 or saving_best_cond.
    The exploiters of one poll act with the same weights, so one poll saves
    at most once per trigger kind: under the last best-reward episode's
    (counter, reward) and under the last periodic one's (one save when they
    are the same episode), so the directory names are ones the reference
    writes.  save(counter, reward, best) is told whether the save is a
    best-reward one (the reference logs 'best reward' only then,
    explorers.py:220-221)."""

    def __init__(self, config, save):
        t = config['training']
        self.tolerance = float(t.get('saving_reward_tolerance', 0.0))
        self.every = int(t.get('save_every_episode', 0) or 0)
        self.best = -np.inf
        self.counter = 0
        self.save = save           # save(episode_counter, reward, best) -> directory
        self.saved = []            # (counter, reward, directory or None)

    def __call__(self, rewards):
        """Feed one poll's rewards; returns the directories saved to."""
        best_t = per_t = None
        for r in np.asarray(rewards, np.float64):
            self.counter += 1
            if r > self.best + self.tolerance:
                self.best = float(r)
                best_t = (self.counter, float(r))
            if self.every and self.counter % self.every == 0:
                per_t = (self.counter, float(r))
        out = []
        for trig in sorted({t for t in (best_t, per_t) if t is not None}):
            d = self.save(trig[0], trig[1], trig == best_t)
            self.saved.append(trig + (d,))
            out.append(d)
        return out


COLUMNS = ('rank', 'env', 'tick', 'episode', 'reward', 'reward_modified', 'step')


class EpisodeBook:
    """What the reference's explorers do with finished episodes, for one
    rank's share of the envs (envs [n_explore, n) of every rank exploit).

    poll(recs) gathers every rank's records (a collective: every rank calls
    it), orders them by (tick, rank, env), feeds the exploiting envs' rewards
    to the ExploiterSaver (rank 0 saves, `save(counter, reward)`), logs the
    explorers' scalars and returns the table as a dict of numpy arrays
    (COLUMNS + 'exploiting'), in the explorers' units."""

    def __init__(self, config, device, n_explore, save=None, log_dir=None):
        w = config['environment']['wrapper']
        self.reward_scale = w.get('reward_scale', 1.0)
        self.repeat_actions = w.get('repeat_actions', 3)
        self.rank, self.world = D.world()
        self.device = torch.device(device)
        self.n_explore = int(n_explore)
        self.exploiter = ExploiterSaver(config, self._save)
        self._save_fn = save if self.rank == 0 else None
        self.log = ScalarLog(log_dir if self.rank == 0 else None)
        self.episodes_done = 0          # finished episodes, all ranks
        self.episode_steps = 0          # their env-steps (decisions x repeat_actions)
        self.best_reward = -np.inf      # explorers.py:217-218 (the shared best_reward)
        self.start_time = time.time()

    def _save(self, counter, reward, best):
        if self._save_fn is None:
            return None
        d = self._save_fn(counter, reward)
        if best:   # explorers.py:220-221: the new saving_best_reward
            self.log.scalar_summary('best reward', reward, counter)
        return d

    def table(self, recs):
        """One rank's records as the [m, 7] float64 table poll() gathers."""
        m = metrics(recs, self.reward_scale, self.repeat_actions)
        if not len(recs):
            return np.zeros((0, len(COLUMNS)))
        return np.stack([np.full(len(recs), self.rank, np.float64),
                         recs['env'].astype(np.float64), recs['tick'].astype(np.float64),
                         recs['episode'].astype(np.float64), m['reward'], m['reward_modified'],
                         m['step'].astype(np.float64)], 1)

    def poll(self, recs):
        tab = torch.from_numpy(np.ascontiguousarray(self.table(recs)))
        tab = D.gather_returns(tab.to(D.collective_device(self.device))).cpu().numpy()
        tab = tab[np.lexsort((tab[:, 1], tab[:, 0], tab[:, 2]))]
        out = {k: tab[:, i] for i, k in enumerate(COLUMNS)}
        for k in ('rank', 'env', 'tick', 'episode', 'step'):
            out[k] = out[k].astype(np.int64)
        out['exploiting'] = out['env'] >= self.n_explore
        self._log(out)
        self.exploiter(out['reward'][out['exploiting']])
        return out

    def _log(self, out):
        """explorers.py:215-240 per poll: the explorers' scalars, averaged over
        the poll's episodes of each kind (thousands of envs finish episodes
        every decision, so per-episode rows would be ~1e5 a second)."""
        n = len(out['reward'])
        if not n:
            return
        self.episodes_done += n
        self.episode_steps += int(out['step'].sum())
        self.best_reward = max(self.best_reward, float(out['reward'].max()))
        step = self.episodes_done
        for kind, sel in (('exploring', ~out['exploiting']), ('exploiting', out['exploiting'])):
            if sel.any():
                for k in ('reward', 'reward_modified', 'step'):
                    self.log.scalar_summary('%s/%s' % (kind, k), out[k][sel].mean(), step)
        el = max(time.time() - self.start_time, 1e-9)
        self.log.scalar_summary('episode per minute', self.episodes_done / el * 60, step)
        self.log.scalar_summary('step per second', self.episode_steps / el, step)
