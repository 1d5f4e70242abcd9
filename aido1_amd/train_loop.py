"""Full DDPG training on the GPU (BASELINE configs[4]).

The reference splits this over processes and HTTP: explorers step envs and
push episodes (training/explorers.py:164-211), a sampling worker fills a
replay buffer and hands batches to the trainer through a queue
(training/workers_client.py:16-60), the trainer updates and soft-updates the
shared target model the explorers act with (training/trainers.py:143-237).
Here one process per GPU runs, per iteration:

  ActorRollout.step          one decision for n envs (actor on the frame ring,
                             exploration noise, 3 sim steps, render)
  replay.add_batch_ring      n transitions (obs, mapped action, reward_mod,
                             next_obs, done), HBM-resident; the frame store
                             copies each env's newest frame from the ring
                             and keeps frame indices for obs / next_obs
  replay.sample              batch_size transitions (proportional, GPU trees)
  DDPGTrainer.update         critic + actor + soft target update (grads
                             all-reduced over ranks with RCCL)
  replay.update_priorities   |td_error| + eps
  rollout actor refresh      the exploring envs act with the trained (online)
                             actor, as the reference's model workers do
                             (training/managers.py:182-208 pass
                             models[p_id], the models DDPGTrainer.update
                             steps); the exploiting envs with the target
                             actor (explorers.py:104-105, managers.py:239-262)

With overlap=True the update of decision t runs on a side stream while the
main stream runs decision t+1's rollout (actor, exploration, steps, render);
the main stream waits for it before decision t+1's add_batch_ring (the add
and update_priorities both write the sum tree) and only then refreshes the
acting copy, so the explorers act with weights one update older -- the
reference's explorers act with whatever the asynchronous trainer last
published (training/managers.py:113-124), so a lag of one update is within
its semantics.  overlap=False keeps the strictly sequential order.

Episodes (training/explorers.py:118-154, 215-240): the rollout keeps every
env's episode sums on the device (episodes.EpisodeTracker);
poll_episodes() drains the finished episodes, gathers them from every rank
(distributed.gather_returns), feeds the exploiting envs' ones to the
exploiter checkpoint rule (save() under save_dir) and logs the explorers'
scalars to log_dir (episodes.EpisodeBook).  step() calls it every
`poll_every` decisions and check() every `check_every` (0: the caller does;
both synchronise with the host).

Nothing else in the loop synchronises with the host.  Transition semantics: the
stored next_obs of a finished env is its respawn stack (auto-reset), harmless
because notdone = 0 removes Q(s') from its target.
"""
import os

import torch

from aido1_amd.actor import ConfigActor, ConfigCritic
from aido1_amd.episodes import EpisodeBook
from aido1_amd.guard import Guard
from aido1_amd.replay import PrioritizedReplayBuffer, ReplayBuffer
from aido1_amd.rollout import ActorRollout
from aido1_amd.trainer import DDPGTrainer

PRIORITY_EPS = 1e-6


class TrainLoop:
    def __init__(self, config, n_envs=4096, maps=('small_loop', 'zigzag'), device=0, seed=1234,
                 env_id_base=0, buffer_size=None, prioritized=True, batch_size=None,
                 updates_per_step=1, refresh_every=1, obs_dtype=None, actor_dtype=torch.float32,
                 actor_mode='reference', masks=False, graph=True, overlap=False, n_exploit=None,
                 save_dir=None, log_dir=None, poll_every=0, check_every=0, frames='index'):
        t = config['training']
        self.config = config
        self.device = torch.device('cuda', device)
        self.batch_size = int(batch_size or t['batch_size'])
        self.beta = t['beta']
        self.reward_modified = t.get('reward_modified', True)
        self.updates_per_step = updates_per_step
        self.refresh_every = refresh_every
        torch.manual_seed(seed)                         # identical init on every rank
        actor = ConfigActor(config['model']['actor'])
        critic = ConfigCritic(config['model']['critic'])
        # one non-finite guard for every stage of the loop (guard.py, check())
        self.guard = Guard(self.device)
        self.trainer = DDPGTrainer(config, actor, critic, device=self.device, graph=graph,
                                   guard=self.guard)
        self.rollout = ActorRollout(config, n_envs, maps=maps, device=device, seed=seed,
                                    env_id_base=env_id_base, actor=self.trainer.actor,
                                    dtype=actor_dtype, masks=masks, actor_mode=actor_mode,
                                    n_exploit=n_exploit, guard=self.guard, frames=frames)
        self.rollout.load_exploit_actor(self.trainer.target_actor)
        size = int(buffer_size or t['buffer_size'])
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed * 7919 + env_id_base)
        # the frame store (replay.py): one frame per env a decision instead of
        # two stacked observations per transition
        fe = n_envs if (size % n_envs == 0 and obs_dtype in (None, torch.float32)) else None
        if prioritized:
            self.replay = PrioritizedReplayBuffer(size, t['alpha'], device=self.device,
                                                  obs_dtype=obs_dtype, generator=gen,
                                                  frame_envs=fe)
        else:
            self.replay = ReplayBuffer(size, device=self.device, obs_dtype=obs_dtype, generator=gen,
                                       frame_envs=fe)
        self.prioritized = prioritized
        self.obs = None
        self.updates = 0
        self.decisions = 0
        self.metrics = None
        self.side = torch.cuda.Stream(self.device) if overlap else None
        self.pending = False        # an update is in flight on self.side
        self.refresh_due = False
        # episode accounting (explorers.py:118-154, 215-240)
        self.save_dir = save_dir
        self.book = EpisodeBook(config, self.device, self.rollout.n_explore,
                                save=self._save_exploiter if save_dir else None, log_dir=log_dir)
        self.poll_every, self.check_every = int(poll_every), int(check_every)

    def reset(self):
        self.rollout.reset()
        # the frame store keeps the ring's own frames (index bytes or grey)
        self.obs = self.rollout.stack(raw=self.replay.frame_envs is not None)

    def step(self, timing=None, update_timing=None):
        """One decision: rollout, add, and the update(s).  timing: an event
        pair around the actor forward (ActorRollout.step); update_timing: one
        around this decision's updates (recorded on the stream they run on)."""
        r, rm, done = self.rollout.step(timing)
        rew = rm if self.reward_modified else r        # explorers.py:205-206
        if self.pending:   # the previous update (side stream) precedes this add
            torch.cuda.current_stream(self.device).wait_stream(self.side)
            self.pending = False
            if self.refresh_due:
                self._refresh()
                self.refresh_due = False
        # next_obs straight from the frame ring into the buffer (frame store:
        # the newest frame only; otherwise the stored rows are the next
        # decision's obs); self.obs is None after the first add
        self.obs = self.replay.add_batch_ring(self.obs, self.rollout.actions, rew,
                                              self.rollout.ring, self.rollout.order(), done)
        self.decisions += 1
        if len(self.replay) >= max(self.batch_size, 2):
            if self.side is not None:
                self.side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(self.side):
                    if update_timing is not None:
                        update_timing[0].record()
                    for _ in range(self.updates_per_step):
                        self._update()
                    if update_timing is not None:
                        update_timing[1].record()
                self.pending = True
            else:
                if update_timing is not None:
                    update_timing[0].record()
                for _ in range(self.updates_per_step):
                    self._update()
                if update_timing is not None:
                    update_timing[1].record()
        if self.poll_every and self.decisions % self.poll_every == 0:
            self.poll_episodes()
        if self.check_every and self.decisions % self.check_every == 0:
            self.check()
        return r, rm, done

    def flush(self):
        """Join an in-flight update (overlap=True) and apply its refresh."""
        if self.pending:
            torch.cuda.current_stream(self.device).wait_stream(self.side)
            self.pending = False
            if self.refresh_due:
                self._refresh()
                self.refresh_due = False

    # ---- episodes -------------------------------------------------------------------
    def poll_episodes(self):
        """Drain this rank's finished episodes and hand them to the episode book
        (gather over ranks, exploiter checkpoints, scalars; episodes.EpisodeBook).
        Returns the gathered table.  Every rank must call it (a collective)."""
        return self.book.poll(self.rollout.episodes.drain())

    def _save_exploiter(self, counter, reward):
        """explorers.py:75,150-152: the exploiters' model under
        save_dir/exploiting_virtual_thread_<p_id>, p_id the first virtual
        exploiter's: its index 0 plus num_threads_exploiting
        (training/managers.py:238-255; num_threads_exploring_virtual only
        shifts its TCP port), so exploiting_virtual_thread_0 under
        config.json, the directory the reference's submit and afterlearn
        configs load from."""
        p_id = self.config['training'].get('num_threads_exploiting', 0)
        return self.save(os.path.join(self.save_dir, 'exploiting_virtual_thread_%d' % p_id),
                         counter, reward)

    def save(self, directory, episode, reward):
        """The exploiters' checkpoint (training/explorers.py:142-152): the
        target networks the exploiting envs act with, in the reference's
        layout (aido1_amd/checkpoint.py).  Returns the episode directory."""
        return self.trainer.save(directory, episode, reward, target=True)

    def load(self, directory):
        """Start from a checkpoint (the reference's or save()'s): online and
        target networks, then the acting copies."""
        self.trainer.load(directory)
        self._refresh()

    def check(self):
        """Synchronise and raise if anything went wrong since the last check:
        guard.NonFiniteError naming the first stages that produced NaN / Inf
        (rollout actor outputs, rewards, the sampled batch, each stage of the
        update, the TD errors), or the replay's rejected priorities
        (update_priorities' asserts, counted on the device).  Returns the
        guard's record."""
        self.flush()
        r = self.guard.check('training loop')
        if self.prioritized:
            self.replay.check()
        return r

    def _refresh(self):
        self.rollout.load_actor(self.trainer.actor)
        self.rollout.load_exploit_actor(self.trainer.target_actor)

    def _update(self):
        if self.prioritized and self.trainer.dtype == torch.float32:
            # the sampled rows gathered straight into the update's inputs
            # (one dt_frame_gather launch, replay.gather_into)
            idx, _w = self.replay.sample_indices(self.batch_size, self.beta)
            self.replay.gather_into(idx, self.trainer.static_inputs(self.batch_size))
            self.metrics, info = self.trainer.update_prepared()
        elif self.prioritized:
            obs, act, rew, nxt, done, _w, idx = self.replay.sample(self.batch_size, self.beta)
            self.metrics, info = self.trainer.update((obs, act, rew, nxt, done))
        else:
            obs, act, rew, nxt, done = self.replay.sample(self.batch_size)
            self.metrics, info = self.trainer.update((obs, act, rew, nxt, done))
        if self.prioritized:   # |td| + eps formed in the tree kernel (dt_per_update_td)
            self.replay.update_priorities_td(idx, info['td_error'], PRIORITY_EPS)
        self.updates += 1
        if self.updates % self.refresh_every == 0:
            if self.side is not None:
                self.refresh_due = True     # applied on the main stream (step / flush)
            else:
                self._refresh()
