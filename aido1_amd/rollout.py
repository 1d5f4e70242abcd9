"""Actor-in-loop batched rollout (BASELINE configs[3]).

One GPU runs `n_envs` environments split over maps (mixed small_loop /
zigzag), all rendering into ONE shared frame ring so one actor forward covers
every exploring env.  Per decision:

  actor (fp16 MFMA, ring read zero-copy; actor_mode 'reference' = the reference's
  train-mode batch-of-one BatchNorm + live dropout, 'eval' = BN folded)  -> DDPG.act noise / every-
  second-random (explore.py)  -> dt_step per map handle (tanh head mapping,
  repeat 3, reward shaping, respawn) -> dt_render per handle into the ring
  (+ line masks) -> OU reset for finished envs

which is SingleThreadExplorer._explore_episode's loop body
(training/explorers.py:177-211) for thousands of explorers at once.

Exploring and exploiting explorers (config.json:183-186: 7 exploring_virtual +
1 exploiting_virtual): the last n_exploit envs (n / 8 by default) are
exploiters.  They act with their own copy of the weights (load_exploit_actor;
TrainLoop gives it the target actor, which the reference's exploiters
hard-copy, explorers.py:104-105) with epsilon 0: no noise, no random actions,
the action the clipped actor output (explorers.py:116, 182-184).  The OU
process still advances for them, as the reference samples it every step.

frames='index' (the default) keeps the ring as palette-index frames (u8,
render.py): the renderer writes a quarter of the bytes, the actor's first conv
reads a quarter (dt_conv1_index_split), the replay's frame store keeps u8
frames, and every consumer sees the same grey values bit for bit
(stack() decodes; frames='gray' keeps float32 grey frames).
"""
import math

import numpy as np
import torch

from aido1_amd.actor import ConfigActor, FusedActor
from aido1_amd.config import EnvConfig
from aido1_amd.episodes import EpisodeTracker
from aido1_amd.env_wrappers import map_tanh_in_place
from aido1_amd.explore import FusedExplore, OUNoise, act, explore_actions
from aido1_amd.render import FRAME_DTYPES, H, W, RenderOutput, as_gray
from aido1_amd.vec_env import StepOutput, VecEnv


class CycleEpsilon:
    """Vectorised EpsilonSchedule: per-env cycle length in [L/2, 2L]
    (explorers.py:92-99), epsilon = clip(cycle_decay(episode), final, initial)."""

    def __init__(self, config, n, device, generator=None):
        t = config['training']
        L = t['epsilon_cycle_len']
        self.i, self.f = t['initial_epsilon'], t['final_epsilon']
        self.cl = torch.randint(L // 2, 2 * L + 1, (n,), device=device,
                                generator=generator).double()
        self.max_step = self.cl * torch.floor(t['max_episodes'] / self.cl)

    def __call__(self, episodes):
        ep = episodes.double()
        rel = 1.0 - ep / self.max_step
        cosv = 0.5 * (torch.cos(math.pi * torch.remainder(ep, self.cl) / self.cl) + 1.0)
        return (cosv * (self.i - self.f) * rel + self.f).clamp(self.f, self.i)


class ActorRollout:
    def __init__(self, config, n_envs=4096, maps=('small_loop', 'zigzag'), device=0, seed=1234,
                 env_id_base=0, actor=None, dtype=torch.float32, masks=True,
                 actor_mode='reference', fused_explore=True, n_exploit=None, guard=None,
                 frames='index'):
        self.config = config
        self.guard = guard      # non-finite guard (guard.py): actor outputs, rewards
        self.device = torch.device('cuda', device)
        self.n = n_envs
        k = len(maps)
        sizes = [n_envs // k + (1 if i < n_envs % k else 0) for i in range(k)]
        self.frames = frames
        self.ring = torch.zeros(n_envs, 3, H, W, dtype=FRAME_DTYPES[frames], device=self.device)
        self.masks = torch.zeros(n_envs, 4, H, W, dtype=torch.uint8, device=self.device) \
            if masks else None
        self.actions = torch.zeros(n_envs, 2, dtype=torch.float32, device=self.device)
        self.reward = torch.zeros(n_envs, dtype=torch.float64, device=self.device)
        self.reward_mod = torch.zeros(n_envs, dtype=torch.float64, device=self.device)
        self.done = torch.zeros(n_envs, dtype=torch.uint8, device=self.device)
        self.envs, self.outs, self.renders, self.slices = [], [], [], []
        head = config['model']['actor'][-1]['modules'][-1][-1]['name']
        self.head = head
        off = 0
        for m, sz in zip(maps, sizes):
            ec = EnvConfig.from_reference_config(config, map_name=m)
            env = VecEnv(sz, seed=seed, device=device, config=ec, env_id_base=env_id_base + off)
            sl = slice(off, off + sz)
            out = StepOutput(sz, self.device, lanepos=False, tile=False)
            out.reward, out.reward_mod, out.done = self.reward[sl], self.reward_mod[sl], \
                self.done[sl]
            ro = RenderOutput(sz, self.device, slots=3, ring=self.ring[sl],
                              masks=False, frames=frames)
            if masks:
                ro.masks = self.masks[sl]
            self.envs.append(env)
            self.outs.append(out)
            self.renders.append(ro)
            self.slices.append(sl)
            off += sz
        if actor is None:
            actor = ConfigActor(config['model']['actor'])
        self.actor_mode = actor_mode
        self.actor_src = actor.to(self.device)     # the module the acting copies derive from
        self.actor = FusedActor(self.actor_src, dtype=dtype, mode=actor_mode)
        if n_exploit is None:
            t = config['training']
            n_xpl = t.get('num_threads_exploiting', 0) + t.get('num_threads_exploiting_virtual', 0)
            n_exp = t.get('num_threads_exploring', 0) + t.get('num_threads_exploring_virtual', 0)
            n_exploit = (n_envs * n_xpl) // (n_xpl + n_exp) if n_xpl + n_exp else 0
        self.n_exploit = int(n_exploit)
        self.n_explore = n_envs - self.n_exploit
        self.exploit_actor = FusedActor(actor, dtype=dtype, mode=actor_mode) \
            if self.n_exploit else None
        self.actor_out = torch.zeros(n_envs, 2, dtype=torch.float32, device=self.device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed + 17 * env_id_base)
        self.ou = OUNoise.from_config(config, n_envs, device=self.device, generator=self.gen)
        self.eps = CycleEpsilon(config, n_envs, self.device, generator=self.gen)
        self.episode = torch.zeros(n_envs, dtype=torch.int64, device=self.device)
        # the p_id parity decides every_second_random; exploiters get odd ids
        # (their actions are replaced by the clipped actor output anyway)
        ids = torch.arange(env_id_base, env_id_base + n_envs, device=self.device)
        ids[self.n_explore:] = ids[self.n_explore:] | 1
        self.explorer_id = ids
        self.actor_events = None
        # dt_explore (include/dtactor.h); fused_explore=False keeps the torch
        # restatement (explore.py), which draws the same numbers
        self.fx = FusedExplore(config, self.ou, self.eps, self.explorer_id, head=head) \
            if fused_explore else None
        # the explorers' episode sums and finished-episode records
        # (explorers.py:118-123, 202-204; aido1_amd/episodes.py)
        self.episodes = EpisodeTracker(n_envs, self.device)

    def reset(self):
        for env, ro in zip(self.envs, self.renders):
            env.reset()
            ro.restart()
            env.render_into(ro)
        self.ou.reset_states()
        self.episode.zero_()
        self.episodes.reset()       # every env starts a new episode

    def order(self):
        return self.renders[0].order()

    def stack(self, raw=False):
        """[n, 3, 120, 160] oldest-first observation (a copy of the ring), grey
        float32; raw=True keeps the ring's dtype (palette-index bytes)."""
        st = self.ring[:, self.order()]
        return st if raw else as_gray(st)

    def gray_ring(self):
        """The ring as grey float32 frames (decoded: a copy for index frames)."""
        return as_gray(self.ring)

    def load_actor(self, actor):
        """The exploring envs act with `actor`'s current weights from the next
        decision on (the reference's model workers act with the trained
        model, training/managers.py:182-208)."""
        self.actor.refresh(actor)

    def load_exploit_actor(self, actor):
        """The exploiting envs act with `actor`'s weights (explorers.py:104-105
        hard-copies the target model at every episode start; here the whole
        exploiter block is refreshed at once)."""
        if self.exploit_actor is not None:
            self.exploit_actor.refresh(actor)

    def _step_envs(self):
        """dt_step + dt_render of every map's envs.  Several maps (config 4's
        small_loop / zigzag mix) run on their own streams, side by side: each
        launch covers only its share of the envs (a latency-bound step, a
        render filling part of the chip)."""
        groups = list(zip(self.envs, self.outs, self.renders, self.slices))
        if len(groups) == 1 or self.device.type != 'cuda':
            for env, o, ro, sl in groups:
                env.step_into(self.actions[sl], o)
                env.render_into(ro, fresh=o.done)
            return
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, '_env_streams', None) is None:
            self._env_streams = [torch.cuda.Stream(self.device) for _ in groups[1:]]
        streams = [cur] + self._env_streams
        for s in self._env_streams:
            s.wait_stream(cur)
        for s, (env, o, ro, sl) in zip(streams, groups):
            with torch.cuda.stream(s):
                env.step_into(self.actions[sl], o)
                env.render_into(ro, fresh=o.done)
        for s in self._env_streams:
            cur.wait_stream(s)

    def step(self, timing=None):
        """One decision for every env; returns (reward, reward_mod, done) views."""
        if timing is not None:
            timing[0].record()
        ne = self.n_explore
        if self.exploit_actor is None:
            out = self.actor(self.ring, self.order())
        else:
            # one launch per convolution over both weight sets (dt_conv*_split)
            out = self.actor.forward_pair(self.exploit_actor, self.ring, self.order(), ne,
                                          out=self.actor_out)
        if timing is not None:
            timing[1].record()
        if self.guard is not None:   # before DDPG.act's clip, which would hide a NaN
            self.guard.scan('actor_out', out)
        if self.fx is not None:
            self.fx(out, self.episode, self.actions, generator=self.gen)
        else:
            eps = self.eps(self.episode)
            self.actions.copy_(explore_actions(out, self.ou, eps, self.explorer_id, self.config,
                                               generator=self.gen, head=self.head))
        if self.exploit_actor is not None:   # epsilon 0: DDPG.act without noise
            if self.head == 'tanh':              # its clip, written in place (one kernel)
                torch.clamp(out[ne:], -1.0, 1.0, out=self.actions[ne:])
            else:
                self.actions[ne:] = act(out[ne:], None, self.head)
        self._step_envs()
        if self.guard is not None:
            self.guard.scan('env', self.reward, self.reward_mod)
        self.episodes.account(self.reward, self.reward_mod, self.done)
        if self.fx is not None:   # tanh map, OU reset and episode count in one kernel
            self.fx.done(self.done, self.episode, self.actions)
            return self.reward, self.reward_mod, self.done
        if self.head == 'tanh':   # the wrapper's in-place a/2 + 0.5 (env_wrappers.py:214-216)
            map_tanh_in_place(self.actions)
        d = self.done.bool()
        self.ou.reset_states(d)
        self.episode += d.long()
        return self.reward, self.reward_mod, self.done

    def stats(self, reset=False):
        tot = {}
        for env in self.envs:
            for k, v in env.stats(reset).items():
                tot[k] = tot.get(k, 0) + v
        return tot

    def close(self):
        for env in self.envs:
            env.close()
