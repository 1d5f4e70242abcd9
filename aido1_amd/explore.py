"""Batched exploration for the actor-in-loop rollout.

Restates, with a leading env dimension on the GPU:
  - OrnsteinUhlenbeckProcess (utils/random_process.py:30-61): x += theta (mu - x)
    dt + sigma_t sqrt(dt) N(0, 1), sigma annealed linearly from sigma to
    sigma_min over n_steps_annealing samples, float64 state, float32 output;
    reset_states() per episode (training/explorers.py:170);
  - the decay schedules of utils/util.py:22-74 (create_decay_fn);
  - DDPG.act (models/ddpg/model.py:74-102): action = actor(obs) + noise
    (noise doubled for a tanh head), clipped to the head's range;
  - SingleThreadExplorer's action choice (training/explorers.py:178-194): noise
    = epsilon * OU sample; with every_second_random, explorers with an even id
    take a U[0,1)^2 action with probability epsilon_ratio * epsilon.
The normals come from torch's Philox generator instead of numpy's global
RandomState (tests pin the arithmetic by feeding the reference's normals).
"""
import math

import numpy as np
import torch


# ---- utils/util.py:22-74 -------------------------------------------------------------
def create_decay_fn(decay_type, **kw):
    if decay_type == 'linear':
        i, f, m = kw['initial_value'], kw['final_value'], kw['max_step']

        def fn(step):
            rel = 1. - step / m
            return i * rel + f * (1. - rel)
        return fn
    if decay_type == 'cycle':
        i, f, cl, nc = kw['initial_value'], kw['final_value'], kw['cycle_len'], kw['num_cycles']
        max_step = cl * nc

        def fn(step):
            rel = 1. - step / max_step
            cosv = 0.5 * (np.cos(np.pi * np.mod(step, cl) / cl) + 1.0)
            return cosv * (i - f) * rel + f
        return fn
    if decay_type == 'exponential':
        i, f, m, u = kw['initial_value'], kw['final_value'], kw['max_step'], kw['updates']
        coeff = (f / i) ** (1 / u)
        every = m / u

        def fn(step):
            return i * (coeff ** int(step / every))
        return fn
    if decay_type == 'cyclic_cosine':
        i, f, base = kw['initial_value'], kw['final_value'], kw['period_base']
        mod = kw.get('period_modifier', 1)
        lm = np.log(mod)

        def fn(step):
            if abs(lm) > 1e-3 and step // base > 0:
                cl = base * mod ** (int(np.log(step / base) / lm))
            else:
                cl = base
            return f + (i - f) * 0.5 * (1 + np.cos(np.pi * (step % cl) / cl))
        return fn
    raise NotImplementedError(decay_type)


class OUNoise:
    """N independent OrnsteinUhlenbeckProcess instances on one device."""

    def __init__(self, n, size=2, theta=0.15, mu=0.0, sigma=0.3, sigma_min=None, dt=1e-2,
                 n_steps_annealing=int(1e6), device='cpu', generator=None):
        self.n, self.size = n, size
        self.theta, self.mu, self.dt = theta, mu, dt
        if sigma_min is not None:
            self.m = -float(sigma - sigma_min) / float(n_steps_annealing)
            self.c = sigma
            self.sigma_min = sigma_min
        else:
            self.m, self.c, self.sigma_min = 0., sigma, sigma
        self.device = torch.device(device)
        self.gen = generator
        self.x = torch.zeros(n, size, dtype=torch.float64, device=self.device)
        self.n_steps = torch.zeros(n, dtype=torch.float64, device=self.device)

    @classmethod
    def from_config(cls, config, n, device='cpu', generator=None):
        t = config['training']
        return cls(n, size=config['model'].get('num_action', 2), theta=t['rp_theta'],
                   mu=t['rp_mu'], sigma=t['rp_sigma'], sigma_min=t['rp_sigma_min'],
                   device=device, generator=generator)

    def current_sigma(self):
        return torch.clamp(self.m * self.n_steps + self.c, min=self.sigma_min)

    def sample(self, normals=None):
        if normals is None:
            normals = torch.randn(self.n, self.size, dtype=torch.float64, device=self.device,
                                  generator=self.gen)
        x = self.x + self.theta * (self.mu - self.x) * self.dt + \
            self.current_sigma().unsqueeze(1) * math.sqrt(self.dt) * normals
        self.x = x
        self.n_steps += 1
        return x.float()

    def reset_states(self, mask=None):
        if mask is None:
            self.x.zero_()
        else:
            self.x[mask.bool()] = 0.0


def act(actor_out, noise=None, head='tanh'):
    """DDPG.act on a batch of actor outputs (models/ddpg/model.py:74-102)."""
    a = actor_out
    if noise is not None:
        a = a + (2 * noise if head == 'tanh' else noise)
    if head == 'tanh':
        return a.clamp(-1.0, 1.0)
    if head == 'sigmoid':
        return a.clamp(0.0, 1.0)
    return a


class EpsilonSchedule:
    """Per-env epsilon of SingleThreadExplorer (training/explorers.py:92-111):
    each explorer draws its cycle length in [len/2, 2 len]; epsilon =
    min(initial, max(final, cycle_decay(episode)))."""

    def __init__(self, config, n, rng=None):
        t = config['training']
        rng = rng or np.random.default_rng(t['global_seed'])
        L = t['epsilon_cycle_len']
        self.init, self.final = t['initial_epsilon'], t['final_epsilon']
        self.cycle = rng.integers(L // 2, L * 2 + 1, n)
        self.fns = [create_decay_fn('cycle', initial_value=self.init, final_value=self.final,
                                    cycle_len=int(c), num_cycles=t['max_episodes'] // int(c))
                    for c in self.cycle]

    def __call__(self, episodes):
        eps = [min(self.init, max(self.final, fn(int(e)))) for fn, e in zip(self.fns, episodes)]
        return np.asarray(eps, np.float64)


def explore_actions(actor_out, ou, epsilon, explorer_id, config, generator=None, head='tanh'):
    """training/explorers.py:178-194 for a batch: epsilon [n] tensor, explorer_id
    [n] int tensor (the p_id each env plays)."""
    t = config['training']
    noise = (epsilon.unsqueeze(1) * ou.sample()).float()
    a = act(actor_out, noise, head)
    if t.get('every_second_random'):
        n = actor_out.shape[0]
        dev = actor_out.device
        coin = torch.rand(n, device=dev, generator=generator)
        rnd = (explorer_id % 2 == 0) & (coin < t['epsilon_ratio'] * epsilon.float())
        u = torch.rand(n, actor_out.shape[1], device=dev, generator=generator)
        a = torch.where(rnd.unsqueeze(1), u, a)
    return a
