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
RandomState, the coin (float64) and uniforms likewise; tests pin the
arithmetic and the loop's order of draws by feeding the reference's own
(tests/golden/explorer.json).
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
    """DDPG.act on a batch of actor outputs (models/ddpg/model.py:74-102).  noise
    is float64 (epsilon is an np.float64 there, so epsilon * sample is float64
    under numpy 2), and `action += noise` adds in float64 and rounds once to
    the float32 action."""
    a = actor_out
    if noise is not None:
        a = (a.double() + (2 * noise if head == 'tanh' else noise)).float()
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


def explore_actions(actor_out, ou, epsilon, explorer_id, config, generator=None, head='tanh',
                    draws=None):
    """training/explorers.py:178-194 for a batch: epsilon [n] float64 tensor,
    explorer_id [n] int tensor (the p_id each env plays).  draws: optional
    (normals [n, 2] f64, coin [n] f64, uniforms [n, 2] f32) to use instead of
    the generator's (tests inject the reference's own draws)."""
    t = config['training']
    normals, coin, u = draws if draws is not None else (None, None, None)
    noise = epsilon.double().unsqueeze(1) * ou.sample(normals).double()
    a = act(actor_out, noise, head)
    if t.get('every_second_random'):
        n = actor_out.shape[0]
        dev = actor_out.device
        if coin is None:
            coin = torch.rand(n, dtype=torch.float64, device=dev, generator=generator)
        rnd = (explorer_id % 2 == 0) & (coin < t['epsilon_ratio'] * epsilon.double())
        if u is None:
            u = torch.rand(n, actor_out.shape[1], device=dev, generator=generator)
        a = torch.where(rnd.unsqueeze(1), u, a)
    return a


_HEADS = {'tanh': 0, 'sigmoid': 1}


class FusedExplore:
    """explore_actions + rollout.CycleEpsilon (+ the post-step OU reset and
    episode count) as the dt_explore / dt_explore_done HIP kernels
    (include/dtactor.h): one launch each instead of ~25 element-wise torch
    kernels per decision.  The random numbers are the torch restatement's own
    draws in its order (randn [n, 2] f64 for the OU normals, then rand [n] f64 and
    rand [n, 2] f32 for every_second_random), so for one generator state both
    paths produce the same actions and states bit for bit
    (tests/test_gpu_explore.py)."""

    def __init__(self, config, ou, cycle_eps, explorer_id, head='tanh'):
        from aido1_amd import _lib
        t = config['training']
        self.L = _lib.lib()
        self.ou, self.ce, self.ids = ou, cycle_eps, explorer_id.long().contiguous()
        self.every_second_random = bool(t.get('every_second_random'))
        p = _lib.DtExploreParams()
        p.pi, p.eps_span = math.pi, cycle_eps.i - cycle_eps.f
        p.eps_final, p.eps_initial = cycle_eps.f, cycle_eps.i
        p.ou_m, p.ou_c, p.ou_sigma_min = ou.m, ou.c, ou.sigma_min
        p.ou_sqrt_dt, p.ou_theta, p.ou_mu, p.ou_dt = math.sqrt(ou.dt), ou.theta, ou.mu, ou.dt
        p.eps_ratio = float(t['epsilon_ratio']) if self.every_second_random else 0.0
        p.head = _HEADS.get(head, 2)
        self.params = p
        self.tanh = head == 'tanh'
        assert ou.size == 2 and ou.x.is_contiguous() and ou.n_steps.is_contiguous()

    def __call__(self, actor_out, episode, actions, generator=None):
        """actions[:] = explore_actions(actor_out, ou, cycle_eps(episode), ...)."""
        from aido1_amd import _lib
        n, dev = self.ou.n, self.ou.x.device
        ao = actor_out.float().contiguous()
        assert ao.shape == (n, 2) and actions.shape == (n, 2) and actions.is_contiguous()
        assert episode.dtype == torch.int64 and episode.is_contiguous()
        normals = torch.randn(n, 2, dtype=torch.float64, device=dev, generator=generator)
        coin = uni = None
        if self.every_second_random:
            coin = torch.rand(n, dtype=torch.float64, device=dev, generator=generator)
            uni = torch.rand(n, 2, device=dev, generator=generator)
        rc = self.L.dt_explore(n, ao.data_ptr(), normals.data_ptr(),
                               coin.data_ptr() if coin is not None else None,
                               uni.data_ptr() if uni is not None else None,
                               self.ou.x.data_ptr(), self.ou.n_steps.data_ptr(), episode.data_ptr(),
                               self.ce.cl.data_ptr(), self.ce.max_step.data_ptr(),
                               self.ids.data_ptr(), self.params, actions.data_ptr(),
                               torch.cuda.current_stream(dev).cuda_stream)
        if rc != 0:
            raise _lib.DtError('dt_explore failed (%d)' % rc)
        return actions

    def done(self, done, episode, actions=None):
        """After the step: the wrapper's tanh map of `actions` (when given and
        the head is tanh), then OU reset + episode += 1 where done."""
        from aido1_amd import _lib
        n, dev = self.ou.n, self.ou.x.device
        assert done.dtype == torch.uint8 and done.numel() == n and done.is_contiguous()
        tm = int(actions is not None and self.tanh)
        rc = self.L.dt_explore_done(n, done.data_ptr(), self.ou.x.data_ptr(), episode.data_ptr(),
                                    actions.data_ptr() if tm else None, tm,
                                    torch.cuda.current_stream(dev).cuda_stream)
        if rc != 0:
            raise _lib.DtError('dt_explore_done failed (%d)' % rc)
