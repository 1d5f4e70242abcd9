"""Deterministic, torch-version-independent weights and inputs for the actor
golden vectors (used by make_golden.py to drive the reference's actors and by
tests to drive aido1_amd's)."""
import math

import torch


def hash_u(n, salt):
    """n uniforms in [0, 1) from an integer hash (no RNG state involved)."""
    idx = torch.arange(n, dtype=torch.int64)
    h = (idx * 2654435761 + salt * 2246822519 + 374761393) % 4294967296
    h = (h ^ (h >> 15)) * 2246822519 % 4294967296
    h = h ^ (h >> 13)
    return h.double() / 4294967296.0


def formula_state_dict(state_dict):
    """Same keys/shapes as `state_dict`, values from hash_u: He-uniform weights,
    BatchNorm gamma in [0.5, 1.5), beta +-0.1, running var [0.5, 1.5), mean +-0.2."""
    sd = {}
    bn = {k.rsplit('.', 1)[0] for k in state_dict if k.endswith('running_mean')}
    for k, (name, t) in enumerate(state_dict.items()):
        n = t.numel()
        u = hash_u(n, k + 1)
        mod = name.rsplit('.', 1)[0]
        if name.endswith('num_batches_tracked'):
            sd[name] = t.clone()
        elif name.endswith('running_var'):
            sd[name] = (0.5 + u).reshape(t.shape).float()
        elif name.endswith('running_mean'):
            sd[name] = (0.2 * (2 * u - 1)).reshape(t.shape).float()
        elif mod in bn and name.endswith('weight'):
            sd[name] = (0.5 + u).reshape(t.shape).float()
        elif mod in bn and name.endswith('bias'):
            sd[name] = (0.1 * (2 * u - 1)).reshape(t.shape).float()
        else:
            fan = max(1, n // t.shape[0]) if t.dim() > 1 else 64
            sd[name] = (math.sqrt(6.0 / fan) * (2 * u - 1)).reshape(t.shape).float()
    return sd


def formula_input(n=4):
    """[n,3,120,160] float32 frames in [0,1] with per-sample brightness/gradient."""
    noise = hash_u(n * 3 * 120 * 160, 999).reshape(n, 3, 120, 160)
    r = torch.arange(120, dtype=torch.float64).view(1, 1, 120, 1) / 120
    c = torch.arange(160, dtype=torch.float64).view(1, 1, 1, 160) / 160
    b = torch.linspace(0.1, 1.0, n, dtype=torch.float64).view(n, 1, 1, 1)
    g = torch.tensor([1.0, -1.0, 0.5, -0.5] * ((n + 3) // 4), dtype=torch.float64)[:n]
    g = g.view(n, 1, 1, 1)
    return (b * (0.5 + 0.5 * g * (r - c)) * (0.7 + 0.3 * noise)).clamp(0, 1).float()


def formula_batch(n=16):
    """A replay batch (obs, actions, rewards, next_obs, dones) as numpy, the
    layout DDPGTrainer.update receives (training/trainers.py:143-146)."""
    obs = formula_input(n)
    nxt = obs.roll(1, 0).flip(3).contiguous()
    act = hash_u(2 * n, 4242).reshape(n, 2).float()
    rew = (20 * hash_u(n, 4343) - 10).float()
    done = (torch.arange(n) % 5 == 3)
    return obs.numpy(), act.numpy(), rew.numpy(), nxt.numpy(), done.numpy()


def param_summary(module):
    """Per-tensor (sum, abs-sum, 32 strided elements) of a state_dict — small
    enough for a fixture, dense enough to catch a wrong update."""
    out = {}
    for k, t in module.state_dict().items():
        v = t.detach().double().reshape(-1)
        stride = max(1, v.numel() // 32)
        out[k] = [float(v.sum()), float(v.abs().sum())] + [float(x) for x in v[::stride][:32]]
    return out
