"""Exploration pieces against the reference's golden vectors
(tests/golden/random_process.json: OU samples from numpy's global RNG with the
normals it drew, and the decay curves of utils/util.py)."""
import numpy as np
import torch

from conftest import golden


def test_ou_matches_reference_given_its_normals():
    from aido1_amd.explore import OUNoise
    fx = golden('random_process.json')
    ou = OUNoise(1, size=2, theta=0.15, mu=0.0, sigma=0.3, sigma_min=0.15)
    normals = torch.tensor(fx['normals'], dtype=torch.float64)
    for t, ref in enumerate(fx['ou']):
        got = ou.sample(normals[t].view(1, 2))[0].numpy()
        assert np.array_equal(got, np.array(ref, np.float32)), t


def test_decay_curves():
    from aido1_amd.explore import create_decay_fn
    fx = golden('random_process.json')
    steps = fx['decay_steps']
    cases = {
        'cycle': dict(initial_value=0.5, final_value=0.025, cycle_len=32, num_cycles=24000 // 32),
        'linear': dict(initial_value=0.002, final_value=1e-5, max_step=4000000),
        'exponential': dict(initial_value=1.0, final_value=0.01, max_step=1000, updates=10),
        'cyclic_cosine': dict(initial_value=1.0, final_value=0.1, period_base=10,
                              period_modifier=2)}
    for kind, kw in cases.items():
        fn = create_decay_fn(kind, **kw)
        assert [float(fn(s)) for s in steps] == fx['decay'][kind], kind


def test_act_clip_and_noise_doubling():
    from aido1_amd.explore import act
    out = torch.tensor([[0.5, -0.9], [0.0, 0.0]])
    noise = torch.tensor([[0.3, -0.1], [0.1, 0.2]])
    a = act(out, noise, 'tanh')
    assert torch.allclose(a, torch.tensor([[1.0, -1.0], [0.2, 0.4]]))
    a = act(out, noise, 'sigmoid')
    assert torch.allclose(a, torch.tensor([[0.8, 0.0], [0.1, 0.2]]))


def test_every_second_random():
    from aido1_amd.explore import OUNoise, explore_actions
    cfg = golden('reference_config.json')
    n = 4000
    ou = OUNoise.from_config(cfg, n)
    eps = torch.full((n,), 0.5)
    ids = torch.arange(n)
    out = torch.zeros(n, 2)
    a = explore_actions(out, ou, eps, ids, cfg, generator=torch.Generator().manual_seed(0))
    odd_rand = ((a[1::2] >= 0) & (a[1::2] < 1)).all(1) & (a[1::2].abs() > 0.5).all(1)
    assert not odd_rand.any()           # odd explorers never take the random branch
    frac = ((a[0::2] >= 0).all(1) & (a[0::2] < 1).all(1)).float().mean().item()
    assert 0.2 < frac < 0.45            # ~epsilon_ratio * eps = 0.25 (+ noise hits)
