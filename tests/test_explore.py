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


def _explorer_fixture():
    return golden('explorer.json')['explorers']


def test_explorer_loop_matches_reference_fixture():
    """The reference's own SingleThreadExplorer._explore_episode (training/
    explorers.py:164-213), recorded in tests/golden/explorer.json with every
    draw of its loop: the batched restatement (explore.py: OU sample ->
    DDPG.act noise / every-second-random -> the wrapper's in-place tanh map),
    fed those draws and the recorded actor outputs, reproduces each decision's
    action and stored replay action bit for bit, for exploring (even and odd
    p_id) and exploiting explorers, across episodes (OU reset per episode,
    sigma annealing carried over)."""
    from aido1_amd.env_wrappers import map_tanh_in_place
    from aido1_amd.explore import OUNoise, act, explore_actions
    cfg = golden('reference_config.json')
    for ex in _explorer_fixture():
        exploit = ex['exploration_type'].startswith('exploiting')
        ou = OUNoise.from_config(cfg, 1)
        ids = torch.tensor([ex['p_id']])
        for epi in ex['episodes']:
            ou.reset_states()
            assert float(ou.n_steps[0]) == epi['ou_steps_before']
            eps = torch.tensor([epi['epsilon']], dtype=torch.float64)
            for st in epi['steps']:
                normals = torch.tensor([st['normals']], dtype=torch.float64)
                out = torch.tensor([st.get('actor_out', [0.0, 0.0])], dtype=torch.float32)
                if exploit:
                    ou.sample(normals)          # drawn every step, unused (explorers.py:178)
                    a = act(out, None, 'tanh')
                else:
                    coin = torch.tensor([st['coin']], dtype=torch.float64) if 'coin' in st \
                        else torch.tensor([1.0], dtype=torch.float64)
                    uni = torch.tensor([st.get('random', [0.0, 0.0])], dtype=torch.float32)
                    a = explore_actions(out, ou, eps, ids, cfg, head='tanh',
                                        draws=(normals, coin, uni))
                assert a.view(-1).tolist() == [float(np.float32(v)) for v in st['action']], st
                map_tanh_in_place(a)
                assert a.view(-1).tolist() == [float(np.float32(v)) for v in st['replay_action']]
