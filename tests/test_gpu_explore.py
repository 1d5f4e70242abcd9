"""A20 on the GPU: DDPG.act noise / epsilon / every-second-random on cuda
against the reference's golden vectors (tests/golden/random_process.json:
OrnsteinUhlenbeckProcess.sample given the normals numpy drew,
utils/random_process.py:42-47, and the cycle decay of utils/util.py:20-74 that
training/explorers.py:92-114 clips into epsilon).  The same code runs in
ActorRollout for 4096 explorers at once."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def test_ou_on_gpu_matches_reference_given_its_normals(gpu):
    """One OU process per env, 4096 envs, every env fed the reference's normals:
    each row reproduces the reference's samples exactly (f64 +, *, sqrt)."""
    from aido1_amd.explore import OUNoise
    fx = golden('random_process.json')
    n = 4096
    ou = OUNoise(n, size=2, theta=0.15, mu=0.0, sigma=0.3, sigma_min=0.15, device=gpu)
    normals = torch.tensor(fx['normals'], dtype=torch.float64, device=gpu)
    got = []
    for t in range(len(fx['ou'])):
        got.append(ou.sample(normals[t].view(1, 2).expand(n, 2)))
    got = torch.stack(got).cpu().numpy()                     # [T, n, 2] f32
    ref = np.asarray(fx['ou'], np.float32)                   # [T, 2]
    assert np.array_equal(got, np.broadcast_to(ref[:, None, :], got.shape))
    # sigma annealing state after T samples
    assert float(ou.n_steps[0]) == len(fx['ou'])


def test_ou_reset_of_finished_envs_on_gpu(gpu):
    from aido1_amd.explore import OUNoise
    fx = golden('random_process.json')
    ou = OUNoise(8, size=2, theta=0.15, mu=0.0, sigma=0.3, sigma_min=0.15, device=gpu)
    normals = torch.tensor(fx['normals'], dtype=torch.float64, device=gpu)
    for t in range(5):
        ou.sample(normals[t].view(1, 2).expand(8, 2))
    mask = torch.tensor([1, 0, 1, 0, 0, 0, 0, 1], dtype=torch.uint8, device=gpu)
    ou.reset_states(mask)
    x = ou.x.cpu().numpy()
    assert (x[[0, 2, 7]] == 0).all()
    assert np.array_equal(x[1], np.asarray(x[3]))           # untouched rows keep the state
    assert (x[[1, 3, 4, 5, 6]] != 0).all()


def test_cycle_epsilon_on_gpu_matches_decay_fn(gpu):
    """CycleEpsilon (rollout.py) on cuda vs the reference's cycle decay with the
    golden parameters (cycle_len 32, 24000 episodes); GPU cos may differ from
    libm's in the last place."""
    from aido1_amd.rollout import CycleEpsilon
    fx = golden('random_process.json')
    cfg = golden('reference_config.json')
    n = 4096
    ce = CycleEpsilon(cfg, n, gpu)
    ce.cl.fill_(32.0)
    ce.max_step.fill_(32.0 * (24000 // 32))
    steps = torch.tensor(fx['decay_steps'], dtype=torch.int64, device=gpu)
    for s, ref in zip(steps, fx['decay']['cycle']):
        got = ce(s.expand(n)).cpu().numpy()
        assert np.max(np.abs(got - ref)) <= 1e-15, (int(s), got[0], ref)


def test_cycle_lengths_drawn_in_reference_range(gpu):
    from aido1_amd.rollout import CycleEpsilon
    cfg = golden('reference_config.json')
    L = cfg['training']['epsilon_cycle_len']
    ce = CycleEpsilon(cfg, 4096, gpu)
    cl = ce.cl.cpu().numpy()
    assert cl.min() >= L // 2 and cl.max() <= 2 * L          # explorers.py:92-99
    assert len(np.unique(cl)) > L                             # drawn per explorer


def test_explore_actions_on_gpu(gpu):
    """explorers.py:178-194 for 4096 explorers on cuda: the non-random rows are
    DDPG.act (actor + 2*eps*OU for a tanh head, clipped to [-1, 1],
    models/ddpg/model.py:74-102) of the OU state the call advanced; the random
    rows are only even explorer ids, at about epsilon_ratio * epsilon."""
    from aido1_amd.explore import OUNoise, act, explore_actions
    cfg = golden('reference_config.json')
    n = 4096
    g = torch.Generator(device=gpu)
    g.manual_seed(0)
    ou = OUNoise.from_config(cfg, n, device=gpu, generator=g)
    eps = torch.full((n,), 0.5, dtype=torch.float64, device=gpu)
    ids = torch.arange(n, device=gpu)
    out = torch.rand(n, 2, device=gpu, generator=g) * 2.4 - 1.2
    a = explore_actions(out, ou, eps, ids, cfg, generator=g, head='tanh')
    det = act(out, eps.unsqueeze(1) * ou.x.float().double(), 'tanh')
    same = (a == det).all(1)
    odd = ids % 2 == 1
    assert same[odd].all()                                    # odd: never random
    rnd = ~same
    assert not rnd[odd].any()
    frac = rnd[~odd].float().mean().item()
    ratio = cfg['training']['epsilon_ratio'] * 0.5
    assert abs(frac - ratio) < 0.05, frac
    r = a[rnd]
    assert ((r >= 0) & (r < 1)).all()                        # U[0,1)^2 random action
    assert (a.abs() <= 1.0).all()


@pytest.mark.parametrize('esr', [True, False])
def test_fused_explore_matches_torch_path(gpu, esr):
    """dt_explore / dt_explore_done (include/dtactor.h, the rollout's product
    path) vs the torch restatement above (explore_actions + CycleEpsilon +
    map_tanh_in_place + reset_states), 4096 explorers over 6 decisions with
    done envs in between: same generator state -> identical actions, OU
    states, annealing counters and episode counts (bit for bit)."""
    import copy
    from aido1_amd.env_wrappers import map_tanh_in_place
    from aido1_amd.explore import FusedExplore, OUNoise, explore_actions
    from aido1_amd.rollout import CycleEpsilon
    cfg = copy.deepcopy(golden('reference_config.json'))
    cfg['training']['every_second_random'] = esr
    n = 4096

    def build():
        g = torch.Generator(device=gpu)
        g.manual_seed(5)
        return g, OUNoise.from_config(cfg, n, device=gpu, generator=g), \
            CycleEpsilon(cfg, n, gpu, generator=g)
    ga, oua, cea = build()
    gb, oub, ceb = build()
    assert torch.equal(cea.cl, ceb.cl)
    g3 = torch.Generator(device=gpu)
    g3.manual_seed(11)
    ids = torch.arange(n, device=gpu)
    epa = torch.randint(0, 5000, (n,), device=gpu, generator=g3)
    epb = epa.clone()
    fx = FusedExplore(cfg, oub, ceb, ids, head='tanh')
    actb = torch.empty(n, 2, device=gpu)
    n_rand = 0
    for t in range(6):
        out = torch.rand(n, 2, device=gpu, generator=g3) * 2.4 - 1.2
        a = explore_actions(out, oua, cea(epa), ids, cfg, generator=ga, head='tanh')
        fx(out, epb, actb, generator=gb)
        assert torch.equal(a, actb), t
        assert torch.equal(oua.x, oub.x) and torch.equal(oua.n_steps, oub.n_steps), t
        n_rand += int(((a >= 0) & (a < 1)).all(1).sum())
        done = (torch.rand(n, device=gpu, generator=g3) < 0.2).to(torch.uint8)
        map_tanh_in_place(a)
        oua.reset_states(done.bool())
        epa += done.long()
        fx.done(done, epb, actb)
        assert torch.equal(a, actb) and torch.equal(epa, epb) and torch.equal(oua.x, oub.x), t
    assert n_rand > 0


def test_dt_explore_matches_reference_explorer_loop(gpu):
    """dt_explore / dt_explore_done (the kernels ActorRollout runs) against the
    reference's own _explore_episode (tests/golden/explorer.json): the recorded
    OU normals, coin, random action and actor outputs injected, 64 copies of
    each explorer; actions, stored (mapped) actions, OU reset at episode ends
    and the epsilon of the episode counter (cycle schedule) reproduced bit for
    bit.  The exploiting explorer (explorers.py:182-184) acts with the clipped
    actor output, as ActorRollout's exploiter block does."""
    from aido1_amd.explore import FusedExplore, OUNoise
    from aido1_amd.rollout import CycleEpsilon
    cfg = golden('reference_config.json')
    m = 64
    for ex in golden('explorer.json')['explorers']:
        exploit = ex['exploration_type'].startswith('exploiting')
        ou = OUNoise.from_config(cfg, m, device=gpu)
        ce = CycleEpsilon(cfg, m, gpu)
        L = ex['cycle_len']
        ce.cl.fill_(float(L))
        ce.max_step.fill_(float(L * (cfg['training']['max_episodes'] // L)))
        ids = torch.full((m,), ex['p_id'], dtype=torch.int64, device=gpu)
        fx = FusedExplore(cfg, ou, ce, ids, head='tanh')
        episode = torch.zeros(m, dtype=torch.int64, device=gpu)
        actions = torch.zeros(m, 2, dtype=torch.float32, device=gpu)
        for epi in ex['episodes']:
            episode.fill_(epi['episode_counter'])
            ou.reset_states()
            for st in epi['steps']:
                out = torch.tensor(st.get('actor_out', [0.0, 0.0]), dtype=torch.float32,
                                   device=gpu).expand(m, 2).contiguous()
                normals = torch.tensor(st['normals'], dtype=torch.float64,
                                       device=gpu).expand(m, 2).contiguous()
                coin = torch.full((m,), st.get('coin', 1.0), dtype=torch.float64, device=gpu)
                uni = torch.tensor(st.get('random', [0.0, 0.0]), dtype=torch.float32,
                                   device=gpu).expand(m, 2).contiguous()
                rc = fx.L.dt_explore(m, out.data_ptr(), normals.data_ptr(),
                                     coin.data_ptr() if fx.every_second_random else None,
                                     uni.data_ptr(), ou.x.data_ptr(), ou.n_steps.data_ptr(),
                                     episode.data_ptr(), ce.cl.data_ptr(), ce.max_step.data_ptr(),
                                     ids.data_ptr(), fx.params, actions.data_ptr(),
                                     torch.cuda.current_stream(gpu).cuda_stream)
                assert rc == 0
                if exploit:
                    actions.copy_(out.clamp(-1.0, 1.0))
                want = torch.tensor(st['action'], dtype=torch.float32, device=gpu)
                assert torch.equal(actions, want.expand(m, 2)), (ex['p_id'], st)
                done = torch.full((m,), int(st['done']), dtype=torch.uint8, device=gpu)
                ep0 = episode.clone()
                fx.done(done, episode, actions)
                want = torch.tensor(st['replay_action'], dtype=torch.float32, device=gpu)
                assert torch.equal(actions, want.expand(m, 2))
                if st['done']:
                    assert torch.equal(episode, ep0 + 1) and not ou.x.any()
