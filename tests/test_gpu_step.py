"""GPU parity: libdtsim step/reset kernels vs the CPU oracle (C restatement).

Bar (BASELINE.json north_star): pose/reward max-abs-err <= 1e-5, tile index and
done flags bit-exact.  The kernels follow numpy's rounding sequence, so the
measured error is ulp-level (only ocml vs glibc sin/cos/acos can differ) and
the tests also assert a much tighter 1e-9 to catch regressions early.
"""
import numpy as np
import pytest
import torch

from conftest import golden, map_objects, map_rows
from oracle import dtsim_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu

TOL_SPEC = 1e-5     # north_star tolerance on pose / reward
TOL_TIGHT = 1e-9    # regression tripwire


def make_pair(n, map_name='loop_empty', seed=1234, env_base=0, **cfg_kw):
    from aido1_amd.config import EnvConfig
    from aido1_amd.vec_env import VecEnv
    ec = EnvConfig(map_name=map_name, **cfg_kw)
    env = VecEnv(n, seed=seed, config=ec, env_id_base=env_base)
    sc_kw = {k: v for k, v in cfg_kw.items() if k in R.SimConfig().__dict__}
    sc = R.SimConfig(**sc_kw)
    ob = OC.OracleBatch(map_rows(map_name), n, seed=seed, sim_config=sc,
                        auto_reset=ec.auto_reset, env_base=env_base,
                        objects=map_objects(map_name))
    return env, ob


def compare_state(env, ob, tol=TOL_TIGHT):
    g = env.get_state()
    o = ob.state()
    for k in ('x', 'z', 'angle'):
        err = np.max(np.abs(g[k] - o[k])) if len(g[k]) else 0.0
        assert err <= tol, (k, err)
    for k in ('step_count', 'env_step', 'episode'):
        assert np.array_equal(g[k], o[k]), k
    return max(float(np.max(np.abs(g[k] - o[k]))) for k in ('x', 'z', 'angle'))


def compare_out(out, ref, tol=TOL_TIGHT):
    assert np.array_equal(out.done.cpu().numpy(), ref['done'])
    assert np.array_equal(out.tile.cpu().numpy(), ref['tile'])
    r = np.max(np.abs(out.reward.cpu().numpy() - ref['reward']))
    rm = np.max(np.abs(out.reward_mod.cpu().numpy() - ref['reward_mod']))
    lp = out.lanepos.cpu().numpy()
    assert np.array_equal(np.isnan(lp), np.isnan(ref['lanepos']))
    m = ~np.isnan(lp)
    le = np.max(np.abs(lp[m] - ref['lanepos'][m])) if m.any() else 0.0
    o = np.max(np.abs(out.obs.cpu().numpy() - ref['obs']))
    assert r <= tol and rm <= tol, (r, rm)
    assert le <= tol * 1e3, le   # angle_deg = rad * 57.3
    assert o <= 1e-6, o
    return max(r, rm)


@pytest.mark.parametrize('n', [1, 63, 65, 4096])
def test_reset_bit_exact(gpu, n):
    env, ob = make_pair(n)
    env.reset()
    ob.reset()
    g = env.get_state()
    o = ob.state()
    for k in g:
        assert np.array_equal(g[k], o[k]), k
    env.check()


def test_reset_properties_full_size(gpu):
    env, _ = make_pair(4096, seed=77)
    env.reset()
    s = env.get_state()
    sim = R.SimulatorRef(map_rows('loop_empty'))
    for i in range(0, 4096, 8):
        pos = np.array([s['x'][i], 0.0, s['z'][i]])
        assert sim._valid_pose(pos, s['angle'][i], 1.3)
        lp = sim.get_lane_pos2(pos, s['angle'][i])
        assert -4 < lp.angle_deg < 4
    assert (s['episode'] == 1).all() and (s['env_step'] == 0).all()


@pytest.mark.parametrize('map_name,mode,n,steps', [
    ('loop_empty', 'wheels', 4096, 60),
    ('loop_empty', 'tanh', 1000, 40),
    ('zigzag', 'steering', 4096, 40),
    ('small_loop', 'wheels', 65, 100),
    ('intersections', 'wheels', 4096, 60),   # 3-way / 4-way tiles
    ('loop_obstacles', 'wheels', 4096, 80),  # static objects
])
def test_step_parity(gpu, map_name, mode, n, steps):
    env, ob = make_pair(n, map_name=map_name, action_mode=mode)
    env.reset()
    ob.reset()
    compare_state(env, ob, 0.0)
    rng = np.random.default_rng(11)
    lo = 0.0 if mode == 'wheels' else -1.0
    worst = 0.0
    ndone = 0
    for t in range(steps):
        a = rng.uniform(lo, 1.0, (n, 2)).astype(np.float32)
        out = env.step_into(torch.from_numpy(a).to(gpu))
        ref = ob.step(a)
        torch.cuda.synchronize()
        worst = max(worst, compare_out(out, ref))
        worst = max(worst, compare_state(env, ob))
        ndone += int(ref['done'].sum())
    assert worst <= TOL_SPEC
    assert ndone > 0  # the auto-reset path was exercised
    env.check()


def test_step_parity_variants(gpu):
    """frame_skip 2, repeat 1, measured-speed reward, width front probe, no clip."""
    for kw in (dict(frame_skip=2), dict(repeat_actions=1), dict(reward_speed_measured=True),
               dict(front_probe_length=False), dict(clip_action=False)):
        env, ob = make_pair(256, **kw)
        env.reset()
        ob.reset()
        rng = np.random.default_rng(5)
        for t in range(30):
            a = rng.uniform(-0.2, 1.3, (256, 2)).astype(np.float32)
            out = env.step_into(torch.from_numpy(a).to(gpu))
            ref = ob.step(a)
            torch.cuda.synchronize()
            compare_out(out, ref)
            compare_state(env, ob)


def test_injected_edge_states(gpu):
    """Injected states: off-road start (invalid pose), wrapper cap boundary,
    Simulator max_steps boundary, straight-line (Vl == Vr) branch."""
    n = 256
    env, ob = make_pair(n, max_steps=1000)
    env.reset()
    ob.reset()
    s = ob.state()
    rng = np.random.default_rng(2)
    ts = 0.61
    s['x'][:32] = rng.uniform(-0.3, 3.5 * ts, 32)       # anywhere, incl. off grid/grass
    s['z'][:32] = rng.uniform(-0.3, 3.5 * ts, 32)
    s['env_step'][32:64] = 1998                         # crosses max_env_steps=2000
    s['step_count'][64:96] = 998                        # crosses max_steps=1000
    s['x'][96:100] = 1.5 * ts                           # grass centre
    s['z'][96:100] = 1.5 * ts
    ob.set_state(**s)
    env.set_state(**s)
    a = rng.uniform(0, 1, (n, 2)).astype(np.float32)
    a[100:140, 1] = a[100:140, 0]                       # Vl == Vr
    out = env.step_into(torch.from_numpy(a).to(gpu))
    ref = ob.step(a)
    torch.cuda.synchronize()
    compare_out(out, ref)
    compare_state(env, ob)
    assert ref['done'][96:100].all()
    assert ref['done'][32:64].sum() > 0 and ref['done'][64:96].sum() > 0


def test_golden_env_wrapper_fixture(gpu):
    """The reference's EnvironmentWrapper trajectories (tests/golden/env_wrapper.json)
    reproduced by the kernel, n = 1."""
    from aido1_amd.config import EnvConfig
    from aido1_amd.vec_env import VecEnv
    for fx in golden('env_wrapper.json'):
        env = VecEnv(1, seed=fx['seed'],
                     config=EnvConfig(max_env_steps=fx['max_env_steps'], action_mode=fx['mode']))
        env.reset()
        env.reset()
        for st in fx['steps']:
            out = env.step_into(torch.tensor([st['action_in']], dtype=torch.float32,
                                             device=gpu))
            torch.cuda.synchronize()
            assert abs(out.reward.item() - st['reward']) <= TOL_SPEC
            assert abs(out.reward_mod.item() - st['reward_mod']) <= TOL_SPEC
            assert bool(out.done.item()) == st['done']


def test_sharded_streams_disjoint(gpu):
    """env_id_base keys the spawn stream: two shards == one big batch."""
    a, _ = make_pair(128, seed=5, env_base=0)
    b, _ = make_pair(128, seed=5, env_base=128)
    big, _ = make_pair(256, seed=5)
    for e in (a, b, big):
        e.reset()
    sa, sb, sg = a.get_state(), b.get_state(), big.get_state()
    for k in ('x', 'z', 'angle'):
        assert np.array_equal(np.concatenate([sa[k], sb[k]]), sg[k])


def test_graph_capture_matches_eager(gpu):
    env1, _ = make_pair(512, seed=9)
    env2, _ = make_pair(512, seed=9)
    env1.reset()
    env2.reset()
    torch.cuda.synchronize()
    rng = np.random.default_rng(0)
    acts = torch.from_numpy(rng.uniform(0, 1, (8, 512, 2)).astype(np.float32)).to(gpu)
    buf = torch.empty(512, 2, dtype=torch.float32, device=gpu)
    # warm up on a side stream as torch requires, then capture one step
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        pass
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        env2.step_into(buf)
    # capture does not execute: state unchanged
    for k in range(8):
        env1.step_into(acts[k])
        r1 = env1.out.reward.clone()
        buf.copy_(acts[k])
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(r1, env2.out.reward)
    for k in ('x', 'z', 'angle', 'episode'):
        assert np.array_equal(env1.get_state()[k], env2.get_state()[k])


def test_step_graph_chunks_match_eager(gpu):
    """VecEnv.capture: two replays of a 6-decision graph == 12 eager decisions
    (auto-reset on; the spawn-ahead slots advance across replays)."""
    n = 1024
    env1, _ = make_pair(n, seed=11)
    env2, _ = make_pair(n, seed=11)
    env1.reset()
    env2.reset()
    rng = np.random.default_rng(3)
    acts = torch.from_numpy(rng.uniform(0, 1, (12, n, 2)).astype(np.float32)).to(gpu)
    buf = torch.empty(6, n, 2, dtype=torch.float32, device=gpu)
    sg = env2.capture(buf)
    rewards = []
    for k in range(12):
        env1.step_into(acts[k])
        rewards.append(env1.out.reward.clone())
    for c in range(2):
        buf.copy_(acts[6 * c:6 * c + 6])
        sg.replay()
        torch.cuda.synchronize()
        assert torch.equal(rewards[6 * c + 5], env2.out.reward)
    for k in ('x', 'z', 'angle', 'episode', 'step_count', 'env_step'):
        assert np.array_equal(env1.get_state()[k], env2.get_state()[k])
    assert env1.stats() == env2.stats()
    env1.check()
    env2.check()


@pytest.mark.parametrize('k,map_name', [(1, 'loop_empty'), (7, 'loop_empty'), (16, 'loop_empty'),
                                        (20, 'loop_empty'), (30, 'zigzag'),
                                        (12, 'loop_obstacles'), (64, 'small_loop')],
                         ids=['1-loop_empty', '7-loop_empty', '16-loop_empty', '20-loop_empty',
                              '30-zigzag', '12-loop_obstacles', '64-small_loop'])
def test_step_many_matches_oracle(gpu, k, map_name):
    """dt_step_many: k decisions per launch == k oracle steps, per decision;
    three launches back to back, then an eager dt_step continues the state.
    Envs finishing more often than their ready slots cover spawn inline.
    (The fan kernel, step_fan_kernel; test_step_many_generic_path covers
    step_kernel over k decisions.)"""
    from aido1_amd.vec_env import StepOutput
    n = 4096
    env, ob = make_pair(n, map_name=map_name)
    env.reset()
    ob.reset()
    rng = np.random.default_rng(31)
    out = StepOutput(k * n, gpu, lanepos=False, tile=False)
    ndone = 0
    multi = 0
    for _ in range(3):
        a = rng.uniform(0, 1, (k, n, 2)).astype(np.float32)
        env.step_many_into(torch.from_numpy(a).to(gpu), out)
        torch.cuda.synchronize()
        rew = out.reward.view(k, n).cpu().numpy()
        rewm = out.reward_mod.view(k, n).cpu().numpy()
        done = out.done.view(k, n).cpu().numpy()
        obs = out.obs.view(k, n, 2).cpu().numpy()
        per_env = np.zeros(n, np.int64)
        for d in range(k):
            ref = ob.step(a[d])
            assert np.array_equal(done[d], ref['done']), d
            assert np.max(np.abs(rew[d] - ref['reward'])) <= TOL_TIGHT, d
            assert np.max(np.abs(rewm[d] - ref['reward_mod'])) <= TOL_TIGHT, d
            assert np.max(np.abs(obs[d] - ref['obs'])) <= 1e-6, d
            per_env += ref['done']
        compare_state(env, ob)
        ndone += int(per_env.sum())
        multi += int((per_env >= 8).sum())
    assert ndone > 0
    a = rng.uniform(0, 1, (n, 2)).astype(np.float32)
    out1 = env.step_into(torch.from_numpy(a).to(gpu))
    ref = ob.step(a)
    torch.cuda.synchronize()
    compare_out(out1, ref)
    compare_state(env, ob)
    print('k=%d %s: dones %d, envs with >= 8 in a launch %d' % (k, map_name, ndone, multi))
    env.check()


@pytest.mark.parametrize('k,repeat,map_name', [(16, 4, 'loop_empty'), (9, 5, 'loop_obstacles')])
def test_step_many_generic_path(gpu, k, repeat, map_name):
    """More Simulator steps per decision than the fan kernel holds (repeat 4-5):
    dt_step_many runs step_kernel over the k decisions; same check against the
    oracle, with and without the per-decision poses (which then take one
    launch per decision)."""
    from aido1_amd.vec_env import StepOutput
    n = 2048
    for with_pose in (False, True):
        env, ob = make_pair(n, map_name=map_name, repeat_actions=repeat)
        env.reset()
        ob.reset()
        rng = np.random.default_rng(37)
        out = StepOutput(k * n, gpu, lanepos=False, tile=False)
        pose = torch.empty(k, 3, n, dtype=torch.float64, device=gpu) if with_pose else None
        for _ in range(2):
            a = rng.uniform(0, 1, (k, n, 2)).astype(np.float32)
            env.step_many_into(torch.from_numpy(a).to(gpu), out, pose=pose)
            torch.cuda.synchronize()
            rew = out.reward.view(k, n).cpu().numpy()
            done = out.done.view(k, n).cpu().numpy()
            for d in range(k):
                ref = ob.step(a[d])
                assert np.array_equal(done[d], ref['done']), d
                assert np.max(np.abs(rew[d] - ref['reward'])) <= TOL_TIGHT, d
                if with_pose:
                    o = ob.state()
                    p = pose[d].cpu().numpy()
                    assert np.max(np.abs(p[0] - o['x'])) <= TOL_TIGHT
                    assert np.max(np.abs(p[2] - o['angle'])) <= TOL_TIGHT
            compare_state(env, ob)
        env.check()


@pytest.mark.parametrize('k', [1, 20, 64])
def test_step_many_pose_output(gpu, k):
    """dt_step_many's per-decision poses (fan kernel) == the oracle's pose after
    each decision (the reset pose after a respawn), i.e. what a render of that
    decision draws."""
    from aido1_amd.vec_env import StepOutput
    n = 4096
    env, ob = make_pair(n)
    env.reset()
    ob.reset()
    rng = np.random.default_rng(41)
    out = StepOutput(k * n, gpu, lanepos=False, tile=False)
    pose = torch.empty(k, 3, n, dtype=torch.float64, device=gpu)
    for _ in range(2):
        a = rng.uniform(0, 1, (k, n, 2)).astype(np.float32)
        env.step_many_into(torch.from_numpy(a).to(gpu), out, pose=pose)
        torch.cuda.synchronize()
        p = pose.cpu().numpy()
        for d in range(k):
            ob.step(a[d])
            o = ob.state()
            for j, key in enumerate(('x', 'z', 'angle')):
                assert np.max(np.abs(p[d, j] - o[key])) <= TOL_TIGHT, (d, key)
        compare_state(env, ob)
    env.check()
