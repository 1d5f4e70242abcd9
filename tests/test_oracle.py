"""Pinning the CPU oracle (oracle/) before it is trusted as the checker.

- Philox4x32-10 against Random123's known-answer vectors.
- The Simulator restatement (dtsim_ref.py) against analytic known answers.
- The wrapper pieces against golden vectors generated from the reference
  (tests/golden/make_golden.py).
- The C restatement (dtsim_oracle.c) bit-for-bit against dtsim_ref.py.
"""
import math

import numpy as np
import pytest

from conftest import golden, map_objects, map_rows
from oracle import dtsim_ref as R
from oracle import oracle_c as OC
from oracle import philox_ref as P

# Random123 kat_vectors, philox4x32 R=10: (ctr, key) -> out
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff),
     (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.mark.parametrize('ctr,key,out', KAT)
def test_philox_kat_python(ctr, key, out):
    assert P.philox4x32_10(ctr, key) == out


@pytest.mark.parametrize('ctr,key,out', KAT)
def test_philox_kat_c(ctr, key, out):
    assert OC.philox(ctr, key) == out


def test_u01_range():
    assert P.u01(0, 0) == 0.0
    assert P.u01(0xffffffff, 0xffffffff) < 1.0
    assert P.u01(0x80000000, 0) == 0.5


LOOP = map_rows('loop_empty')


def sim(**kw):
    return R.SimulatorRef(LOOP, seed=1, env_id=0, cfg=R.SimConfig(**kw))


def test_straight_line_motion():
    # Vl == Vr: pos += dt * v * dir(angle) (update_pos straight branch)
    s = sim()
    s.cur_pos = np.array([0.3, 0.0, 1.0])
    s.cur_angle = -math.pi / 2  # heading +z
    s.step(np.array([0.5, 0.5]))
    dt = 1.0 / 30
    assert s.cur_pos[0] == pytest.approx(0.3, abs=1e-15)
    assert s.cur_pos[2] == pytest.approx(1.0 + dt * 0.6, abs=1e-15)
    assert s.cur_angle == -math.pi / 2
    assert s.step_count == 1


def test_pure_rotation():
    # Vl = -Vr: ICC at the robot centre, angle += (Vr - Vl)/l * dt, position fixed
    s = sim()
    s.cur_pos = np.array([0.3, 0.0, 1.0])
    s.cur_angle = 0.25
    s.step(np.array([-0.5, 0.5]))
    w = (0.6 - (-0.6)) / 0.102
    assert s.cur_angle == pytest.approx(0.25 + w / 30, abs=1e-14)
    assert s.cur_pos[0] == pytest.approx(0.3, abs=1e-15)
    assert s.cur_pos[2] == pytest.approx(1.0, abs=1e-15)


def test_on_centre_line():
    # straight/S tile (0, 1): right lane heading +z sits at x = (0.5 - 0.2) * 0.61
    s = sim()
    x = (0.5 - 0.2) * 0.61
    for z in (0.7, 0.9, 1.1):
        lp = s.get_lane_pos2(np.array([x, 0.0, z]), -math.pi / 2)
        assert lp.dist == pytest.approx(0.0, abs=1e-12)
        assert lp.dot_dir == pytest.approx(1.0, abs=1e-12)
        assert abs(lp.angle_deg) < 1e-4
        # heading the other way selects the other lane; dist measured from it
        lp2 = s.get_lane_pos2(np.array([x, 0.0, z]), math.pi / 2)
        assert lp2.dot_dir == pytest.approx(1.0, abs=1e-12)
        assert lp2.dist == pytest.approx(-0.4 * 0.61, abs=1e-12)


def test_lane_angle_sign():
    s = sim()
    x = (0.5 - 0.2) * 0.61
    lp = s.get_lane_pos2(np.array([x, 0.0, 0.9]), -math.pi / 2 + 0.1)
    lm = s.get_lane_pos2(np.array([x, 0.0, 0.9]), -math.pi / 2 - 0.1)
    assert lp.angle_rad == pytest.approx(-lm.angle_rad, abs=1e-12)
    assert abs(lp.angle_rad) == pytest.approx(0.1, abs=1e-12)
    assert lp.angle_deg == lp.angle_rad * (180.0 / math.pi)


def test_tile_edges_and_not_in_lane():
    s = sim()
    ts = 0.61
    assert s.get_grid_coords(np.array([ts, 0, 2 * ts])) == (1, 2)
    assert s.get_grid_coords(np.array([np.nextafter(ts, 0), 0, 0.0])) == (0, 0)
    assert s.get_grid_coords(np.array([-1e-12, 0, 0.0])) == (-1, 0)
    assert not s._drivable_pos(np.array([1.5 * ts, 0, 1.5 * ts]))   # grass centre
    assert not s._drivable_pos(np.array([-0.01, 0, 0.5]))           # off grid
    with pytest.raises(R.NotInLane):
        s.get_lane_pos2(np.array([1.5 * ts, 0, 1.5 * ts]), 0.0)


def test_invalid_pose_reward_and_done():
    s = sim()
    s.cur_pos = np.array([1.5 * 0.61, 0.0, 1.5 * 0.61])
    s.cur_angle = 0.0
    _, r, d, _ = s.step(np.array([0.0, 0.0]))
    assert r == -1000 and d


def test_max_steps_done():
    s = sim(max_steps=3)
    s.reset()
    for k in range(3):
        _, r, d, _ = s.step(np.array([0.0, 0.0]))
    assert d and r == 0


def test_reset_properties():
    s = sim()
    for _ in range(30):
        s.reset()
        assert s._valid_pose(s.cur_pos, s.cur_angle, 1.3)
        lp = s.get_lane_pos2(s.cur_pos, s.cur_angle)
        assert -4 < lp.angle_deg < 4
        assert s.step_count == 0


def test_rad2deg_constant():
    assert float(np.rad2deg(1.0)) == 180.0 / math.pi
    x = np.random.default_rng(0).normal(size=100)
    assert np.array_equal(np.rad2deg(x), x * (180.0 / math.pi))


# ---- golden vectors from the reference ------------------------------------------
def test_golden_aggregation():
    for c in golden('aggregation.json'):
        assert R.baseline_aggregation(c['r']) == c['baseline']
        assert c['baseline'] == c['dt_reward_wrapper']


def test_golden_steering():
    for c in golden('steering.json'):
        if 'action' in c:   # float64 inputs: bit-exact
            got = R.steering_to_wheels(np.array(c['action'], np.float64))
            assert got == c['sim_action'], c
        else:
            # float32 inputs: the fixture was generated under numpy 2 (NEP 50), where
            # `vel, angle = action` stay float32 scalars and the wrapper's arithmetic
            # runs in float32.  The aido1-era numpy 1.x promoted float32-scalar x
            # Python-float to float64, which is what the build (and this oracle)
            # computes, so these agree to float32 rounding only.
            got = R.steering_to_wheels(np.array(c['action32'], np.float64))
            assert got == pytest.approx(c['sim_action'], abs=2e-7, rel=1e-6), c


def test_golden_env_wrapper_on_oracle():
    """The reference's own EnvironmentWrapper.step, driven over SimulatorRef,
    reproduced by the restated wrapper (EnvironmentWrapperRef) exactly."""
    for fx in golden('env_wrapper.json'):
        cfg = R.SimConfig(max_env_steps=fx['max_env_steps'], action_mode=fx['mode'])
        w = R.EnvironmentWrapperRef(R.SimulatorRef(LOOP, seed=fx['seed'], env_id=0, cfg=cfg))
        w.reset()
        w.reset()  # EnvironmentWrapper.__init__ resets once, the script once more
        for st in fx['steps']:
            a = np.array(st['action_in'], np.float32)
            if fx['mode'] == 'tanh':
                m = a.copy()
                m /= 2
                m += np.float32(0.5)
                assert m.tolist() == st['action_after']
            r, rm, d = w.step(a)
            assert (r, rm, d) == (st['reward'], st['reward_mod'], st['done'])
            if d:
                w.reset()


def test_golden_env_wrapper_on_c_oracle():
    for fx in golden('env_wrapper.json'):
        sc = R.SimConfig(max_env_steps=fx['max_env_steps'], action_mode=fx['mode'])
        ob = OC.OracleBatch(LOOP, 1, seed=fx['seed'], sim_config=sc, auto_reset=True)
        ob.reset()
        ob.reset()
        for st in fx['steps']:
            out = ob.step(np.array([st['action_in']], np.float32))
            assert out['reward'][0] == st['reward']
            assert out['reward_mod'][0] == st['reward_mod']
            assert bool(out['done'][0]) == st['done']


# ---- C restatement == numpy restatement ---------------------------------------
@pytest.mark.parametrize('map_name,mode', [('loop_empty', 'wheels'), ('zigzag', 'tanh'),
                                           ('small_loop', 'steering'),
                                           ('intersections', 'wheels'),
                                           ('loop_obstacles', 'wheels')])
def test_c_oracle_matches_numpy(map_name, mode):
    rows = map_rows(map_name)
    objs = map_objects(map_name)
    n = 12
    sc = R.SimConfig(action_mode=mode, max_env_steps=60)
    ob = OC.OracleBatch(rows, n, seed=99, sim_config=sc, objects=objs)
    envs = [R.EnvironmentWrapperRef(R.SimulatorRef(rows, seed=99, env_id=i, cfg=sc,
                                                   objects=objs))
            for i in range(n)]
    ob.reset()
    for e in envs:
        e.reset()
    st = ob.state()
    for i, e in enumerate(envs):
        assert (st['x'][i], st['z'][i], st['angle'][i]) == \
            (e.sim.cur_pos[0], e.sim.cur_pos[2], e.sim.cur_angle)
        assert ob.spawn_k[i] == e.sim.last_spawn_k
    rng = np.random.default_rng(3)
    lo = -1.0 if mode != 'wheels' else 0.0
    for t in range(80):
        a = rng.uniform(lo, 1.0, (n, 2)).astype(np.float32)
        out = ob.step(a)
        for i, e in enumerate(envs):
            r, rm, d = e.step(a[i])
            assert out['reward'][i] == r and out['reward_mod'][i] == rm
            assert bool(out['done'][i]) == d
            assert out['tile'][i] == e.tile_index()
            lp = e.lane_pos()
            if lp is None:
                assert np.isnan(out['lanepos'][i]).all()
            else:
                assert tuple(out['lanepos'][i]) == tuple(lp)
            if d:
                e.reset()
        st = ob.state()
        for i, e in enumerate(envs):
            assert (st['x'][i], st['z'][i], st['angle'][i]) == \
                (e.sim.cur_pos[0], e.sim.cur_pos[2], e.sim.cur_angle)
            assert st['step_count'][i] == e.sim.step_count
