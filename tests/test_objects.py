"""Static objects: upstream Simulator._load_objects,
_collision, proximity_penalty2 and _inconvenient_spawn.

gym-duckietown (and its object meshes) is absent, so these are pinned to the
restatement (oracle/dtsim_ref.py), to analytic cases and to the C oracle --
parity against upstream itself is unpinned."""
import math

import numpy as np
import pytest

from conftest import map_objects, map_rows
from oracle import dtsim_ref as R
from oracle import oracle_c as OC


def test_corners_and_axes():
    # an unrotated box: corners at pos + scaled extents, axes = world x / z
    c = R.generate_corners(np.array([1.0, 0, 2.0]), np.array([-1.0, 0, -0.5]),
                           np.array([1.0, 1, 0.5]), 0.0, 0.1)
    assert np.allclose(c, [[0.9, 1.95], [1.1, 1.95], [1.1, 2.05], [0.9, 2.05]])
    n = R.generate_norm(c)
    assert np.allclose(np.abs(n @ n.T), np.eye(2))
    # rotated by 30 degrees: the long axis follows the rotation
    c = R.generate_corners(np.zeros(3), np.array([-1.0, 0, -0.5]), np.array([1.0, 1, 0.5]),
                           math.radians(30), 1.0)
    n = R.generate_norm(c)
    long_axis = n[np.argmax([np.ptp(c @ a) for a in n])]
    assert abs(abs(long_axis @ [math.cos(math.radians(30)), -math.sin(math.radians(30))]) - 1) < 1e-12


def test_square_footprint_axes_quirk():
    """A square footprint's covariance is isotropic, so generate_norm's axes are
    whatever eig makes of the rounding noise -- here neither the box's edges
    nor the world axes (upstream behaviour, kept: the product loader calls the
    same numpy routines, so its tables are bit-identical to the oracle's)."""
    c = R.generate_corners(np.zeros(3), np.array([-1.0, 0, -1.0]), np.array([1.0, 1, 1.0]),
                           math.radians(30), 1.0)
    n = R.generate_norm(c)
    assert np.allclose(n @ n.T, np.eye(2))
    edge = np.array([math.cos(math.radians(30)), -math.sin(math.radians(30))])
    assert not np.isclose(np.max(np.abs(n @ edge)), 1.0)
    from aido1_amd.maps import generate_norm
    assert np.array_equal(generate_norm(c), n)


def test_product_loader_matches_oracle_tables():
    from aido1_amd.maps import load_map
    m = load_map('loop_obstacles')
    om = OC.OracleMap(map_rows('loop_obstacles'), objects=map_objects('loop_obstacles'))
    assert m.object_table.shape == om.objects.shape == (4, 20)
    assert np.array_equal(m.object_table, om.objects)
    assert np.array_equal(m.spawn_table, om.spawn_objects)
    assert [o.collidable for o in m.objects] == [True, True, True, False, True]


def test_default_mesh_extents_and_errors():
    from aido1_amd.maps import parse_object, parse_rows
    o = parse_object({'kind': 'duckie', 'pos': [1, 1], 'rotate': 0, 'height': 0.08}, 0.61)
    assert o.scale == pytest.approx(0.08)
    with pytest.raises(ValueError):
        parse_object({'kind': 'unicorn', 'pos': [1, 1], 'height': 0.1}, 0.61)
    with pytest.raises(ValueError):
        parse_object({'kind': 'cone', 'pos': [1, 1], 'height': 0.1, 'scale': 1}, 0.61)
    with pytest.raises(NotImplementedError):
        parse_object({'kind': 'duckie', 'pos': [1, 1], 'height': 0.1, 'static': False}, 0.61)
    # an object on grass only is not collidable
    m = parse_rows([['grass', 'straight/S']], objects=[
        {'kind': 'tree', 'pos': [0.5, 0.5], 'height': 0.2}])
    assert not m.objects[0].collidable and len(m.object_table) == 0
    assert len(m.spawn_table) == 1


def _sim(**kw):
    return R.SimulatorRef(map_rows('loop_obstacles'), seed=5, env_id=0,
                          objects=map_objects('loop_obstacles'), **kw)


def test_collision_and_penalty_at_an_object():
    sim = _sim()
    duck = sim.map.collidable_centers[0]
    angle = math.pi   # driving -x along the top straight's right lane
    off = R.CAMERA_FORWARD_DIST - R.ROBOT_LENGTH / 2
    # actual centre on the duckie: invalid pose (collision), penalty negative
    pos = duck - off * R.get_dir_vec(angle)
    pos[1] = 0.0
    assert sim._drivable_pos(R._actual_center(pos, angle))
    assert not sim._valid_pose(pos, angle)
    assert sim.proximity_penalty2(pos, angle) < 0
    # 0.4 m away along the lane: valid, penalty 0 (outside both safety circles)
    far = pos + 0.4 * R.get_dir_vec(angle)
    assert sim._valid_pose(far, angle)
    assert sim.proximity_penalty2(far, angle) == 0
    # in between: valid but penalised, d - AGENT_SAFETY_RAD - r < 0
    near = pos + 0.2 * R.get_dir_vec(angle)
    d = np.linalg.norm(duck - R._actual_center(near, angle))
    want = d - R.AGENT_SAFETY_RAD - sim.map.collidable_safety_radii[0]
    assert want < 0 and sim._valid_pose(near, angle)
    assert sim.proximity_penalty2(near, angle) == pytest.approx(want, abs=1e-15)
    assert sim.compute_reward(near, angle, 1.2) < sim.compute_reward(far, angle, 1.2) - 1.0


def test_spawns_keep_away_from_objects():
    sim = _sim()
    for ep in range(200):
        sim.reset()
        for o in sim.map.objects:
            r = max(o['max_coords']) * 0.5 * o['scale'] + R.MIN_SPAWN_OBJ_DIST
            assert np.linalg.norm(o['pos'] - sim.cur_pos) >= r


def test_objects_end_episodes_in_the_c_oracle():
    """Driving straight ahead from every spawn: some envs hit an object and get
    REWARD_INVALID_POSE on a drivable tile; rewards carry the penalty."""
    rows, objs = map_rows('loop_obstacles'), map_objects('loop_obstacles')
    sc = R.SimConfig(max_env_steps=400, repeat_actions=1)
    ob = OC.OracleBatch(rows, 512, seed=7, sim_config=sc, auto_reset=False, objects=objs)
    plain = OC.OracleBatch(rows, 512, seed=7, sim_config=sc, auto_reset=False)
    ob.reset()
    plain.reset()
    a = np.full((512, 2), 0.4, np.float32)
    hit = penalised = 0
    alive = np.ones(512, bool)
    for t in range(120):
        o = ob.step(a)
        p = plain.step(a)
        hit += int(np.sum(alive & (o['reward'] == -1000) & (p['reward'] != -1000)))
        penalised += int(np.sum(alive & (o['reward'] < p['reward']) & (o['reward'] != -1000)))
        alive &= ~o['done'].astype(bool)
    assert hit > 0 and penalised > 0
