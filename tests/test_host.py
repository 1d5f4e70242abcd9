"""Host-side logic that needs no GPU: config translation, ring order, spaces."""
import json
import math
import os

import numpy as np
import pytest
import torch

from conftest import REPO, golden


def test_envconfig_constants_bit_identical():
    from aido1_amd.config import EnvConfig
    from oracle import oracle_c as OC
    from oracle import dtsim_ref as R
    c = EnvConfig().to_c()
    o = OC.make_cfg(R.SimConfig())
    for name, _ in c._fields_:
        assert getattr(c, name) == getattr(o, name), name
    assert c.robot_width == 0.13 + 0.02
    assert c.rad2deg == float(np.rad2deg(1.0))
    assert c.two_pi == 2 * math.pi


def test_envconfig_from_reference_config():
    from aido1_amd.config import EnvConfig
    with open(os.path.join(REPO, 'tests', 'golden', 'reference_config.json')) as f:
        cfg = json.load(f)
    ec = EnvConfig.from_reference_config(cfg)
    assert (ec.max_env_steps, ec.repeat_actions, ec.reward_scale) == (2000, 3, 1.0)
    assert ec.action_mode == 'tanh'   # config.json:88 actor head is tanh
    with pytest.raises(ValueError):
        EnvConfig(action_mode='bogus').to_c()


def test_render_ring_order_matches_transformer():
    """RenderOutput.order() reproduces the Transformer's oldest-first stack
    (tests/golden/stacking.json, generated from the reference)."""
    from aido1_amd.render import RenderOutput
    fx = golden('stacking.json')['transformer']
    out = RenderOutput(1, 'cpu', slots=3, masks=False)
    frames = [100] + list(range(1, 6))
    for k, v in enumerate(frames):
        if out.slot < 0:   # first frame fills every slot (Transformer.reset)
            out.advance()
            out.ring[0, :] = v
        else:
            out.ring[0, out.advance()] = v
        stack = out.stack_view()[0, :, 0, 0].tolist()
        assert stack == fx[k], (k, stack, fx[k])


def test_box_space():
    from aido1_amd.simulator import Box
    b = Box(-1, 1, (2,), np.float32, seed=0)
    for _ in range(20):
        assert b.contains(b.sample())
    u = Box(0, 255, (120, 160, 3), np.uint8)
    assert u.low[0, 0, 0] == 0 and u.high[0, 0, 0] == 255


def test_maps_parse_errors():
    from aido1_amd.maps import parse_rows
    with pytest.raises(ValueError):
        parse_rows([['straight/S', 'grass'], ['grass']])
    with pytest.raises(NotImplementedError):
        parse_rows([['roundabout/N']])
    assert parse_rows([['4way']]).kind.tolist() == [6]
    m = parse_rows([['empty', 'grass', 'straight/E']])
    assert m.kind.tolist() == [-1, 0, 1]
