"""GPU parity of the observation path: the fused raster + grey + line-detector
kernel and the standalone LineDetectorHSV kernel vs the C oracle
(oracle/render_oracle.c).  Integer/byte outputs (raster, masks) must match bit
for bit; grey is float32 of the same expression (bit-exact expected)."""
import math

import numpy as np
import pytest
import torch

from conftest import map_rows
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu


def poses(n, rng, env=None):
    ts = 0.61
    x = rng.uniform(-0.2, 3 * ts + 0.2, n)
    z = rng.uniform(-0.2, 3 * ts + 0.2, n)
    a = rng.uniform(-math.pi, 3 * math.pi, n)
    x[:4] = [(0.5 - 0.2) * ts, 1.5 * ts, -40.0, 1e3]
    z[:4] = [0.7, 1.5 * ts, 7.0, -1e3]
    a[:4] = [-math.pi / 2, 0.0, 1.0, 2.0]
    return x, z, a


@pytest.mark.parametrize('map_name', ['loop_empty', 'zigzag', 'intersections'])
def test_render_parity(gpu, map_name):
    from aido1_amd.config import EnvConfig
    from aido1_amd.render import RenderOutput
    from aido1_amd.vec_env import VecEnv
    n = 384
    env = VecEnv(n, seed=3, config=EnvConfig(map_name=map_name))
    env.reset()
    rng = np.random.default_rng(4)
    x, z, a = poses(n, rng)
    s = env.get_state()   # keep half the envs at their spawn poses
    x[n // 2:], z[n // 2:], a[n // 2:] = s['x'][n // 2:], s['z'][n // 2:], s['angle'][n // 2:]
    env.set_state(x=x, z=z, angle=a)
    out = RenderOutput(n, gpu, slots=1, rgb=True)
    env.render_into(out)
    torch.cuda.synchronize()
    g, m, rgb = OC.OracleRender(map_rows(map_name)).render(x, z, a)
    assert np.array_equal(out.rgb.cpu().numpy(), rgb)
    assert np.array_equal(out.masks.cpu().numpy(), m)
    assert np.array_equal(out.ring[:, 0].cpu().numpy(), g)
    # the pipeline is exercised: lines visible, edges found
    assert (m[:, 0] > 0).any() and (m[:, 1] > 0).any() and (m[:, 3] > 0).any()


def test_ring_and_fresh(gpu):
    from aido1_amd.render import RenderOutput
    from aido1_amd.vec_env import VecEnv
    n = 64
    env = VecEnv(n, seed=5)
    env.reset()
    out = RenderOutput(n, gpu, slots=3, masks=False)
    env.render_into(out)                     # first frame: fills every slot
    f0 = out.ring[:, 0].clone()
    assert torch.equal(out.ring[:, 1], f0) and torch.equal(out.ring[:, 2], f0)
    acts = torch.full((n, 2), 0.6, device=gpu)
    o = env.step_into(acts)
    fresh = o.done.clone()
    env.render_into(out, fresh=fresh)        # slot 1 (or all slots for reset envs)
    f1 = out.ring[:, 1].clone()
    st = out.stack_view()
    assert torch.equal(st[:, 2], f1)         # newest last, as Transformer.transform
    keep = (fresh == 0)
    assert torch.equal(out.ring[keep, 0], f0[keep]) and torch.equal(out.ring[keep, 2], f0[keep])
    if (~keep).any():
        r = out.ring[~keep]
        assert torch.equal(r[:, 0], r[:, 1]) and torch.equal(r[:, 2], r[:, 1])


@pytest.mark.parametrize('map_name', ['loop_empty', 'zigzag'])
def test_index_frames_decode_to_grey(gpu, map_name):
    """Palette-index frames (dt_render_io.index): over launches with respawns
    (fresh refills) the index ring decoded through dt_palette_gray equals the
    grey ring of the same envs bit for bit, slot by slot, and the newest grey
    frame is the oracle's."""
    from aido1_amd.config import EnvConfig
    from aido1_amd.render import RenderOutput, decode_index
    from aido1_amd.vec_env import VecEnv
    n = 300
    envs = [VecEnv(n, seed=11, config=EnvConfig(map_name=map_name)) for _ in range(2)]
    outs = [RenderOutput(n, gpu, slots=3, masks=False, frames=f) for f in ('gray', 'index')]
    for env, out in zip(envs, outs):
        env.reset()
        env.render_into(out)
    g = torch.Generator(device=gpu).manual_seed(1)
    orend = OC.OracleRender(map_rows(map_name))
    for t in range(6):
        acts = torch.rand(n, 2, device=gpu, generator=g) * 2 - 1
        for env, out in zip(envs, outs):
            o = env.step_into(acts)
            env.render_into(out, fresh=o.done)
        assert outs[1].ring.dtype == torch.uint8 and int(outs[1].ring.max()) <= 7
        assert torch.equal(decode_index(outs[1].ring), outs[0].ring)
        assert torch.equal(outs[1].stack_view(), outs[0].stack_view())
    s = envs[0].get_state()
    gr, _, _ = orend.render(s['x'], s['z'], s['angle'])
    assert np.array_equal(outs[0].ring[:, outs[0].slot].cpu().numpy(), gr)


# (150, 200) and (480, 640) are past the LDS image (19,200 px): the workspace
# kernel (dt_line_detect_ws); 480 x 640 is duckietown_rl/env.py:12-16's frame
@pytest.mark.parametrize('shape', [(120, 160), (37, 53), (1, 1), (96, 200), (150, 200),
                                   (480, 640)])
def test_line_detect_parity(gpu, shape):
    from aido1_amd.render import LineParams, line_detect
    h, w = shape
    rng = np.random.default_rng(h * w)
    n = 12 if h * w <= 30000 else 4
    img = rng.integers(0, 256, (n, h, w, 3), dtype=np.uint8)
    # blocky content with real edges and colours in the HSV ranges
    for i in range(n // 2):
        img[i] = 40
        r0, c0 = rng.integers(0, max(1, h - 5)), rng.integers(0, max(1, w - 5))
        img[i, r0:r0 + 20, c0:c0 + 7] = [0, 230, 255]   # yellow (BGR)
        img[i, r0:r0 + 5, c0:] = [250, 250, 250]         # white
        img[i, :, :3] = [30, 30, 220]                   # red
    dev = torch.from_numpy(img).to(gpu)
    for params in (None, 'custom'):
        p = OC.line_params_default()
        lp = LineParams.default()
        if params:
            p.dilation_kernel_size = lp.dilation_kernel_size = 5
            p.canny_lo, p.canny_hi = lp.canny_lo, lp.canny_hi = 40.0, 120.0
        masks, hsv = line_detect(dev, lp, hsv=True)
        torch.cuda.synchronize()
        rm, rh = OC.OracleRender(map_rows('loop_empty'), params=p).line_detect(img, hsv=True)
        assert np.array_equal(hsv.cpu().numpy(), rh)
        assert np.array_equal(masks.cpu().numpy(), rm)


def _render_setup(gpu, map_name, n=256, seed=11):
    from aido1_amd.config import EnvConfig
    from aido1_amd.vec_env import VecEnv
    env = VecEnv(n, seed=seed, config=EnvConfig(map_name=map_name))
    env.reset()
    rng = np.random.default_rng(seed)
    x, z, a = poses(n, rng)
    s = env.get_state()
    x[n // 2:], z[n // 2:], a[n // 2:] = s['x'][n // 2:], s['z'][n // 2:], s['angle'][n // 2:]
    env.set_state(x=x, z=z, angle=a)
    return env, x, z, a


@pytest.mark.parametrize('list_cap', [1, 64, 700])
def test_render_spill_path_matches_oracle(gpu, list_cap):
    """Frames with more non-uniform words than the LDS list holds keep the rest
    in the global spill area: forcing a small cap must not change a bit."""
    from aido1_amd.render import RenderOutput
    env, x, z, a = _render_setup(gpu, 'loop_empty')
    out = RenderOutput(env.n, gpu, slots=1)
    env.render_into(out, list_cap=list_cap)
    torch.cuda.synchronize()
    g, m, _ = OC.OracleRender(map_rows('loop_empty')).render(x, z, a)
    assert np.array_equal(out.masks.cpu().numpy(), m)
    assert np.array_equal(out.ring[:, 0].cpu().numpy(), g)


@pytest.mark.parametrize('dil,lo,hi', [(1, 80.0, 200.0), (5, 40.0, 120.0), (7, 80.0, 200.0),
                                       (3, 200.0, 80.0)])
def test_render_line_params_match_oracle(gpu, dil, lo, hi):
    """Other dilation sizes (radius >= 2: every quad takes the dilation path)
    and Canny thresholds (swapped ones are reordered, as cv2.Canny does)."""
    from aido1_amd.render import LineParams, RenderOutput
    env, x, z, a = _render_setup(gpu, 'zigzag', seed=13)
    lp = LineParams.default()
    lp.dilation_kernel_size, lp.canny_lo, lp.canny_hi = dil, lo, hi
    env.set_line_params(lp)
    p = OC.line_params_default()
    p.dilation_kernel_size, p.canny_lo, p.canny_hi = dil, lo, hi
    out = RenderOutput(env.n, gpu, slots=1)
    env.render_into(out)
    torch.cuda.synchronize()
    g, m, _ = OC.OracleRender(map_rows('zigzag'), params=p).render(x, z, a)
    assert np.array_equal(out.masks.cpu().numpy(), m)
    assert np.array_equal(out.ring[:, 0].cpu().numpy(), g)


def test_render_pose_snapshot(gpu):
    """dt_copy_pose + dt_render_io.pose: the render reads the snapshot, not the
    state a later step has moved on."""
    from aido1_amd.render import RenderOutput
    env, x, z, a = _render_setup(gpu, 'loop_empty', n=128, seed=17)
    snap = torch.empty(3, env.n, dtype=torch.float64, device=gpu)
    env.copy_pose(snap)
    env.step_into(torch.full((env.n, 2), 0.7, device=gpu))   # moves every env
    out = RenderOutput(env.n, gpu, slots=1)
    env.render_into(out, pose=snap)
    torch.cuda.synchronize()
    assert np.array_equal(snap.cpu().numpy(), np.stack([x, z, a]))
    g, m, _ = OC.OracleRender(map_rows('loop_empty')).render(x, z, a)
    assert np.array_equal(out.masks.cpu().numpy(), m)
    assert np.array_equal(out.ring[:, 0].cpu().numpy(), g)


def test_render_dispatch_order(gpu):
    """dt_render dispatches the envs longest recorded render first: after each
    launch the next order is a permutation of the envs, and over launches in
    that order the outputs stay the oracle's bit for bit.  A launch of <= 512
    envs runs at once and keeps the identity.  (The order follows measured
    shader-clock costs, which depend on the load of the box: only these
    deterministic properties are asserted.)"""
    from aido1_amd.render import RenderOutput
    from aido1_amd.vec_env import VecEnv
    orend = OC.OracleRender(map_rows('loop_empty'))
    for n in (4096, 100):
        env = VecEnv(n, seed=9)
        env.reset()
        out = RenderOutput(n, gpu, slots=1)
        rng = np.random.default_rng(n)
        l0, _, order0 = env.render_order()
        assert l0 == 0 and np.array_equal(order0, np.arange(n))
        for k in range(4):
            x, z, a = poses(n, rng)
            env.set_state(x=x, z=z, angle=a)
            env.render_into(out)
            launches, cost, order = env.render_order()
            assert launches == k + 1
            assert np.array_equal(np.sort(order), np.arange(n))          # a permutation
            if n <= 512:
                assert np.array_equal(order, np.arange(n))
            else:
                assert (cost > 0).all()
            g, m, _ = orend.render(x, z, a)
            assert np.array_equal(out.masks.cpu().numpy(), m)
            assert np.array_equal(out.ring[:, 0].cpu().numpy(), g)
        if n > 512:   # the later launches really ran in another order
            assert not np.array_equal(order, np.arange(n))


@pytest.mark.parametrize('frames', ['gray', 'index'])
@pytest.mark.parametrize('n', [1024, 300])
def test_render2_matches_two_renders(gpu, frames, n):
    """dt_render2 (two consecutive decisions in one launch) leaves the frame
    ring and both decisions' masks exactly as dt_render of the first then of
    the second: with fresh flags in either, both or neither decision, over
    several pairs (the first pair right after the ring's creation)."""
    from aido1_amd.render import RenderOutput, render2_into
    from aido1_amd.vec_env import VecEnv
    env = VecEnv(n, seed=21)
    env.reset()
    ref = RenderOutput(n, gpu, frames=frames)
    pair = RenderOutput(n, gpu, frames=frames)
    masks_b = torch.zeros_like(pair.masks)
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    for it in range(4):
        poses, fresh = [], []
        for _ in range(2):
            env.step_into(torch.rand(n, 2, generator=g, device=gpu))
            p = torch.empty(3, n, dtype=torch.float64, device=gpu)
            env.copy_pose(p)
            poses.append(p)
            fresh.append((torch.rand(n, generator=g, device=gpu) < 0.3).to(torch.uint8))
        env.render_into(ref, fresh=fresh[0], pose=poses[0])
        masks_a_ref = ref.masks.clone()
        env.render_into(ref, fresh=fresh[1], pose=poses[1])
        render2_into(env, pair, masks_b, fresh[0], poses[0], fresh[1], poses[1])
        torch.cuda.synchronize()
        assert pair.slot == ref.slot
        assert torch.equal(pair.masks, masks_a_ref), it
        assert torch.equal(masks_b, ref.masks), it
        assert torch.equal(pair.ring, ref.ring), it


@pytest.mark.parametrize('frames', ['gray', 'index'])
def test_render3_matches_three_renders(gpu, frames):
    """dt_render3 (three consecutive decisions, the ring's three slots, in one
    launch) equals dt_render of each in order: the ring and all three
    decisions' masks, fresh flags anywhere, over several groups."""
    from aido1_amd.render import RenderOutput, render_group_into
    from aido1_amd.vec_env import VecEnv
    n = 1024
    env = VecEnv(n, seed=23)
    env.reset()
    ref = RenderOutput(n, gpu, frames=frames)
    grp = RenderOutput(n, gpu, frames=frames)
    extra = [torch.zeros_like(grp.masks) for _ in range(2)]
    g = torch.Generator(device=gpu)
    g.manual_seed(7)
    for it in range(4):
        poses, fresh, want = [], [], []
        for _ in range(3):
            env.step_into(torch.rand(n, 2, generator=g, device=gpu))
            p = torch.empty(3, n, dtype=torch.float64, device=gpu)
            env.copy_pose(p)
            poses.append(p)
            fresh.append((torch.rand(n, generator=g, device=gpu) < 0.3).to(torch.uint8))
        for f, p in zip(fresh, poses):
            env.render_into(ref, fresh=f, pose=p)
            want.append(ref.masks.clone())
        render_group_into(env, grp, extra, fresh, poses)
        torch.cuda.synchronize()
        assert grp.slot == ref.slot
        for got, w in zip([grp.masks] + extra, want):
            assert torch.equal(got, w), it
        assert torch.equal(grp.ring, ref.ring), it
