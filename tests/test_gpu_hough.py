"""dt_hough_lines (one wave per image) and render.find_normals on the GPU
against the CPU restatements (oracle/hough_oracle.c, oracle/linedet_ref.py):
identical segments, counts and centres, normals to 1e-12, on synthetic edge
images and on the renderer's own masks (features/line_detector1.py:55,63-132)."""
import numpy as np
import pytest
import torch

from oracle import linedet_ref as LR

pytestmark = pytest.mark.gpu


def _synthetic(n, seed):
    rng = np.random.default_rng(seed)
    imgs = np.zeros((n, 120, 160), np.uint8)
    for i in range(n):
        for _ in range(rng.integers(1, 6)):
            x0, x1 = rng.integers(0, 160, 2)
            y0, y1 = rng.integers(0, 120, 2)
            m = max(abs(x1 - x0), abs(y1 - y0), 1)
            t = np.linspace(0, 1, m + 1)
            imgs[i, np.round(y0 + t * (y1 - y0)).astype(int),
                 np.round(x0 + t * (x1 - x0)).astype(int)] = 255
        imgs[i][rng.random((120, 160)) < 0.01] = 255
    return imgs


@pytest.mark.parametrize('params', [(2, 3, 1), (10, 10, 3), (1, 1, 0)])
def test_hough_matches_oracle_synthetic(gpu, params):
    from aido1_amd.render import hough_lines
    imgs = _synthetic(48, sum(params))
    lines, counts = hough_lines(torch.from_numpy(imgs).to(gpu), *params)
    lines, counts = lines.cpu().numpy(), counts.cpu().numpy()
    for i in range(len(imgs)):
        want = LR.hough_lines(imgs[i], *params)
        assert counts[i] == len(want), (i, counts[i], len(want))
        assert np.array_equal(lines[i, :counts[i]], want), i


@pytest.mark.parametrize('map_name', ['loop_empty', 'intersections'])
def test_detect_lines_on_rendered_masks(gpu, map_name):
    from aido1_amd.config import EnvConfig
    from aido1_amd.render import RenderOutput, detect_lines, COLOR_PLANE, MASK_EDGES
    from aido1_amd.vec_env import StepOutput, VecEnv
    n = 96
    env = VecEnv(n, seed=3, device=0, config=EnvConfig(map_name=map_name))
    env.reset()
    out = StepOutput(n, gpu, lanepos=False, tile=False)
    ro = RenderOutput(n, gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(1)
    for _ in range(5):
        env.step_into(torch.rand(n, 2, generator=g, device=gpu), out)
        env.render_into(ro, fresh=out.done)
    torch.cuda.synchronize()
    masks = ro.masks
    total = 0
    for color in ('white', 'yellow'):
        det = detect_lines(masks, color)
        bw = masks[:, COLOR_PLANE[color]].cpu().numpy()
        ec = (masks[:, COLOR_PLANE[color]] & masks[:, MASK_EDGES]).cpu().numpy()
        counts = det['counts'].cpu().numpy()
        for i in range(n):
            raw = LR.hough_lines(ec[i])
            assert counts[i] == len(raw), (color, i)
            want_l, want_c, want_n = LR.find_normals(bw[i], raw)
            k = counts[i]
            assert np.array_equal(det['lines'][i, :k].cpu().numpy(), want_l), (color, i)
            assert np.array_equal(det['centers'][i, :k].cpu().numpy(), want_c), (color, i)
            # float64 to the last bits: the reference's `** 0.5` is numpy's
            # power (glibc pow) where the device takes sqrt, and its divisions
            # run on the GPU
            np.testing.assert_allclose(det['normals'][i, :k].cpu().numpy(), want_n, rtol=0,
                                       atol=1e-12, err_msg='%s %d' % (color, i))
            total += k
    assert total > 0
    env.close()
