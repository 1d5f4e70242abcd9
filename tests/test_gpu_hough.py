"""dt_hough_lines (one wave per image) and render.find_normals on the GPU
against the CPU restatements (oracle/hough_oracle.c, oracle/linedet_ref.py):
identical segments, counts and centres, normals to 1e-12, on synthetic edge
images and on the renderer's own masks (features/line_detector1.py:55,63-132)."""
import numpy as np
import pytest
import torch

from oracle import linedet_ref as LR

pytestmark = pytest.mark.gpu


def _synthetic(n, seed, h=120, w=160, noise=0.01, max_segs=6):
    rng = np.random.default_rng(seed)
    imgs = np.zeros((n, h, w), np.uint8)
    for i in range(n):
        for _ in range(rng.integers(1, max_segs)):
            x0, x1 = rng.integers(0, w, 2)
            y0, y1 = rng.integers(0, h, 2)
            m = max(abs(x1 - x0), abs(y1 - y0), 1)
            t = np.linspace(0, 1, m + 1)
            imgs[i, np.round(y0 + t * (y1 - y0)).astype(int),
                 np.round(x0 + t * (x1 - x0)).astype(int)] = 255
        imgs[i][rng.random((h, w)) < noise] = 255
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


@pytest.mark.parametrize('shape', [(120, 160), (240, 320), (480, 640)])
def test_hough_workspace_kernel_matches_oracle(gpu, shape):
    """dt_hough_lines_ws: accumulator, mask and point list in HBM, any size
    (the 640x480 camera frame of duckietown_rl/env.py:12-16)."""
    from aido1_amd.render import hough_lines
    h, w = shape
    imgs = _synthetic(6, h + w, h, w, noise=0.004, max_segs=12)
    lines, counts = hough_lines(torch.from_numpy(imgs).to(gpu), workspace=True, max_lines=2048)
    lines, counts = lines.cpu().numpy(), counts.cpu().numpy()
    for i in range(len(imgs)):
        want = LR.hough_lines(imgs[i], max_lines=2048)
        assert counts[i] == len(want), (i, counts[i], len(want))
        assert np.array_equal(lines[i, :counts[i]], want), i


def test_hough_point_overflow_goes_to_workspace(gpu):
    """An image with more edge pixels than the LDS point list (~16k at
    120x160) is flagged -1 by the LDS kernel; the workspace kernel takes it."""
    from aido1_amd.render import HOUGH_OVERFLOW, hough_lines
    rng = np.random.default_rng(7)
    imgs = ((rng.random((2, 120, 160)) < 0.9) * 255).astype(np.uint8)
    dev = torch.from_numpy(imgs).to(gpu)
    _, counts = hough_lines(dev)
    assert (counts.cpu().numpy() == HOUGH_OVERFLOW).all()
    lines, counts = hough_lines(dev, workspace=True, max_lines=8192)
    lines, counts = lines.cpu().numpy(), counts.cpu().numpy()
    for i in range(2):
        want = LR.hough_lines(imgs[i], max_lines=8192)
        assert counts[i] == len(want), (i, counts[i], len(want))
        assert np.array_equal(lines[i, :counts[i]], want), i


@pytest.mark.parametrize('workspace', [None, True])
def test_hough_truncation_flag(gpu, workspace):
    """max_lines reached with edge points unvisited: count -2 and the first
    max_lines lines (OpenCV has no cap, so the list is cut short)."""
    from aido1_amd.render import HOUGH_TRUNCATED, hough_lines
    imgs = _synthetic(24, 11, max_segs=10)
    cap = 2
    lines, counts = hough_lines(torch.from_numpy(imgs).to(gpu), max_lines=cap,
                                workspace=workspace)
    lines, counts = lines.cpu().numpy(), counts.cpu().numpy()
    flagged = 0
    for i in range(len(imgs)):
        want = LR.hough_lines(imgs[i], max_lines=4096)
        if len(want) > cap:
            assert counts[i] == HOUGH_TRUNCATED, (i, counts[i])
            flagged += 1
        elif len(want) < cap:
            assert counts[i] == len(want), (i, counts[i])
        else:
            assert counts[i] in (cap, HOUGH_TRUNCATED)
        assert np.array_equal(lines[i, :min(cap, len(want))], want[:cap]), i
    assert flagged > 0


def test_detect_lines_grows_a_truncated_list(gpu):
    from aido1_amd.render import COLOR_PLANE, MASK_EDGES, detect_lines
    imgs = _synthetic(8, 3, max_segs=10)
    masks = np.zeros((8, 4, 120, 160), np.uint8)
    masks[:, COLOR_PLANE['white']] = 255
    masks[:, MASK_EDGES] = imgs
    det = detect_lines(torch.from_numpy(masks).to(gpu), 'white', max_lines=1)
    counts = det['counts'].cpu().numpy()
    for i in range(8):
        want = LR.hough_lines(imgs[i], max_lines=4096)
        assert counts[i] == len(want), (i, counts[i], len(want))
        assert np.array_equal(det['lines'][i, :counts[i]].cpu().numpy(),
                              LR.find_normals(masks[i, COLOR_PLANE['white']], want)[0]), i
