"""LineDetectorHSV's line stage on the CPU: the HoughLinesP restatement
(oracle/hough_oracle.c) on known answers, and the numpy _findNormal
restatement (oracle/linedet_ref.py) on hand-computed cases
(features/line_detector1.py:63-123).  OpenCV is absent, so HoughLinesP parity
against OpenCV itself is unpinned; the GPU kernel is pinned to this
restatement in tests/test_gpu_hough.py."""
import numpy as np

from oracle import linedet_ref as LR


def test_empty_and_isolated_points():
    img = np.zeros((120, 160), np.uint8)
    assert len(LR.hough_lines(img)) == 0
    img[10, 10] = img[50, 100] = 255          # two points never reach a 3-px extent
    assert len(LR.hough_lines(img, min_line_length=3)) == 0


def test_diagonal_line_segments_lie_on_it():
    """A 60-px diagonal: every segment end is a pixel of the line, and the
    segments (PPHT may split a line where its walk drifts by a pixel) cover
    most of it."""
    img = np.zeros((120, 160), np.uint8)
    for t in range(60):
        img[20 + t, 30 + t] = 1
    ls = LR.hough_lines(img)
    assert len(ls) >= 1
    assert np.all(ls[:, 0] - ls[:, 1] == 10) and np.all(ls[:, 2] - ls[:, 3] == 10)
    assert np.sum(np.abs(ls[:, 2] - ls[:, 0]) + 1) >= 50


def test_every_pixel_consumed_once():
    """Each kept segment clears its pixels: a second pass on what the segments
    cover finds nothing new (no segment double-counts)."""
    rng = np.random.default_rng(0)
    img = (rng.random((120, 160)) < 0.02).astype(np.uint8)
    for r in (30, 70):
        img[r, 20:140] = 1
    ls = LR.hough_lines(img)
    assert len(ls) >= 2
    assert np.all((ls[:, [0, 2]] >= 0) & (ls[:, [0, 2]] < 160))
    assert np.all((ls[:, [1, 3]] >= 0) & (ls[:, [1, 3]] < 120))
    ext = np.maximum(np.abs(ls[:, 2] - ls[:, 0]), np.abs(ls[:, 3] - ls[:, 1]))
    assert np.all(ext >= 3)


def test_find_normals_hand_computed():
    # horizontal segment at y = 40 from x = 10 to 20, colour area above it
    # (rows 30..40): the normal points away from the area
    bw = np.zeros((120, 160), np.uint8)
    bw[30:41] = 255
    lines, centers, normals = LR.find_normals(bw, [[10, 40, 20, 40]])
    assert centers.tolist() == [[15.0, 40.0]]
    # dx = (y2 - y1) / len = 0, dy = (x1 - x2) / len = -1; (15, 43) is outside
    # the area and (15, 37) inside, so the sign flips: normal (0, 1)
    assert normals.tolist() == [[-0.0, 1.0]]
    # flag = (x2 - x1) * ny - (y2 - y1) * nx = 10 > 0: endpoints swapped
    assert lines.tolist() == [[20, 40, 10, 40]]


def test_find_normals_clamps_probe_points():
    bw = np.zeros((10, 10), np.uint8)
    lines, centers, normals = LR.find_normals(bw, [[0, 0, 0, 9]])
    assert normals.shape == (1, 2) and np.isfinite(normals).all()
