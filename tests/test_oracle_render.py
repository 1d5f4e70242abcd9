"""Pinning the observation-path oracle (oracle/render_oracle.c).

cv2 is absent, so each OpenCV piece is pinned against an independent source:
bresenham against the reference's own generator (golden vectors), HSV against
colorsys (+-1 from OpenCV's fixed point), dilation against scipy.ndimage; the
Canny edge map has no independent implementation here (parity unpinned), so
only its invariants are checked."""
import colorsys
import math

import numpy as np
import pytest
from scipy import ndimage

from conftest import golden, map_rows
from oracle import oracle_c as OC


def test_bresenham_golden():
    for c in golden('bresenham.json'):
        assert [list(p) for p in OC.bresenham(*c['line'])] == c['points'], c['line']


@pytest.fixture(scope='module')
def orc():
    return OC.OracleRender(map_rows('loop_empty'))


def test_hsv_vs_colorsys(orc):
    rng = np.random.default_rng(0)
    bgr = rng.integers(0, 256, (1, 40, 50, 3), dtype=np.uint8)
    bgr[0, 0, :5] = [[0, 0, 0], [255, 255, 255], [0, 0, 255], [0, 255, 0], [255, 0, 0]]
    _, hsv = orc.line_detect(bgr, hsv=True)
    for (b, g, r), (H, S, V) in zip(bgr.reshape(-1, 3), hsv.reshape(-1, 3)):
        h, s, v = colorsys.rgb_to_hsv(r / 255, g / 255, b / 255)
        assert V == max(r, g, b)
        assert abs(int(S) - s * 255) <= 1.0
        dh = abs(int(H) - h * 180) % 180
        assert min(dh, 180 - dh) <= 1.0 or S == 0


@pytest.mark.parametrize('k', [1, 3, 5, 7])
def test_dilation_vs_scipy(orc, k):
    # white mask = V >= 150 & S <= 60: build an image whose white pixels are known
    rng = np.random.default_rng(k)
    m = rng.random((60, 80)) < 0.03
    bgr = np.zeros((1, 60, 80, 3), np.uint8)
    bgr[0][m] = 255
    p = OC.line_params_default()
    p.dilation_kernel_size = k
    r = OC.OracleRender(map_rows('loop_empty'), params=p)
    masks = r.line_detect(bgr)
    rad = k // 2
    fp = np.zeros((k, k), bool)
    for i in range(k):
        dy = i - rad
        dx = int(round(rad * math.sqrt((rad * rad - dy * dy) / (rad * rad)))) if rad else 0
        fp[i, max(rad - dx, 0):min(rad + dx + 1, k)] = True
    ref = ndimage.binary_dilation(m, structure=fp, border_value=0)
    assert np.array_equal(masks[0, 0] > 0, ref)
    if k == 3:   # MORPH_ELLIPSE 3x3 is the cross
        assert np.array_equal(fp, ndimage.generate_binary_structure(2, 1))


def test_canny_invariants(orc):
    rng = np.random.default_rng(1)
    img = np.zeros((1, 60, 80, 3), np.uint8)
    img[0, 20:40, 30:60] = 200           # a bright rectangle: edges on its border only
    masks = orc.line_detect(img)
    e = masks[0, 3] > 0
    assert e.any()
    assert not e[25:35, 35:55].any() and not e[:15].any() and not e[45:].any()
    noise = rng.integers(0, 256, (1, 60, 80, 3), dtype=np.uint8)
    m2 = orc.line_detect(noise)
    p = OC.line_params_default()
    p.canny_lo, p.canny_hi = 2000, 3000   # above any L1 Sobel magnitude of 8-bit data
    assert not OC.OracleRender(map_rows('loop_empty'), params=p).line_detect(noise)[0, 3].any()
    assert m2[0, 3].any()


def test_render_on_lane(orc):
    # straight/S tile (0,1), right lane centre, heading +z: yellow centre line
    # 0.2 tile to the left, white edge 0.26 tile to the right
    x = (0.5 - 0.2) * 0.61
    gray, masks, rgb = orc.render(np.array([x]), np.array([0.70]), np.array([-math.pi / 2]))
    row = rgb[0, 110]
    cols_w = [c for c in range(80, 160) if tuple(row[c]) == (250, 250, 250)]
    assert cols_w
    assert abs(np.mean(cols_w) - (79.5 + 0.26 * 61)) < 2.5
    # the centre line is dashed: take the rows that have it
    ys = [c for r in range(90, 120) for c in range(40, 80) if tuple(rgb[0, r, c]) == (255, 230, 0)]
    assert abs(np.mean(ys) - (79.5 - 0.2 * 61)) < 2.5
    assert masks[0, 0].any() and masks[0, 1].any() and not masks[0, 2].any()
    # grey = skimage rgb2gray of the raster
    ref = (rgb[0].astype(np.float64) / 255.0) @ np.array([0.2125, 0.7154, 0.0721])
    assert np.max(np.abs(gray[0] - ref)) < 1e-6


def test_render_off_map(orc):
    gray, masks, rgb = orc.render(np.array([-50.0]), np.array([-50.0]), np.array([0.0]))
    assert not rgb.any() and not masks.any() and not gray.any()


def test_palette_gray_table_is_the_oracle_grey(orc):
    """dt_palette_gray (the library's 8 grey levels, which decode palette-index
    frames): every grey value of oracle frames is the table's entry for that
    pixel's colour, bit for bit -- so decoding an index frame gives the grey
    frame.  Host call only (no GPU)."""
    import ctypes
    from aido1_amd import _lib
    buf = (ctypes.c_float * 8)()
    assert _lib.lib().dt_palette_gray(buf) == 0
    table = np.array(list(buf), dtype=np.float32)
    rng = np.random.default_rng(2)
    n = 16
    x, z = rng.uniform(0, 3 * 0.61, n), rng.uniform(0, 3 * 0.61, n)
    a = rng.uniform(-math.pi, math.pi, n)
    gray, _, rgb = orc.render(x, z, a)
    cols = {}
    for c, g in zip(rgb.reshape(-1, 3), gray.reshape(-1)):
        cols.setdefault(tuple(int(v) for v in c), set()).add(float(g))
    assert len(cols) >= 4                      # floor / grass / road / markings seen
    for c, gs in cols.items():
        assert len(gs) == 1, c                 # one grey per colour
        g = np.float32(next(iter(gs)))
        r8, g8, b8 = (v / 255.0 for v in c)
        assert g == np.float32((r8 * 0.2125 + g8 * 0.7154) + b8 * 0.0721)
        assert (table == g).any(), (c, g, table)
