"""Tile maps -> the C ABI's ``dt_map`` arrays.

Follows upstream Simulator._load_map / _get_curve (un-vendored gym-duckietown,
aido1 era): tiles "kind/orient" are drivable with
orient index ['S','E','N','W'], anything else without a slash is an off-road
tile, a tile containing "4" is a 4-way intersection (angle 2), anything else
without a slash is an off-road tile, 'empty' is no tile at all.  Each drivable
tile gets its cubic Bezier lane curves -- 2 for straight / curves, 6 for a
3-way, 12 for a 4-way (its 3-curve template at all four rotations) -- the
unit-tile template scaled by the tile size, rotated by ``pts @ R_y(angle *
pi / 2)`` (quaternion-form matrix) and translated to the tile centre.  The
computation is done once per map on the host in float64 with the same numpy
expressions, so the control points are the reference's.

Curves are stored compactly for the C ABI (dt_map): tile t owns curves
curve_start[t] .. curve_start[t+1]-1 of ``curves`` [C,4,3] / ``headings`` [C,3].
"""
import math
import os
from dataclasses import dataclass

import numpy as np
import yaml

MAP_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'maps')

TILE_EMPTY, TILE_OFFROAD, TILE_STRAIGHT, TILE_CURVE_LEFT, TILE_CURVE_RIGHT = -1, 0, 1, 2, 3
TILE_3WAY_LEFT, TILE_3WAY_RIGHT, TILE_4WAY = 4, 5, 6
KIND_CODES = {'straight': TILE_STRAIGHT, 'curve_left': TILE_CURVE_LEFT,
              'curve_right': TILE_CURVE_RIGHT, '3way_left': TILE_3WAY_LEFT,
              '3way_right': TILE_3WAY_RIGHT, '4way': TILE_4WAY}

# unit-tile lane templates (two lanes per tile, right-hand traffic)
LANE_TEMPLATES = {
    TILE_STRAIGHT: np.array([
        [[-0.20, 0, -0.50], [-0.20, 0, -0.25], [-0.20, 0, 0.25], [-0.20, 0, 0.50]],
        [[0.20, 0, 0.50], [0.20, 0, 0.25], [0.20, 0, -0.25], [0.20, 0, -0.50]],
    ]),
    TILE_CURVE_LEFT: np.array([
        [[-0.20, 0, -0.50], [-0.20, 0, 0.00], [0.00, 0, 0.20], [0.50, 0, 0.20]],
        [[0.50, 0, -0.20], [0.30, 0, -0.20], [0.20, 0, -0.30], [0.20, 0, -0.50]],
    ]),
    TILE_CURVE_RIGHT: np.array([
        [[-0.20, 0, -0.50], [-0.20, 0, -0.20], [-0.30, 0, -0.20], [-0.50, 0, -0.20]],
        [[-0.50, 0, 0.20], [-0.30, 0, 0.20], [0.30, 0, 0.00], [0.20, 0, -0.50]],
    ]),
    # 3-way: straight through both ways + the four turns to / from the side road
    TILE_3WAY_LEFT: np.array([
        [[-0.20, 0, -0.50], [-0.20, 0, -0.25], [-0.20, 0, 0.25], [-0.20, 0, 0.50]],
        [[-0.20, 0, -0.50], [-0.20, 0, 0.00], [0.00, 0, 0.20], [0.50, 0, 0.20]],
        [[0.20, 0, 0.50], [0.20, 0, 0.25], [0.20, 0, -0.25], [0.20, 0, -0.50]],
        [[0.50, 0, -0.20], [0.30, 0, -0.20], [0.20, 0, -0.20], [0.20, 0, -0.50]],
        [[0.20, 0, 0.50], [0.20, 0, 0.20], [0.30, 0, 0.20], [0.50, 0, 0.20]],
        [[0.50, 0, -0.20], [0.30, 0, -0.20], [-0.20, 0, 0.00], [-0.20, 0, 0.50]],
    ]),
    # 4-way: left / straight / right from one entry, rotated to all four sides
    TILE_4WAY: np.array([
        [[-0.20, 0, -0.50], [-0.20, 0, 0.00], [0.00, 0, 0.20], [0.50, 0, 0.20]],
        [[-0.20, 0, -0.50], [-0.20, 0, -0.25], [-0.20, 0, 0.25], [-0.20, 0, 0.50]],
        [[-0.20, 0, -0.50], [-0.20, 0, -0.20], [-0.30, 0, -0.20], [-0.50, 0, -0.20]],
    ]),
}
LANE_TEMPLATES[TILE_3WAY_RIGHT] = LANE_TEMPLATES[TILE_3WAY_LEFT]  # upstream: kind.startswith('3way')


def rotation_y(angle):
    """Counter-clockwise rotation about +y, upstream gen_rot_matrix form."""
    axis = np.array([0, 1, 0])
    axis = axis / math.sqrt(np.dot(axis, axis))
    a = math.cos(angle / 2.0)
    b, c, d = -axis * math.sin(angle / 2.0)
    return np.array([
        [a * a + b * b - c * c - d * d, 2 * (b * c - a * d), 2 * (b * d + a * c)],
        [2 * (b * c + a * d), a * a + c * c - b * b - d * d, 2 * (c * d - a * b)],
        [2 * (b * d - a * c), 2 * (c * d + a * b), a * a + d * d - b * b - c * c],
    ])


@dataclass
class TileMap:
    name: str
    width: int
    height: int
    tile_size: float
    kind: np.ndarray         # [H*W] int8
    orient: np.ndarray       # [H*W] int8
    curves: np.ndarray       # [C, 4, 3] float64, tile t's at curve_start[t]:curve_start[t+1]
    headings: np.ndarray     # [C, 3] float64
    curve_start: np.ndarray  # [H*W + 1] int32
    rows: list

    def tile_curves(self, t):
        return self.curves[self.curve_start[t]:self.curve_start[t + 1]]

    @property
    def drivable(self):
        return np.nonzero(self.kind > 0)[0]


def tile_curves(kind, orient, i, j, tile_size):
    """upstream _get_curve for one drivable tile."""
    pts = LANE_TEMPLATES[kind] * tile_size
    centre = np.array([(i + .5) * tile_size, 0, (j + .5) * tile_size])
    if kind == TILE_4WAY:
        sides = []
        for rot in np.arange(0, 4):
            side = np.matmul(pts, rotation_y(rot * math.pi / 2))
            side += centre
            sides.append(side)
        return np.reshape(np.array(sides), (12, 4, 3))
    pts = np.matmul(pts, rotation_y(int(orient) * math.pi / 2))
    pts += centre
    return pts


def parse_rows(rows, name='custom', tile_size=0.61):
    H, W = len(rows), len(rows[0])
    kind = np.full(H * W, TILE_EMPTY, np.int8)
    orient = np.zeros(H * W, np.int8)
    per_tile = [None] * (H * W)
    for j, row in enumerate(rows):
        if len(row) != W:
            raise ValueError('each row of tiles must have the same length')
        for i, tile in enumerate(row):
            tile = tile.strip()
            t = j * W + i
            if tile == 'empty':
                continue
            if '/' in tile:
                k, o = (s.strip(' ') for s in tile.split('/'))
                if k not in KIND_CODES:
                    raise NotImplementedError('tile kind %r' % k)
                kind[t] = KIND_CODES[k]
                orient[t] = ['S', 'E', 'N', 'W'].index(o)
            elif '4' in tile:        # upstream: kind '4way', angle 2
                kind[t] = TILE_4WAY
                orient[t] = 2
            else:
                kind[t] = TILE_OFFROAD
                continue
            per_tile[t] = tile_curves(int(kind[t]), orient[t], i, j, tile_size)
    counts = [0 if c is None else len(c) for c in per_tile]
    curve_start = np.zeros(H * W + 1, np.int32)
    curve_start[1:] = np.cumsum(counts)
    C = int(curve_start[-1])
    curves = np.zeros((C, 4, 3), np.float64)
    headings = np.zeros((C, 3), np.float64)
    for t, pts in enumerate(per_tile):
        if pts is None:
            continue
        a, b = curve_start[t], curve_start[t + 1]
        curves[a:b] = pts
        h = pts[:, -1, :] - pts[:, 0, :]          # closest_curve_point: one Frobenius norm
        headings[a:b] = h / np.linalg.norm(h).reshape(1, -1)
    return TileMap(name, W, H, tile_size, kind, orient, curves, headings, curve_start,
                   [list(r) for r in rows])


def load_map(name_or_path, tile_size=0.61):
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(MAP_DIR, name_or_path + '.yaml')
    with open(path) as f:
        doc = yaml.safe_load(f)
    if doc.get('objects'):
        raise NotImplementedError('maps with objects (collision / proximity penalty) are '
                                  'SURVEY §8f item 3')
    name = os.path.splitext(os.path.basename(path))[0]
    return parse_rows(doc['tiles'], name, tile_size)


def available_maps():
    return sorted(os.path.splitext(f)[0] for f in os.listdir(MAP_DIR) if f.endswith('.yaml'))
