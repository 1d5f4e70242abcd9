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

Static objects follow upstream Simulator._load_objects and
collision.py: world position = tile_size * (x, y, z), scale = height /
mesh max y, footprint corners = the mesh's x/z box scaled, offset to the
position and rotated about it by `rotate` degrees (rotate_point), axes =
generate_norm (eigenvectors of the corners' covariance -- for a square
footprint that is the world x/z axes whatever the rotation, as upstream),
safety radius = SAFETY_RAD_MULT * hypot(max |x|, max |z|) * scale.  An object
is collidable (checked by _collision / proximity_penalty2) when it is static,
not a traffic light, and its box meets a drivable tile (_collidable_object);
every object counts for _inconvenient_spawn.  The meshes are not in this
container, so the per-kind boxes below are assumptions (override them per
object with ``mesh_min`` / ``mesh_max``).
"""
import math
import os
from dataclasses import dataclass

import numpy as np
import yaml

MAP_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'maps')

SAFETY_RAD_MULT = 1.8
MIN_SPAWN_OBJ_DIST = 0.25
# mesh bounding boxes (min, max) in mesh units, y up -- ASSUMED (the upstream
# .obj meshes are absent); with `height` only their proportions matter
MESH_EXTENTS = {
    'duckie': ((-0.5, 0.0, -0.4), (0.5, 1.0, 0.4)),
    'cone': ((-0.35, 0.0, -0.35), (0.35, 1.0, 0.35)),
    'barrier': ((-1.0, 0.0, -0.2), (1.0, 1.0, 0.2)),
    'duckiebot': ((-0.6, 0.0, -0.45), (0.6, 1.0, 0.45)),
    'truck': ((-1.2, 0.0, -0.5), (1.2, 1.0, 0.5)),
    'bus': ((-1.5, 0.0, -0.5), (1.5, 1.0, 0.5)),
    'house': ((-0.6, 0.0, -0.5), (0.6, 1.0, 0.5)),
    'building': ((-0.6, 0.0, -0.6), (0.6, 1.0, 0.6)),
    'tree': ((-0.4, 0.0, -0.4), (0.4, 1.0, 0.4)),
    'trafficlight': ((-0.1, 0.0, -0.1), (0.1, 1.0, 0.1)),
    'sign': ((-0.15, 0.0, -0.02), (0.15, 1.0, 0.02)),
}

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


# ---- static objects: upstream collision.py restated -----------------------------------
def rotate_point(px, py, cx, cy, theta):
    """Rotate (px, py) about (cx, cy) by theta (upstream graphics/collision)."""
    dx = px - cx
    dy = py - cy
    new_dx = dx * math.cos(theta) + dy * math.sin(theta)
    new_dy = dy * math.cos(theta) - dx * math.sin(theta)
    return cx + new_dx, cy + new_dy


def generate_corners(pos, min_coords, max_coords, theta, scale):
    """Footprint corners [4, 2] (x, z) of an object at world `pos`."""
    px, pz = pos[0], pos[-1]
    return np.array([
        rotate_point(min_coords[0] * scale + px, min_coords[-1] * scale + pz, px, pz, theta),
        rotate_point(max_coords[0] * scale + px, min_coords[-1] * scale + pz, px, pz, theta),
        rotate_point(max_coords[0] * scale + px, max_coords[-1] * scale + pz, px, pz, theta),
        rotate_point(min_coords[0] * scale + px, max_coords[-1] * scale + pz, px, pz, theta),
    ])


def generate_norm(corners):
    """The box's two axes (rows, unit): eigenvectors of the corners' covariance."""
    ca = np.cov(corners, y=None, rowvar=False, bias=True)
    _, vect = np.linalg.eig(ca)
    return np.ascontiguousarray(vect.T.real)


def _proj(corners, axis):
    p = corners @ axis
    return p.min(), p.max()


def sat_intersects(c1, n1, c2, n2):
    """Separating-axis test of two boxes (corners [4,2], axes [2,2]): no axis of
    either separates their closed projection intervals."""
    for axis in np.concatenate([n1, n2]):
        a0, a1 = _proj(c1, axis)
        b0, b1 = _proj(c2, axis)
        if a1 < b0 or b1 < a0:
            return False
    return True


def tile_corners(i, j, width):
    px, pz = i * width, j * width
    return np.array([[px, pz], [px + width, pz], [px + width, pz + width], [px, pz + width]])


def find_candidate_tiles(corners, tile_size):
    mn = np.floor(np.amin(corners, axis=0) / tile_size).astype(int)
    mx = np.floor(np.amax(corners, axis=0) / tile_size).astype(int)
    return [(x, y) for x in range(mn[0], mx[0] + 1) for y in range(mn[1], mx[1] + 1)]


@dataclass
class MapObject:
    kind: str
    pos: np.ndarray            # world (x, y, z)
    rotate: float              # degrees
    scale: float
    min_coords: np.ndarray
    max_coords: np.ndarray
    static: bool
    corners: np.ndarray        # [4, 2]
    norms: np.ndarray          # [2, 2]
    safety_radius: float
    collidable: bool = False

    @property
    def spawn_radius(self):
        """_inconvenient_spawn: max(max_coords) * 0.5 * scale + MIN_SPAWN_OBJ_DIST."""
        return float(np.max(self.max_coords)) * 0.5 * self.scale + MIN_SPAWN_OBJ_DIST

    def record(self):
        """The DT_OBJ_STRIDE doubles of include/dtsim.h for this object."""
        r = np.zeros(20, np.float64)
        r[0:3] = self.pos
        r[3] = self.safety_radius
        r[4:12] = self.corners.reshape(-1)
        r[12:16] = self.norms.reshape(-1)
        for a in range(2):
            r[16 + 2 * a:18 + 2 * a] = _proj(self.corners, self.norms[a])
        return r


def parse_object(desc, tile_size):
    kind = desc['kind']
    pos = desc['pos']
    x, z = pos[0:2]
    y = pos[2] if len(pos) == 3 else 0.0
    world = tile_size * np.array((x, y, z), np.float64)
    if 'mesh_min' in desc or 'mesh_max' in desc:
        mn, mx = desc['mesh_min'], desc['mesh_max']
    elif kind in MESH_EXTENTS or kind.startswith('sign'):
        mn, mx = MESH_EXTENTS[kind if kind in MESH_EXTENTS else 'sign']
    else:
        raise ValueError('object kind %r has no known extents: give mesh_min / mesh_max' % kind)
    mn = np.array(mn, np.float64)
    mx = np.array(mx, np.float64)
    if 'height' in desc and 'scale' in desc:
        raise ValueError('cannot specify both height and scale')
    scale = desc['height'] / mx[1] if 'height' in desc else float(desc.get('scale', 1.0))
    static = bool(desc.get('static', True))
    if not static:
        raise NotImplementedError('dynamic (non-static) objects are not supported')
    rotate = float(desc.get('rotate', 0.0))
    corners = generate_corners(world, mn, mx, np.radians(rotate), scale)
    ext = np.max([np.abs(mn), np.abs(mx)], axis=0)
    safety = SAFETY_RAD_MULT * (np.hypot(ext[0], ext[2]) * scale)
    return MapObject(kind, world, rotate, scale, mn, mx, static, corners,
                     generate_norm(corners), float(safety))


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
    objects: list = None     # [MapObject]

    def tile_curves(self, t):
        return self.curves[self.curve_start[t]:self.curve_start[t + 1]]

    @property
    def object_table(self):
        """[K, 20] float64 records of the collidable objects (dt_map.objects)."""
        recs = [o.record() for o in (self.objects or []) if o.collidable]
        return np.array(recs, np.float64).reshape(-1, 20)

    @property
    def spawn_table(self):
        """[M, 4] float64 (x, y, z, radius) of every object (dt_map.spawn_objects)."""
        recs = [np.r_[o.pos, o.spawn_radius] for o in (self.objects or [])]
        return np.array(recs, np.float64).reshape(-1, 4)

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


def parse_rows(rows, name='custom', tile_size=0.61, objects=()):
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
    objs = [parse_object(d, tile_size) for d in objects]
    for o in objs:   # _collidable_object: static, not a traffic light, meets a drivable tile
        if o.kind == 'trafficlight':
            continue
        for (ti, tj) in find_candidate_tiles(o.corners, tile_size):
            if 0 <= ti < W and 0 <= tj < H and kind[tj * W + ti] > 0 and sat_intersects(
                    o.corners, o.norms, tile_corners(ti, tj, tile_size),
                    np.array([[1.0, 0.0], [0.0, 1.0]])):
                o.collidable = True
                break
    return TileMap(name, W, H, tile_size, kind, orient, curves, headings, curve_start,
                   [list(r) for r in rows], objs)


def load_map(name_or_path, tile_size=0.61):
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(MAP_DIR, name_or_path + '.yaml')
    with open(path) as f:
        doc = yaml.safe_load(f)
    objects = doc.get('objects') or []
    if isinstance(objects, dict):   # newer map format: named objects
        objects = list(objects.values())
    name = os.path.splitext(os.path.basename(path))[0]
    return parse_rows(doc['tiles'], name, tile_size, objects)


def available_maps():
    return sorted(os.path.splitext(f)[0] for f in os.listdir(MAP_DIR) if f.endswith('.yaml'))
