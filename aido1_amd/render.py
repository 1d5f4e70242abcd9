"""Observation path host API (BASELINE.json configs[2]).

- ``RenderOutput`` + ``VecEnv.render_into``: the fused gfx950 kernel that draws
  each env's 120x160 ego-centric top-down frame (build-defined replacement of
  Simulator.render_obs), converts it to grey (PreliminaryTransformer,
  utils/reward_shaping/env_utils.py:48-51) straight into a 3-slot frame ring
  (the Transformer stack, env_utils.py:54-70) and runs the
  features/line_detector1.py colour/edge filter on it.
- ``line_detect``: LineDetectorHSV (setImage + _colorFilter for white, yellow,
  red + the Canny edge map) on caller-supplied BGR images.
- ``stack_view``: the Transformer's oldest-first [N,3,120,160] view of the ring.
- Palette-index frames (``RenderOutput(frames='index')``): the ring holds each
  frame's palette bytes (u8, a quarter of the grey frame) instead of its grey
  floats; ``decode_index`` / ``palette_gray`` give the grey frame bit for bit
  (the renderer's grey IS the palette's grey table applied to those bytes),
  and the actor's first conv and the replay's gather decode them on the fly.
- ``hough_lines`` / ``find_normals`` / ``detect_lines``: LineDetectorHSV's
  _HoughLine, _findNormal and detectLines on those masks.
"""
import ctypes

import torch

from aido1_amd import _lib

H, W = 120, 160
NPIX = H * W
MASK_WHITE, MASK_YELLOW, MASK_RED, MASK_EDGES = range(4)

# Algorithmic HBM bytes per env per render launch (DESIGN.md "render kernel"):
# writes: grey frame f32 76,800 + 4 u8 masks 76,800; reads: pose 24.
RENDER_BYTES_PER_ENV = 4 * NPIX + 4 * NPIX + 24
# ... plus, per env respawned by the step before it, the first frame into the
# ring's other two slots (Transformer.reset stacks three copies,
# utils/reward_shaping/env_utils.py:60-63)
RENDER_BYTES_PER_FRESH = 2 * 4 * NPIX
# the same with palette-index frames (1 byte a pixel instead of 4)
RENDER_INDEX_BYTES_PER_ENV = NPIX + 4 * NPIX + 24
RENDER_INDEX_BYTES_PER_FRESH = 2 * NPIX

_GRAY = {}


def palette_gray(device):
    """The renderer's 8 grey levels (dt_palette_gray) as a float32 tensor on
    `device`: grey frame = palette_gray[index frame]."""
    key = str(torch.device(device))
    if key not in _GRAY:
        buf = (ctypes.c_float * 8)()
        if _lib.lib().dt_palette_gray(buf) != 0:
            raise _lib.DtError('dt_palette_gray failed')
        _GRAY[key] = torch.tensor(list(buf), dtype=torch.float32, device=device)
    return _GRAY[key]


def decode_index(frames):
    """Grey frames (float32, same shape) from palette-index frames (uint8)."""
    if frames.dtype != torch.uint8:
        raise ValueError('decode_index: uint8 palette-index frames expected')
    return palette_gray(frames.device)[frames.long()]


def as_gray(frames):
    """frames as grey float32: decoded if they are palette-index frames."""
    return decode_index(frames) if frames.dtype == torch.uint8 else frames


class LineParams(ctypes.Structure):
    """Mirror of dt_line_params (include/dtsim.h)."""
    _fields_ = [('hsv_white1', ctypes.c_uint8 * 3), ('hsv_white2', ctypes.c_uint8 * 3),
                ('hsv_yellow1', ctypes.c_uint8 * 3), ('hsv_yellow2', ctypes.c_uint8 * 3),
                ('hsv_red1', ctypes.c_uint8 * 3), ('hsv_red2', ctypes.c_uint8 * 3),
                ('hsv_red3', ctypes.c_uint8 * 3), ('hsv_red4', ctypes.c_uint8 * 3),
                ('dilation_kernel_size', ctypes.c_int32),
                ('canny_lo', ctypes.c_double), ('canny_hi', ctypes.c_double)]

    @classmethod
    def default(cls):
        p = cls()
        _lib.lib().dt_default_line_params(ctypes.byref(p))
        return p

    @classmethod
    def from_config(cls, cfg):
        """From a LineDetectorHSV configuration dict (features/line_detector1.py:18-34 keys)."""
        p = cls.default()
        for k in ('hsv_white1', 'hsv_white2', 'hsv_yellow1', 'hsv_yellow2', 'hsv_red1',
                  'hsv_red2', 'hsv_red3', 'hsv_red4'):
            if k in cfg:
                getattr(p, k)[:] = [int(v) for v in cfg[k]]
        if 'dilation_kernel_size' in cfg:
            p.dilation_kernel_size = int(cfg['dilation_kernel_size'])
        if 'canny_thresholds' in cfg:
            p.canny_lo, p.canny_hi = (float(v) for v in cfg['canny_thresholds'])
        return p


class RenderIO(ctypes.Structure):
    _fields_ = [('gray', ctypes.c_void_p), ('gray_slots', ctypes.c_int32),
                ('gray_slot', ctypes.c_int32), ('fresh', ctypes.c_void_p),
                ('masks', ctypes.c_void_p), ('rgb', ctypes.c_void_p),
                ('pose', ctypes.c_void_p), ('list_cap', ctypes.c_int32),
                ('index', ctypes.c_void_p)]


FRAME_DTYPES = {'gray': torch.float32, 'index': torch.uint8}


class RenderOutput:
    """Device buffers of the observation path for n envs: a 3-slot frame
    ring (the Transformer's stack, see stack_view) of grey floats
    (frames='gray') or palette-index bytes (frames='index'), the 4 line masks
    of the latest frame, optionally the RGB raster."""

    def __init__(self, n, device, slots=3, rgb=False, masks=True, ring=None, frames='gray'):
        self.n = n
        self.slots = slots
        self.slot = -1  # slot of the newest frame
        self.frames = frames
        dt = FRAME_DTYPES[frames]
        self._all = torch.ones(n, dtype=torch.uint8, device=device)
        if ring is not None:  # a contiguous [n, slots, 120, 160] view (e.g. a slice)
            assert ring.is_contiguous() and tuple(ring.shape) == (n, slots, H, W)
            assert ring.dtype == dt
        self.ring = ring if ring is not None else torch.zeros(n, slots, H, W, dtype=dt,
                                                              device=device)
        self.masks = torch.zeros(n, 4, H, W, dtype=torch.uint8, device=device) if masks else None
        self.rgb = torch.zeros(n, H, W, 3, dtype=torch.uint8, device=device) if rgb else None

    def restart(self):
        """Next render fills every slot (after VecEnv.reset(): Transformer.reset)."""
        self.slot = -1

    def advance(self):
        self.slot = (self.slot + 1) % self.slots
        return self.slot

    def order(self):
        """Ring slots oldest -> newest (the Transformer's concatenation order)."""
        return [(self.slot + 1 + k) % self.slots for k in range(self.slots)]

    def stack_view(self, raw=False):
        """[n, 3, 120, 160] oldest-first grey stack (a gather copy; the actor
        consumes the ring zero-copy by permuting its first conv's input channels
        instead); raw=True keeps the ring's own dtype (index frames as bytes)."""
        st = self.ring[:, self.order()]
        return st if raw else as_gray(st)


def _render_io(env, out, fresh, pose, list_cap):
    if out.slot < 0:
        fresh = out._all
    slot = out.advance()
    if pose is not None and (pose.dtype != torch.float64 or not pose.is_contiguous() or
                             tuple(pose.shape) != (3, env.n) or pose.device != env.device):
        raise ValueError('pose must be a contiguous float64 [3, %d] tensor on %s'
                         % (env.n, env.device))
    idx = out.ring.dtype == torch.uint8
    ring = ctypes.c_void_p(out.ring.data_ptr())
    return RenderIO(None if idx else ring, out.slots, slot,
                    ctypes.c_void_p(fresh.data_ptr()) if fresh is not None else None,
                    ctypes.c_void_p(out.masks.data_ptr()) if out.masks is not None else None,
                    ctypes.c_void_p(out.rgb.data_ptr()) if out.rgb is not None else None,
                    ctypes.c_void_p(pose.data_ptr()) if pose is not None else None,
                    int(list_cap), ring if idx else None)


def render_into(env, out, fresh=None, pose=None, list_cap=0):
    """Render every env's current pose (or `pose`, a [3, n] f64 x/z/angle
    snapshot from VecEnv.copy_pose) into `out`, advancing the frame ring.
    fresh: optional [n] u8 device tensor; nonzero -> the frame fills every slot
    (Transformer.reset semantics): pass the done flags of an auto-resetting
    step.  The first render after RenderOutput creation / restart() fills every
    slot of every env.  list_cap > 0 (tests only) forces the kernel's
    global-memory overflow path."""
    io = _render_io(env, out, fresh, pose, list_cap)
    rc = env._L.dt_render(env._h, ctypes.byref(io), env._stream())
    env._check(rc, 'dt_render')
    return out


def bind_render(env, out, stream, fresh=None, pose=None):
    """A zero-argument callable that launches render_into(out, fresh, pose) on
    `stream` (a torch.cuda.Stream) with its ctypes arguments built once, for
    timed loops.  The ring slot is taken (advanced) at bind time, so bind the
    calls of consecutive decisions in their order.  Returns dt_render's status."""
    io = _render_io(env, out, fresh, pose, 0)
    fn, h, st = env._L.dt_render, env._h, ctypes.c_void_p(stream.cuda_stream)
    ref = ctypes.byref(io)
    keep = (out, fresh, pose, io, stream)

    def launch():
        keep  # noqa: B018 (the buffers stay alive with the callable)
        return fn(h, ref, st)
    return launch


def _group_ios(env, out, masks, fresh, pose):
    """The dt_render_io of 2 or 3 consecutive decisions of one ring: decision
    0 writes out.masks, decision i > 0 masks[i - 1]."""
    k = len(pose)
    if k not in (2, 3) or len(fresh) != k or len(masks) != k - 1:
        raise ValueError('a render group is 2 or 3 decisions (k - 1 extra masks buffers)')
    if out.masks is None or out.rgb is not None or any(
            m is None or m.shape != out.masks.shape or m.data_ptr() == out.masks.data_ptr()
            for m in masks) or len({m.data_ptr() for m in masks}) != len(masks):
        raise ValueError('render group: separate masks buffers of out.masks\' shape, no rgb')
    if any(p is None for p in pose):
        raise ValueError('render group: every decision\'s pose snapshot')
    ios = [_render_io(env, out, f, p, 0) for f, p in zip(fresh, pose)]
    for io, m in zip(ios[1:], masks):
        io.masks = ctypes.c_void_p(m.data_ptr())
    return ios


def render_group_into(env, out, masks, fresh, pose):
    """2 or 3 consecutive decisions' renders in ONE launch (dt_render2 /
    dt_render3): decision i of the lists (fresh[i], pose[i]) into ring slot
    after the newest + i, its masks into out.masks (i = 0) or masks[i - 1].
    Every output equals render_into of each decision in order."""
    ios = _group_ios(env, out, masks, fresh, pose)
    fn = env._L.dt_render2 if len(ios) == 2 else env._L.dt_render3
    rc = fn(env._h, *[ctypes.byref(io) for io in ios], env._stream())
    env._check(rc, 'dt_render%d' % len(ios))
    return out


def render2_into(env, out, masks_b, fresh_a, pose_a, fresh_b, pose_b):
    """render_group_into of two decisions."""
    return render_group_into(env, out, [masks_b], [fresh_a, fresh_b], [pose_a, pose_b])


def bind_render_group(env, out, stream, masks, fresh, pose):
    """bind_render for render_group_into (2 or 3 decisions, one launch)."""
    ios = _group_ios(env, out, masks, fresh, pose)
    fn = env._L.dt_render2 if len(ios) == 2 else env._L.dt_render3
    refs = [ctypes.byref(io) for io in ios]
    h, st = env._h, ctypes.c_void_p(stream.cuda_stream)
    keep = (out, masks, fresh, pose, ios, stream)

    def launch():
        keep  # noqa: B018
        return fn(h, *refs, st)
    return launch


def bind_render2(env, out, stream, masks_b, fresh_a, pose_a, fresh_b, pose_b):
    """bind_render_group of two decisions."""
    return bind_render_group(env, out, stream, [masks_b], [fresh_a, fresh_b], [pose_a, pose_b])


def line_detect(bgr, params=None, hsv=False, stream=None):
    """LineDetectorHSV.setImage + _colorFilter (features/line_detector1.py
    :134-141, :36-57) on a [n, h, w, 3] uint8 BGR CUDA tensor of any size.
    Images of <= 19200 pixels run in LDS; larger ones (the 640x480 camera frame
    of duckietown_rl/env.py:12-16) through a device workspace
    (dt_line_detect_ws).  Returns masks [n, 4, h, w] u8 ({white, yellow, red,
    edges}) and, if hsv, the cvtColor(BGR2HSV) image [n, h, w, 3]."""
    L = _lib.lib()
    if bgr.dtype != torch.uint8 or bgr.dim() != 4 or bgr.shape[3] != 3 or not bgr.is_cuda:
        raise ValueError('bgr must be a [n,h,w,3] uint8 CUDA tensor')
    bgr = bgr.contiguous()
    n, h, w, _ = bgr.shape
    p = params or LineParams.default()
    masks = torch.empty(n, 4, h, w, dtype=torch.uint8, device=bgr.device)
    hsv_t = torch.empty(n, h, w, 3, dtype=torch.uint8, device=bgr.device) if hsv else None
    if n == 0:
        return (masks, hsv_t) if hsv else masks
    nbytes = L.dt_line_detect_workspace(n, h, w)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=bgr.device) if nbytes else None
    s = stream if stream is not None else torch.cuda.current_stream(bgr.device).cuda_stream
    rc = L.dt_line_detect_ws(ctypes.byref(p), ctypes.c_void_p(bgr.data_ptr()), n, h, w,
                             ctypes.c_void_p(masks.data_ptr()),
                             ctypes.c_void_p(hsv_t.data_ptr()) if hsv else None,
                             ctypes.c_void_p(ws.data_ptr()) if ws is not None else None,
                             nbytes, ctypes.c_void_p(s))
    if rc != 0:
        raise _lib.DtError('dt_line_detect failed (%d)' % rc)
    return (masks, hsv_t) if hsv else masks


# ---- LineDetectorHSV.detectLines (features/line_detector1.py:63-132) ------------------
# Hough parameters are not in the reference (dtu.Configurable, :18-34); these
# are the Duckietown line-detector defaults (recalled).
HOUGH_DEFAULTS = {'hough_threshold': 2, 'hough_min_line_length': 3, 'hough_max_line_gap': 1}
COLOR_PLANE = {'white': MASK_WHITE, 'yellow': MASK_YELLOW, 'red': MASK_RED}


HOUGH_TRUNCATED = -2   # dt_hough_lines: max_lines reached with points left
HOUGH_OVERFLOW = -1    # dt_hough_lines: more edge pixels than the LDS list holds


def hough_lines(edge, threshold=2, min_line_length=3, max_line_gap=1, max_lines=512,
                stream=None, workspace=None):
    """_HoughLine (:63-70): cv2.HoughLinesP(edge, 1, pi/180, threshold,
    min_line_length, max_line_gap) on a [n, h, w] uint8 CUDA tensor (non-zero =
    edge), one wave per image (include/dtsim.h dt_hough_lines).  Returns
    (lines [n, max_lines, 4] int32 (x1, y1, x2, y2) in OpenCV's order, counts
    [n] int32).  A count of -2 (HOUGH_TRUNCATED) marks an image that reached
    max_lines with edge points still unvisited; -1 (HOUGH_OVERFLOW) one with
    more edge pixels than the LDS point list holds.  workspace: None = the LDS
    kernel where the image fits (else the workspace kernel), True = always the
    workspace kernel (any size, never -1)."""
    L = _lib.lib()
    if edge.dtype != torch.uint8 or edge.dim() != 3 or not edge.is_cuda:
        raise ValueError('edge must be a [n,h,w] uint8 CUDA tensor')
    edge = edge.contiguous()
    n, h, w = edge.shape
    lines = torch.zeros(n, max_lines, 4, dtype=torch.int32, device=edge.device)
    counts = torch.zeros(n, dtype=torch.int32, device=edge.device)
    if n == 0:
        return lines, counts
    if threshold < 1 or max_lines < 1:
        raise ValueError('threshold and max_lines must be >= 1')
    s = stream if stream is not None else torch.cuda.current_stream(edge.device).cuda_stream
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def run(ws, nbytes):
        return L.dt_hough_lines_ws(ptr(edge), n, h, w, int(threshold), int(min_line_length),
                                   int(max_line_gap), int(max_lines), ptr(lines), ptr(counts),
                                   ptr(ws) if ws is not None else None, nbytes,
                                   ctypes.c_void_p(s))
    # the LDS kernel refuses (DT_E_ARG) an image whose accumulator does not fit
    rc = run(None, 0) if not workspace else -1
    if rc != 0:
        nbytes = L.dt_hough_workspace(n, h, w)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=edge.device)
        rc = run(ws, nbytes)
        if rc == 0 and stream is not None:   # the workspace lives until that stream is past it
            ws.record_stream(torch.cuda.ExternalStream(s, device=edge.device))
    if rc != 0:
        raise _lib.DtError('dt_hough_lines failed (%d)' % rc)
    return lines, counts


def find_normals(bw, lines, counts):
    """_findNormal + _correctPixelOrdering (:72-123), batched on the device:
    bw [n, h, w] (the dilated colour mask), lines [n, L, 4] int32 with counts
    [n] valid rows.  Returns (lines reordered in place of a copy, centers
    [n, L, 2] f64, normals [n, L, 2] f64); rows past counts[i] are zero.  The
    arithmetic is the reference's float64 numpy, operation for operation."""
    n, nl, _ = lines.shape
    h, w = bw.shape[1], bw.shape[2]
    valid = torch.arange(nl, device=lines.device).view(1, nl) < counts.view(n, 1)
    x1, y1, x2, y2 = (lines[..., k].to(torch.int64) for k in range(4))
    length = ((x1 - x2) ** 2 + (y1 - y2) ** 2).to(torch.float64).sqrt()
    length = torch.where(valid, length, torch.ones_like(length))
    dx = (y2 - y1).to(torch.float64) / length
    dy = (x1 - x2).to(torch.float64) / length
    cx = (x1 + x2).to(torch.float64) / 2
    cy = (y1 + y2).to(torch.float64) / 2

    def bound(v, b):
        v = v.to(torch.int64)            # .astype('int'): truncation toward zero
        return v.clamp(0, b - 1)
    x3, y3 = bound(cx - 3. * dx, w), bound(cy - 3. * dy, h)
    x4, y4 = bound(cx + 3. * dx, w), bound(cy + 3. * dy, h)
    img = torch.arange(n, device=lines.device).view(n, 1)
    sign = ((bw[img, y3, x3] > 0) & (bw[img, y4, x4] == 0)).to(torch.float64) * 2 - 1
    nx, ny = dx * sign, dy * sign
    flip = ((x2 - x1).to(torch.float64) * ny - (y2 - y1).to(torch.float64) * nx) > 0
    out = torch.where(flip.unsqueeze(-1), lines[..., [2, 3, 0, 1]], lines)
    zero = torch.zeros_like(cx)
    centers = torch.stack([torch.where(valid, cx, zero), torch.where(valid, cy, zero)], -1)
    normals = torch.stack([torch.where(valid, nx, zero), torch.where(valid, ny, zero)], -1)
    out = torch.where(valid.unsqueeze(-1), out, torch.zeros_like(out))
    return out, centers, normals


def detect_lines(masks, color, params=None, max_lines=512):
    """detectLines(color) (:125-132) for every image of a dt_render /
    line_detect mask batch [n, 4, h, w]: bw = the dilated colour plane,
    edge_color = bw AND the edge plane (_colorFilter :55), Hough, normals.
    Returns a dict with the reference Detections fields (lines, normals, area,
    centers) plus counts (valid rows per image)."""
    p = dict(HOUGH_DEFAULTS, **(params or {}))
    bw = masks[:, COLOR_PLANE[color]]
    edge_color = bw & masks[:, MASK_EDGES]
    args = (p['hough_threshold'], p['hough_min_line_length'], p['hough_max_line_gap'])
    ws = None
    lines, counts = hough_lines(edge_color, *args, max_lines)
    if bool((counts == HOUGH_OVERFLOW).any()):   # past the LDS point list: workspace kernel
        ws = True
        lines, counts = hough_lines(edge_color, *args, max_lines, workspace=ws)
    while bool((counts == HOUGH_TRUNCATED).any()):   # OpenCV has no cap: grow the list
        max_lines *= 2
        lines, counts = hough_lines(edge_color, *args, max_lines, workspace=ws)
    lines, centers, normals = find_normals(bw, lines, counts)
    return {'lines': lines, 'normals': normals, 'area': bw, 'centers': centers,
            'counts': counts}
