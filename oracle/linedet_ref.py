"""TEST INFRASTRUCTURE ONLY — CPU restatement of LineDetectorHSV's line
stage for the dt_hough_lines / render.find_normals parity tests:
  * hough_lines: oracle/hough_oracle.c (cv2.HoughLinesP restated; OpenCV is
    absent, so parity against OpenCV itself is unpinned);
  * find_normals: features/line_detector1.py:72-123 (_checkBounds,
    _correctPixelOrdering, _findNormal) in the reference's own numpy float64
    operations, on int32 lines as cv2 returns them."""
import ctypes
import os

import numpy as np

from oracle import oracle_c as OC

_tab = None


def _lib():
    if not os.path.exists(OC.SO):
        OC.build()
    L = ctypes.CDLL(OC.SO)
    L.oracle_hough_table.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
                                     ctypes.c_int]
    L.oracle_hough_lines.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p]
    return L


def hough_lines(edge, threshold=2, min_line_length=3, max_line_gap=1, max_lines=512,
                trace=None):
    """edge: [h, w] uint8 -> int32 [k, 4] (x1, y1, x2, y2), OpenCV's order.
    trace: optional int32 [4096, 4] array that receives (idx, pixel, max
    count, its angle) per visited point that votes (diagnostics)."""
    L = _lib()
    tab = np.zeros(360, np.float32)
    theta = np.float32(np.pi / 180)
    na = L.oracle_hough_table(1.0, float(theta), tab.ctypes.data, 180)
    img = np.ascontiguousarray(edge, np.uint8)
    h, w = img.shape
    out = np.zeros((max_lines, 4), np.int32)
    k = L.oracle_hough_lines(img.ctypes.data, h, w, 1.0, tab.ctypes.data, na, threshold,
                             min_line_length, max_line_gap, max_lines, out.ctypes.data,
                             trace.ctypes.data if trace is not None else None)
    return out[:k].copy()


def _check_bounds(val, bound):
    val[val < 0] = 0
    val[val >= bound] = bound - 1
    return val


def find_normals(bw, lines):
    """_findNormal(bw, lines) (:84-123): returns (lines reordered, centers,
    normals) exactly as the reference computes them."""
    lines = np.array(lines, np.int32).reshape(-1, 4)
    normals, centers = [], []
    if len(lines) > 0:
        length = np.sum((lines[:, 0:2] - lines[:, 2:4]) ** 2, axis=1, keepdims=True) ** 0.5
        dx = 1. * (lines[:, 3:4] - lines[:, 1:2]) / length
        dy = 1. * (lines[:, 0:1] - lines[:, 2:3]) / length
        centers = np.hstack([(lines[:, 0:1] + lines[:, 2:3]) / 2,
                             (lines[:, 1:2] + lines[:, 3:4]) / 2])
        x3 = (centers[:, 0:1] - 3. * dx).astype('int')
        y3 = (centers[:, 1:2] - 3. * dy).astype('int')
        x4 = (centers[:, 0:1] + 3. * dx).astype('int')
        y4 = (centers[:, 1:2] + 3. * dy).astype('int')
        x3 = _check_bounds(x3, bw.shape[1])
        y3 = _check_bounds(y3, bw.shape[0])
        x4 = _check_bounds(x4, bw.shape[1])
        y4 = _check_bounds(y4, bw.shape[0])
        flag_signs = (np.logical_and(bw[y3, x3] > 0, bw[y4, x4] == 0)).astype('int') * 2 - 1
        normals = np.hstack([dx, dy]) * flag_signs
        flag = ((lines[:, 2] - lines[:, 0]) * normals[:, 1] -
                (lines[:, 3] - lines[:, 1]) * normals[:, 0]) > 0
        for i in range(len(lines)):
            if flag[i]:
                x1, y1, x2, y2 = lines[i, :]
                lines[i, :] = [x2, y2, x1, y1]
    return lines, np.asarray(centers, np.float64).reshape(-1, 2), \
        np.asarray(normals, np.float64).reshape(-1, 2)
