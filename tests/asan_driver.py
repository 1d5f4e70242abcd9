"""Run under AddressSanitizer + UBSan by tests/test_asan.py (not collected by
pytest itself): the host-side entry points of libdtsim_asan.so (`make asan`:
host code instrumented; no kernel is launched here) on valid and invalid arguments, every
map through dt_create's validation, then the oracle's C restatement
(liboracle_asan.so) under the oracle tests.  torch is never imported here:
nothing in this process owns a GPU.  Exit status 0 = clean; a sanitizer
report aborts the process with a non-zero status."""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from aido1_amd import _lib  # noqa: E402  (ctypes only: no torch at import)
from aido1_amd.config import EnvConfig  # noqa: E402
from aido1_amd.maps import available_maps, load_map  # noqa: E402

DT_OK, DT_E_ARG, DT_E_NODEV = 0, -1, -4
vp, i32 = ctypes.c_void_p, ctypes.c_int32


def dt_map(m, kind=None, curve_start=None, curves=None):
    keep = [np.ascontiguousarray(m.kind if kind is None else kind, np.int8),
            np.ascontiguousarray(m.curve_start if curve_start is None else curve_start, np.int32),
            np.ascontiguousarray(m.curves if curves is None else curves, np.float64),
            np.ascontiguousarray(m.headings, np.float64),
            np.ascontiguousarray(m.object_table, np.float64),
            np.ascontiguousarray(m.spawn_table, np.float64)]
    p = [a.ctypes.data_as(vp) for a in keep]
    return _lib.DtMap(m.width, m.height, p[0], p[1], p[2], p[3], len(keep[4]), p[4],
                      len(keep[5]), p[5]), keep


def check_create(L):
    cfg = EnvConfig().to_c()
    h = vp()
    n_ok = 0
    for name in available_maps():
        m = load_map(name)
        dm, _keep = dt_map(m)
        rc = L.dt_create(ctypes.byref(cfg), ctypes.byref(dm), 1234, 64, 0, ctypes.byref(h))
        # every map passes the host validation; without a device the handle is refused
        assert rc in (DT_OK, DT_E_NODEV, -2), (name, rc, L.dt_last_error(None))
        n_ok += 1
        # malformed tables: refused with a message, nothing read past them
        cs = m.curve_start.copy()
        cs[0] = 1
        bad, _k = dt_map(m, curve_start=cs)
        assert L.dt_create(ctypes.byref(cfg), ctypes.byref(bad), 1, 64, 0,
                           ctypes.byref(h)) == DT_E_ARG
        assert b'curve_start' in L.dt_last_error(None)
        cv = m.curves.copy()
        if len(cv):
            cv[0, 1, 1] = 0.5          # a control point off the ground plane
            bad, _k = dt_map(m, curves=cv)
            assert L.dt_create(ctypes.byref(cfg), ctypes.byref(bad), 1, 64, 0,
                               ctypes.byref(h)) == DT_E_ARG
        kd = m.kind.copy()
        kd[np.nonzero(m.kind == 0)[0][:1]] = 1   # a curve-less tile made drivable
        if (m.kind == 0).any():
            bad, _k = dt_map(m, kind=kd)
            assert L.dt_create(ctypes.byref(cfg), ctypes.byref(bad), 1, 64, 0,
                               ctypes.byref(h)) == DT_E_ARG
    dm, _keep = dt_map(load_map('loop_empty'))
    for n in (0, -5):
        assert L.dt_create(ctypes.byref(cfg), ctypes.byref(dm), 1, n, 0,
                           ctypes.byref(h)) == DT_E_ARG
    assert L.dt_create(None, ctypes.byref(dm), 1, 8, 0, ctypes.byref(h)) == DT_E_ARG
    assert L.dt_create(ctypes.byref(cfg), None, 1, 8, 0, ctypes.byref(h)) == DT_E_ARG
    return n_ok


def check_entry_points(L):
    assert L.dt_abi_version() == _lib.ABI_VERSION
    gray = (ctypes.c_float * 8)()
    assert L.dt_palette_gray(gray) == DT_OK
    assert all(0.0 <= g <= 1.0 for g in gray)
    # dtupd.h's argument checks (tests/test_abi.py)
    parts = ctypes.c_int32(0)
    assert L.dt_upd_part_floats() == 256 * 32 * 3
    assert L.dt_upd_conv_fwd_part(16, 4, 2, 1, 57, 77, 1, None, 1, 1, 0.01, 1, 1,
                                  ctypes.byref(parts), None) != 0
    empty = _lib.DtUpdBn()
    assert L.dt_upd_conv_fwd_part(32, 4, 2, 1, 57, 77, 1, ctypes.byref(empty), 1, 1, 0.01, 1, 1,
                                  ctypes.byref(parts), None) != 0
    assert L.dt_upd_bn_finish(126, 7, 16, ctypes.byref(empty), 16, None) != 0
    assert L.dt_upd_linear_work_floats(64, 250, 4032) == -1
    assert L.dt_upd_linear_work_floats(64, 256, 4030) == -1
    assert L.dt_upd_linear_work_floats(64, 256, 4032) % (64 * 256) == 0
    assert L.dt_upd_linear_fwd(64, 256, 4032, None, 16, 16, 0, 0.0, 16, 16, None) != 0
    assert L.dt_upd_wgrad_work_floats(3, 8, 2, 64, 120, 160) == 512 * 32 * 192
    # the actor convolutions' refusals (null buffers, ring order out of range,
    # a second weight set past n) and n = 0 (nothing launched)
    o = (i32 * 3)(0, 1, 5)
    one = ctypes.c_void_p(16)
    assert L.dt_conv1_split(None, 4, 3, o, one, one, None, one, one, 0.01, None) == DT_E_ARG
    assert L.dt_conv1x_split(one, 1, 4, 3, o, one, one, None, one, one, 0.01, None) == DT_E_ARG
    o2 = (i32 * 3)(0, 1, 2)
    s2 = _lib.DtConvSet(9, 16, 16)
    assert L.dt_conv1x_split(one, 1, 4, 3, o2, one, one, ctypes.byref(s2), one, one, 0.01,
                             None) == DT_E_ARG
    assert L.dt_conv1x_split(one, 1, 0, 3, o2, one, one, None, one, one, 0.01, None) == DT_OK
    assert L.dt_conv32x_split(2, 4, one, one, one, None, one, one, 1e-5, one, one, None, None,
                              1e-5, 0.01, None, None) == DT_E_ARG
    assert L.dt_conv32x_split(4, 4, one, one, one, one, one, one, 1e-5, one, None, None, None,
                              1e-5, 0.01, None, None) == DT_E_ARG
    assert L.dt_conv32x_split(7, 4, one, one, one, one, one, one, 1e-5, one, one, one, one,
                              1e-5, 0.01, None, None) == DT_E_ARG
    assert L.dt_conv32x_split(3, 0, one, one, one, one, one, one, 1e-5, one, one, None, None,
                              1e-5, 0.01, None, None) == DT_OK
    for n, h, w in ((1, 120, 160), (4, 480, 640), (0, 1, 1)):
        assert L.dt_line_detect_workspace(n, h, w) >= 0


def main():
    L = _lib.bind(ctypes.CDLL(os.environ['DTSIM_ASAN_LIB'], mode=ctypes.RTLD_GLOBAL))
    check_entry_points(L)
    maps = check_create(L)
    print('libdtsim host entry points clean under ASan/UBSan (%d maps)' % maps, flush=True)
    # the oracle's C restatement under its own tests (this process's runtime)
    r = subprocess.run([sys.executable, '-m', 'pytest', '-q', '-x', '-p', 'no:cacheprovider',
                        '-m', 'not gpu and not slow', os.path.join(REPO, 'tests', 'test_oracle.py'),
                        os.path.join(REPO, 'tests', 'test_oracle_render.py')],
                       cwd=REPO, env=os.environ)
    sys.exit(r.returncode)


if __name__ == '__main__':
    main()
