"""The C-ABI boundary: libdtsim.so builds for gfx950, exports exactly what
include/dtsim.h declares, its ctypes mirrors match the header's layout, and the
product fails loudly (no CPU fallback) when no GPU is present."""
import ctypes
import os
import subprocess

import pytest

from conftest import REPO


@pytest.fixture(scope='module')
def libpath():
    from aido1_amd import _lib
    return _lib.build()


def test_exports_every_declared_symbol(libpath):
    from aido1_amd import _lib
    declared = _lib.exported_symbols()
    assert len(declared) >= 12
    nm = subprocess.run(['nm', '-D', '--defined-only', libpath], capture_output=True,
                        text=True, check=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if ' T ' in line}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing


def test_code_object_is_gfx950(libpath):
    data = open(libpath, 'rb').read()
    assert b'amdgcn-amd-amdhsa--gfx950' in data
    assert b'gfx942' not in data and b'gfx90a' not in data


def test_struct_layout_matches_header(tmp_path):
    from aido1_amd._lib import DtMap
    from aido1_amd.config import DtConfig
    src = tmp_path / 'layout.c'
    fields = [f[0] for f in DtConfig._fields_]
    body = '\n'.join('printf("%%zu ", offsetof(dt_config, %s));' % f for f in fields)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "dtsim.h"\nint main(){'
                   + body + 'printf("%zu %zu %zu\\n", sizeof(dt_config), sizeof(dt_map),'
                   ' offsetof(dt_map, headings)); return 0;}')
    exe = tmp_path / 'layout'
    subprocess.run(['gcc', '-I', os.path.join(REPO, 'include'), '-o', str(exe), str(src)],
                   check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                           check=True).stdout.split()]
    offs = [getattr(DtConfig, f).offset for f in fields]
    assert vals[:len(fields)] == offs
    assert vals[len(fields)] == ctypes.sizeof(DtConfig)
    assert vals[len(fields) + 1] == ctypes.sizeof(DtMap)
    assert vals[len(fields) + 2] == DtMap.headings.offset


def test_library_loads_and_reports_abi(libpath):
    from aido1_amd import _lib
    L = _lib.lib()
    assert L.dt_abi_version() == _lib.ABI_VERSION


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from aido1_amd import _lib
    from aido1_amd.vec_env import VecEnv
    with pytest.raises(_lib.DtError):
        VecEnv(8)


def test_render_io_layout_matches_header(tmp_path):
    from aido1_amd.render import LineParams, RenderIO
    src = tmp_path / 'rio.c'
    fields = [f[0] for f in RenderIO._fields_]
    body = '\n'.join('printf("%%zu ", offsetof(dt_render_io, %s));' % f for f in fields)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "dtsim.h"\nint main(){'
                   + body + 'printf("%zu %zu\\n", sizeof(dt_render_io), sizeof(dt_line_params));'
                   ' return 0;}')
    exe = tmp_path / 'rio'
    subprocess.run(['gcc', '-I', os.path.join(REPO, 'include'), '-o', str(exe), str(src)],
                   check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                           check=True).stdout.split()]
    assert vals[:len(fields)] == [getattr(RenderIO, f).offset for f in fields]
    assert vals[len(fields)] == ctypes.sizeof(RenderIO)
    assert vals[len(fields) + 1] == ctypes.sizeof(LineParams)


def test_upd_bn_layout_matches_header(tmp_path):
    """include/dtupd.h DtUpdBn against its ctypes mirror (_lib.DtUpdBn)."""
    from aido1_amd._lib import DtUpdBn
    fields = [f[0] for f in DtUpdBn._fields_]
    src = tmp_path / 'updbn.c'
    body = '\n'.join('printf("%%zu ", offsetof(DtUpdBn, %s));' % f for f in fields)
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "dtupd.h"\nint main(){'
                   + body + 'printf("%zu\\n", sizeof(DtUpdBn)); return 0;}')
    exe = tmp_path / 'updbn'
    subprocess.run(['gcc', '-I', os.path.join(REPO, 'include'), '-o', str(exe), str(src)],
                   check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                           check=True).stdout.split()]
    assert vals[:-1] == [getattr(DtUpdBn, f).offset for f in fields]
    assert vals[-1] == ctypes.sizeof(DtUpdBn)


def test_upd_entry_points_check_arguments(libpath):
    """dtupd.h's host-side argument checks (no GPU work is issued): other
    geometries, bad linear shapes and an empty hand-off are refused."""
    from aido1_amd import _lib
    L = _lib.lib()
    parts = ctypes.c_int32(0)
    assert L.dt_upd_part_floats() == 256 * 32 * 3
    assert L.dt_upd_conv_fwd_part(16, 4, 2, 1, 57, 77, 1, None, 1, 1, 0.01, 1, 1,
                                  ctypes.byref(parts), None) != 0
    empty = _lib.DtUpdBn()
    assert L.dt_upd_conv_fwd_part(32, 4, 2, 1, 57, 77, 1, ctypes.byref(empty), 1, 1, 0.01, 1, 1,
                                  ctypes.byref(parts), None) != 0
    assert L.dt_upd_bn_finish(126, 7, 16, ctypes.byref(empty), 16, None) != 0   # m % hw
    assert L.dt_upd_linear_work_floats(64, 250, 4032) == -1                    # n % 32
    assert L.dt_upd_linear_work_floats(64, 256, 4030) == -1                    # k % 32
    assert L.dt_upd_linear_work_floats(64, 256, 4032) % (64 * 256) == 0
    assert L.dt_upd_linear_fwd(64, 256, 4032, None, 16, 16, 0, 0.0, 16, 16, None) != 0
    assert L.dt_upd_wgrad_work_floats(3, 8, 2, 64, 120, 160) == 512 * 32 * 192


def test_diagnostic_check_library_is_current():
    """The bounds-checked build (libdtsim_check.so, made by
    __graft_entry__.build() for tests/test_gpu_actor.py) is no older than the
    sources: a stale one lacks the current entry points and fails on the GPU."""
    from aido1_amd import _lib
    if os.path.exists(_lib.CHECK_LIB_PATH):
        assert not _lib._stale(_lib.CHECK_LIB_PATH), 'rebuild: python -c "import __graft_entry__ as g; g.build()"'
