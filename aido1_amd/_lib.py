"""ctypes binding of libdtsim.so (include/dtsim.h) and its in-tree build.

The product path has exactly one implementation — the gfx950 kernels in
aido1_amd/csrc.  If the library is missing it is built in-tree with hipcc (the
same command as __graft_entry__.build()); if that fails, or no gfx950 device
is present when a handle is created, this module raises.  There is no CPU
fallback.
"""
import ctypes
import os
import subprocess
import threading

from aido1_amd.config import DtConfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, 'libdtsim.so')
CSRC = os.path.join(PKG_DIR, 'csrc')
SOURCES = ['dtsim.hip', 'dtrender.hip', 'dtreplay.hip', 'dtactor.hip', 'dtconv.hip',
           'dtconvx.hip', 'dttrain.hip', 'dtupd.hip', 'dthead.hip']
HEADERS = ['dtsim_common.h', 'dtrender.h', 'dtsync.h', 'dtconv_common.h']
PUBLIC_HEADERS = ['dtsim.h', 'dtreplay.h', 'dtactor.h', 'dttrain.h', 'dtupd.h', 'dthead.h']
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ABI_VERSION = 13

HIP_FLAGS = ['--offload-arch=gfx950', '-O3', '-fPIC', '-shared', '-std=c++17',
             '-ffp-contract=off', '-munsafe-fp-atomics']
# per-source extra flags.  dtrender.hip: no SLP vectorisation -- packed f32
# VALU (v_pk_*) measured slower in render_kernel: 0.1634 -> 0.1618 ms, nine
# paired runs; the other sources are neutral or slower with it.
FILE_FLAGS = {'dtrender.hip': ['-fno-slp-vectorize']}


class DtError(RuntimeError):
    pass


class DtMap(ctypes.Structure):
    _fields_ = [('width', ctypes.c_int32), ('height', ctypes.c_int32),
                ('kind', ctypes.c_void_p), ('curve_start', ctypes.c_void_p),
                ('curves', ctypes.c_void_p), ('headings', ctypes.c_void_p),
                ('n_objects', ctypes.c_int32), ('objects', ctypes.c_void_p),
                ('n_spawn_objects', ctypes.c_int32), ('spawn_objects', ctypes.c_void_p)]


class DtConvSet(ctypes.Structure):
    """include/dtactor.h dt_conv_set: the second weight set of a split launch."""
    _fields_ = [('n0', ctypes.c_int32), ('wfrag', ctypes.c_void_p), ('bias', ctypes.c_void_p),
                ('in_gamma', ctypes.c_void_p), ('in_beta', ctypes.c_void_p),
                ('out_gamma', ctypes.c_void_p), ('out_beta', ctypes.c_void_p)]


class DtUpdBn(ctypes.Structure):
    """include/dtupd.h DtUpdBn: a conv trunk block's BatchNorm hand-off."""
    _fields_ = [('part', ctypes.c_void_p), ('parts', ctypes.c_int32), ('m', ctypes.c_int64),
                ('bias', ctypes.c_void_p), ('gamma', ctypes.c_void_p), ('beta', ctypes.c_void_p),
                ('slope', ctypes.c_float), ('eps', ctypes.c_float), ('momentum', ctypes.c_float),
                ('running_mean', ctypes.c_void_p), ('running_var', ctypes.c_void_p),
                ('num_batches_tracked', ctypes.c_void_p), ('updates', ctypes.c_int32),
                ('mean_invstd', ctypes.c_void_p), ('guard', ctypes.c_void_p)]


class DtEpisodeState(ctypes.Structure):
    """include/dtactor.h DtEpisodeState: the episode accumulators and ring."""
    _fields_ = [('reward', ctypes.c_void_p), ('reward_modified', ctypes.c_void_p),
                ('tick', ctypes.c_void_p), ('episode', ctypes.c_void_p),
                ('decisions', ctypes.c_void_p), ('count', ctypes.c_void_p),
                ('ring', ctypes.c_void_p), ('capacity', ctypes.c_int64)]


class DtCopyEntry(ctypes.Structure):
    """Mirror of DtCopyEntry (include/dtactor.h)."""
    _fields_ = [('src', ctypes.c_void_p), ('dst', ctypes.c_void_p), ('map', ctypes.c_void_p),
                ('count', ctypes.c_int64), ('dst_dtype', ctypes.c_int32), ('pad', ctypes.c_int32)]


class DtMlp(ctypes.Structure):
    """include/dthead.h DtMlp: a small fully connected tail."""
    _fields_ = [(k, ctypes.c_int32) for k in ('m', 'k0', 'k1', 'n1', 'n2', 'act1', 'act2')] + \
        [('slope', ctypes.c_float)] + [(k, ctypes.c_void_p) for k in ('w1', 'b1', 'w2', 'b2')]


class DtExploreParams(ctypes.Structure):
    """include/dtactor.h DtExploreParams."""
    _fields_ = [(k, ctypes.c_double) for k in
                ('pi', 'eps_span', 'eps_final', 'eps_initial', 'ou_m', 'ou_c', 'ou_sigma_min',
                 'ou_sqrt_dt', 'ou_theta', 'ou_mu', 'ou_dt')] + \
        [('eps_ratio', ctypes.c_double), ('head', ctypes.c_int32)]


def _sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def _stale(path=None):
    """True when the library at `path` (the product library by default) is
    missing or older than any source or header it is built from."""
    path = path or LIB_PATH
    if not os.path.exists(path):
        return True
    t = os.path.getmtime(path)
    deps = _sources() + [os.path.join(CSRC, h) for h in HEADERS] + \
        [os.path.join(REPO_DIR, 'include', h) for h in PUBLIC_HEADERS]
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


# diagnostic build with conv1s_kernel's ring loads bounds-checked (DTCONV_CHECK,
# tests/test_gpu_actor.py); loaded only by that test, in a subprocess
CHECK_LIB_PATH = os.path.join(PKG_DIR, 'libdtsim_check.so')


def build(force=False, verbose=False, path=LIB_PATH, defines=()):
    """Compile libdtsim.so (or a diagnostic variant at `path` with -D defines)
    for gfx950 in-tree: each source to an object (its FILE_FLAGS added),
    in parallel, then one shared link."""
    if not force and path == LIB_PATH and not _stale():
        return LIB_PATH
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    tmp = path + '.tmp%d' % os.getpid()
    objdir = tempfile.mkdtemp(prefix='dtsim_build_')
    try:
        cflags = [f for f in HIP_FLAGS if f != '-shared'] + ['-D' + d for d in defines]
        jobs = []
        for src in _sources():
            obj = os.path.join(objdir, os.path.basename(src) + '.o')
            extra = FILE_FLAGS.get(os.path.basename(src), [])
            jobs.append(([HIPCC] + cflags + extra + ['-c', src, '-o', obj], obj))
        if verbose:
            for cmd, _ in jobs:
                print(' '.join(cmd))

        def run(cmd):
            return subprocess.run(cmd, capture_output=True, text=True)
        with ThreadPoolExecutor(max_workers=min(8, len(jobs))) as ex:
            results = list(ex.map(run, [c for c, _ in jobs]))
        for (cmd, _), r in zip(jobs, results):
            if r.returncode != 0:
                raise DtError('hipcc failed building %s (%s):\n' % (
                    os.path.basename(path), os.path.basename(cmd[-3])) + r.stderr[-4000:])
        link = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC', '-o', tmp] + \
            [o for _, o in jobs]
        if verbose:
            print(' '.join(link))
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise DtError('hipcc failed linking %s:\n' % os.path.basename(path) + r.stderr[-4000:])
        os.replace(tmp, path)
    finally:
        shutil.rmtree(objdir, ignore_errors=True)
    return path


_OPTIONAL = set()

_lib = None
_lock = threading.Lock()


def bind(L):
    """Declare the C-ABI signatures (include/*.h) on a loaded libdtsim (the
    product library, a diagnostic build, or the host-only sanitizer build of
    `make asan`); returns L."""
    vp, i32, u32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64
    i64, f64 = ctypes.c_int64, ctypes.c_double
    sig = {
        'dt_abi_version': (i32, []),
        'dt_create': (ctypes.c_int, [ctypes.POINTER(DtConfig), ctypes.POINTER(DtMap), u64, i32,
                                     i32, ctypes.POINTER(vp)]),
        'dt_destroy': (ctypes.c_int, [vp]),
        'dt_n_envs': (i32, [vp]),
        'dt_last_error': (ctypes.c_char_p, [vp]),
        'dt_seed': (ctypes.c_int, [vp, vp, u64, u32]),
        'dt_reset': (ctypes.c_int, [vp, vp, vp]),
        'dt_step': (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        'dt_step_masked': (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        'dt_step_many': (ctypes.c_int, [vp, i32, vp, vp, vp, vp, vp, vp, vp]),
        'dt_seed_env': (ctypes.c_int, [vp, i32, u64]),
        'dt_lane_pos': (ctypes.c_int, [vp, vp, vp, vp]),
        'dt_render': (ctypes.c_int, [vp, vp, vp]),
        'dt_render2': (ctypes.c_int, [vp, vp, vp, vp]),
        'dt_render3': (ctypes.c_int, [vp, vp, vp, vp, vp]),
        'dt_copy_pose': (ctypes.c_int, [vp, vp, vp]),
        'dt_render_order': (ctypes.c_int, [vp, ctypes.POINTER(u32), vp, vp]),
        'dt_palette_gray': (ctypes.c_int, [ctypes.POINTER(ctypes.c_float)]),
        'dt_default_line_params': (ctypes.c_int, [vp]),
        'dt_set_line_params': (ctypes.c_int, [vp, vp]),
        'dt_line_detect': (ctypes.c_int, [vp, vp, i32, i32, i32, vp, vp, vp]),
        'dt_hough_lines': (ctypes.c_int, [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                                          vp]),
        'dt_line_detect_workspace': (ctypes.c_size_t, [i32, i32, i32]),
        'dt_line_detect_ws': (ctypes.c_int, [vp, vp, i32, i32, i32, vp, vp, vp,
                                             ctypes.c_size_t, vp]),
        'dt_hough_workspace': (ctypes.c_size_t, [i32, i32, i32]),
        'dt_hough_lines_ws': (ctypes.c_int, [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp,
                                             vp, ctypes.c_size_t, vp]),
        'dt_get_state': (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp]),
        'dt_set_state': (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp]),
        'dt_check': (ctypes.c_int, [vp, ctypes.POINTER(u32)]),
        'dt_stats': (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_uint64), i32]),
        # dtreplay.h
        'dt_per_create': (ctypes.c_int, [i64, f64, i32, ctypes.POINTER(vp)]),
        'dt_per_destroy': (None, [vp]),
        'dt_per_last_error': (ctypes.c_char_p, [vp]),
        'dt_per_capacity': (i64, [vp]),
        'dt_per_len': (i64, [vp]),
        'dt_per_next_idx': (i64, [vp]),
        'dt_per_add': (ctypes.c_int, [vp, i64, vp, vp]),
        'dt_per_sample': (ctypes.c_int, [vp, i32, vp, f64, vp, vp, vp]),
        'dt_per_update': (ctypes.c_int, [vp, i32, vp, vp, vp]),
        'dt_per_update_td': (ctypes.c_int, [vp, i32, vp, vp, f64, vp]),
        'dt_per_read': (ctypes.c_int, [vp, vp, vp, vp, vp]),
        'dt_per_check': (ctypes.c_int, [vp]),
        'dt_frame_add': (ctypes.c_int, [i32, i64, vp, i64, vp, i32, vp, vp, i32, vp, vp, vp]),
        'dt_frame_gather': (ctypes.c_int, [i32, vp, vp, i32, i64, i32, vp, vp, vp, vp, vp,
                                           vp, vp, vp, vp, vp, vp]),
        # dttrain.h
        'dt_train_work_floats': (i64, [i64]),
        'dt_bn_leaky_fwd': (ctypes.c_int, [i64, vp, vp, ctypes.c_float, vp, vp, ctypes.c_float,
                                           ctypes.c_float, vp, vp, vp, i32, vp, vp, vp, vp,
                                           vp, vp]),
        'dt_bn_leaky_bwd': (ctypes.c_int, [i64, vp, vp, vp, vp, vp, ctypes.c_float, vp, vp, vp,
                                           vp, vp, vp, vp]),
        'dt_adam': (ctypes.c_int, [i32, vp, vp, vp, vp, f64, f64, f64, vp, vp, i32, i32, vp]),
        'dt_guard_scan': (ctypes.c_int, [i32, vp, vp, vp]),
        # dtupd.h
        'dt_upd_conv_fwd': (ctypes.c_int, [i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
        'dt_upd_conv_fwd_bn': (ctypes.c_int, [i32, i32, i32, i32, i32, i32, vp, vp, vp,
                                              ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                              vp, vp, vp, i32, vp, vp, vp, vp, vp]),
        'dt_bn_leaky_apply': (ctypes.c_int, [i64, vp, vp, ctypes.c_float, vp, vp, vp, vp,
                                             vp]),
        'dt_upd_wgrad_work_floats': (i64, [i32, i32, i32, i32, i32, i32]),
        'dt_upd_bn_work_floats': (i64, []),
        'dt_upd_conv_wgrad': (ctypes.c_int, [i32, i32, i32, i32, i32, i32, vp, vp, vp, vp,
                                             vp]),
        'dt_upd_conv_dgrad': (ctypes.c_int, [i32, i32, i32, i32, i32, i32, vp, vp, vp, vp]),
        'dt_upd_part_floats': (i64, []),
        'dt_upd_conv_fwd_part': (ctypes.c_int, [i32, i32, i32, i32, i32, i32, vp,
                                                ctypes.POINTER(DtUpdBn), vp, vp,
                                                ctypes.c_float, vp, vp,
                                                ctypes.POINTER(i32), vp]),
        'dt_upd_bn_finish': (ctypes.c_int, [i64, i32, vp, ctypes.POINTER(DtUpdBn), vp, vp]),
        'dt_upd_conv_wgrad_bn': (ctypes.c_int, [i32, i32, i32, i32, i32, i32, vp,
                                                ctypes.POINTER(DtUpdBn), vp, vp, vp, vp]),
        'dt_upd_linear_work_floats': (i64, [i32, i32, i32]),
        'dt_upd_linear_fwd': (ctypes.c_int, [i32, i32, i32, vp, vp, vp, i32, ctypes.c_float,
                                             vp, vp, vp]),
        'dt_upd_linear_dgrad': (ctypes.c_int, [i32, i32, i32, vp, vp, vp, ctypes.c_float, vp,
                                               vp]),
        'dt_upd_linear_wgrad': (ctypes.c_int, [i32, i32, i32, vp, vp, vp, ctypes.c_float, vp,
                                               vp, vp]),
        'dt_upd_linear_fwd_drop': (ctypes.c_int, [i32, i32, i32, vp, vp, ctypes.c_float, vp, vp,
                                                  vp, i32, ctypes.c_float, vp, vp, vp]),
        'dt_upd_linear_dgrad_drop': (ctypes.c_int, [i32, i32, i32, vp, vp, vp, ctypes.c_float,
                                                    vp, ctypes.c_float, vp, vp]),
        'dt_soft_update': (ctypes.c_int, [i32, vp, vp, f64, vp]),
        # dthead.h
        'dt_mlp_fwd': (ctypes.c_int, [ctypes.POINTER(DtMlp), vp, vp, vp, vp, vp]),
        'dt_mlp_bwd': (ctypes.c_int, [ctypes.POINTER(DtMlp), vp, vp, vp, vp, vp, vp, vp, vp,
                                      vp, vp, vp, vp]),
        'dt_mlp_fwd_td': (ctypes.c_int, [ctypes.POINTER(DtMlp), vp, vp, vp, vp, vp, vp,
                                         ctypes.c_float, vp, vp]),
        'dt_loss': (ctypes.c_int, [i32, i32, vp, vp, vp, vp]),
        'dt_loss_bwd': (ctypes.c_int, [i32, i32, vp, vp, vp, vp, vp]),
        # dtactor.h
        'dt_sample_norm': (ctypes.c_int, [vp, vp, i32, i32, i32, vp, vp, ctypes.c_float,
                                          ctypes.c_float, i32, vp]),
        'dt_conv1': (ctypes.c_int, [vp, i32, i32, ctypes.POINTER(i32), vp, vp, vp, vp,
                                    ctypes.c_float, vp]),
        'dt_conv1_split': (ctypes.c_int, [vp, i32, i32, ctypes.POINTER(i32), vp, vp,
                                          ctypes.POINTER(DtConvSet), vp, vp, ctypes.c_float,
                                          vp]),
        'dt_conv1_index_split': (ctypes.c_int, [vp, i32, i32, ctypes.POINTER(i32), vp, vp,
                                                ctypes.POINTER(DtConvSet), vp, vp,
                                                ctypes.c_float, vp]),
        'dt_conv1_norm': (ctypes.c_int, [vp, i32, vp, vp, vp, ctypes.c_float, vp]),
        'dt_conv32': (ctypes.c_int, [i32, i32, vp, vp, vp, vp, vp, vp, ctypes.c_float, vp,
                                     vp, vp, vp, ctypes.c_float, ctypes.c_float, vp]),
        'dt_conv32_split': (ctypes.c_int, [i32, i32, vp, vp, vp, vp, vp, vp, ctypes.c_float,
                                           vp, vp, vp, vp, ctypes.c_float, ctypes.c_float,
                                           ctypes.POINTER(DtConvSet), vp]),
        'dt_conv1x_split': (ctypes.c_int, [vp, i32, i32, i32, ctypes.POINTER(i32), vp, vp,
                                           ctypes.POINTER(DtConvSet), vp, vp,
                                           ctypes.c_float, vp]),
        'dt_conv32x_split': (ctypes.c_int, [i32, i32, vp, vp, vp, vp, vp, vp, ctypes.c_float,
                                            vp, vp, vp, vp, ctypes.c_float, ctypes.c_float,
                                            ctypes.POINTER(DtConvSet), vp]),
        'dt_actor_head_x3': (ctypes.c_int, [i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                            i32, ctypes.c_float, vp, vp, vp]),
        'dt_actor_head_x3_work_floats': (i64, [i32]),
        'dt_actor_head_x3_drop': (ctypes.c_int, [i32, i32, i32, vp, ctypes.c_float, ctypes.c_uint32,
                                                 vp, vp, vp, vp, vp, vp, vp, vp, i32,
                                                 ctypes.c_float, vp, vp, vp]),
        'dt_actor_head_f16_drop': (ctypes.c_int, [i32, i32, i32, vp, ctypes.c_float,
                                                  ctypes.c_uint32, vp, vp, vp, vp, vp, vp, vp, vp,
                                                  i32, ctypes.c_float, vp, vp, vp]),
        'dt_explore': (ctypes.c_int, [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                      ctypes.POINTER(DtExploreParams), vp, vp]),
        'dt_explore_done': (ctypes.c_int, [i32, vp, vp, vp, vp, i32, vp]),
        'dt_episode_account': (ctypes.c_int, [i32, i32, vp, vp, vp,
                                              ctypes.POINTER(DtEpisodeState), vp]),
        'dt_refresh_copy': (ctypes.c_int, [i32, vp, i64, vp]),
        'dt_actor_head': (ctypes.c_int, [i32, i32, i32, vp, i32, vp, vp, vp, vp, i32,
                                         ctypes.c_float, vp, vp]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name):
            if name in _OPTIONAL:
                continue
            raise DtError('libdtsim.so lacks %s (stale build?)' % name)
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def lib():
    """Load (building first if needed) libdtsim.so; raises DtError if impossible."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        # torch (if importable) must own the HIP runtime first: both it and this
        # library NEED libamdhip64.so.7, and loading torch first makes the
        # dynamic linker bind ours to torch's copy (one runtime per process).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = os.environ.get('DTSIM_DIAG_LIB')  # diagnostic builds (tools/), loaded as is
        if not path:
            path = LIB_PATH
            if _stale():
                build()
        L = bind(ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL))
        v = L.dt_abi_version()
        if v != ABI_VERSION:
            raise DtError('libdtsim ABI %d != expected %d (rebuild)' % (v, ABI_VERSION))
        _lib = L
        return L


def exported_symbols():
    """Names declared in include/*.h (checked against the .so by tests)."""
    import re
    names = set()
    for h in PUBLIC_HEADERS:
        with open(os.path.join(REPO_DIR, 'include', h)) as f:
            src = f.read()
        names |= set(re.findall(r'^\s*(?:int|int32_t|int64_t|size_t|void|const char\*)\s+(dt_\w+)\s*\(',
                                src, re.M))
    return sorted(names)


def check(L, handle, rc, what):
    if rc != 0:
        msg = L.dt_last_error(handle)
        raise DtError('%s failed (%d): %s' % (what, rc, msg.decode() if msg else ''))
