"""Diagnostic: the update's convolutions (dtupd.hip) per layer at batch 64,
forward with fused statistics, weight and input gradients, timed for builds
that skip one part of the forward each (DTUPD_SKIP bits, see the source).
`--build` compiles the variants (here, no GPU needed) into
tools/variants/ (shipped to the box); run without it on the GPU box."""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'tools', 'variants')
SKIPS = {'full': 0, 'no_a_loads': 1, 'no_w_stage': 2, 'no_merge': 4, 'no_ksum': 8, 'bare': 15,
         'no_part_loads': 16, 'no_chain_merge': 32, 'no_chain_both': 48}
# other variants: extra -D flags (the f32 MFMA forward, forward K slices)
EXTRA = {'f32': ['-DDTUPD_X3=0'], 'wg_nodb': ['-DDTUPD_WG_DB=0'], 'wg_db1': ['-DDTUPD_WG_DB1=1'], 'f32_bare': ['-DDTUPD_X3=0', '-DDTUPD_SKIP=15'],
         'ks_4_4_4_8': ['-DDTUPD_KS1=4', '-DDTUPD_KS2=4', '-DDTUPD_KS3=4', '-DDTUPD_KS4=8'],
         'ks_1_1_2_4': ['-DDTUPD_KS1=1', '-DDTUPD_KS2=1', '-DDTUPD_KS3=2', '-DDTUPD_KS4=4'],
         'all12': ['-DDTUPD_ALL_LOADS=12'],
         'all16_ks2_4': ['-DDTUPD_ALL_LOADS=16', '-DDTUPD_KS2=4'],
         'all32': ['-DDTUPD_ALL_LOADS=32']}
LAYERS = {1: (3, 8, 2, 120, 160), 2: (32, 4, 2, 57, 77), 3: (32, 4, 2, 27, 37),
          4: (32, 4, 1, 12, 17)}


def build(variants=''):
    sys.path.insert(0, ROOT)
    from aido1_amd import _lib
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, 'aido1_amd', 'csrc', 'dtupd.hip')
    want = set(variants.split(',')) if variants else None
    for name, bits in SKIPS.items():
        if want is not None and name not in want:
            continue
        so = os.path.join(OUT, 'libupd_%s.so' % name)
        subprocess.check_call([_lib.HIPCC] + _lib.HIP_FLAGS + ['-DDTUPD_SKIP=%d' % bits,
                                                                '-o', so, src])
        print('built', so)
    for name, flags in EXTRA.items():
        if want is not None and name not in want:
            continue
        so = os.path.join(OUT, 'libupd_%s.so' % name)
        subprocess.check_call([_lib.HIPCC] + _lib.HIP_FLAGS + flags + ['-o', so, src])
        print('built', so)


class Bn(ctypes.Structure):       # include/dtupd.h DtUpdBn
    _fields_ = [('part', ctypes.c_void_p), ('parts', ctypes.c_int32), ('m', ctypes.c_int64),
                ('bias', ctypes.c_void_p), ('gamma', ctypes.c_void_p), ('beta', ctypes.c_void_p),
                ('slope', ctypes.c_float), ('eps', ctypes.c_float), ('momentum', ctypes.c_float),
                ('running_mean', ctypes.c_void_p), ('running_var', ctypes.c_void_p),
                ('num_batches_tracked', ctypes.c_void_p), ('updates', ctypes.c_int32),
                ('mean_invstd', ctypes.c_void_p), ('guard', ctypes.c_void_p)]


def load(name):
    L = ctypes.CDLL(os.path.join(OUT, 'libupd_%s.so' % name))
    vp, i32, f = ctypes.c_void_p, ctypes.c_int32, ctypes.c_float
    L.dt_upd_conv_fwd.argtypes = [i32] * 6 + [vp] * 4
    L.dt_upd_conv_fwd_bn.argtypes = [i32] * 6 + [vp] * 3 + [f] * 3 + [vp] * 3 + [i32] + [vp] * 5
    L.dt_upd_bn_work_floats.restype = ctypes.c_int64
    L.dt_upd_wgrad_work_floats.restype = ctypes.c_int64
    L.dt_upd_wgrad_work_floats.argtypes = [i32] * 6
    L.dt_upd_conv_wgrad.argtypes = [i32] * 6 + [vp] * 5
    L.dt_upd_conv_dgrad.argtypes = [i32] * 6 + [vp] * 4
    L.dt_upd_part_floats.restype = ctypes.c_int64
    L.dt_upd_conv_fwd_part.argtypes = [i32] * 6 + [vp, ctypes.POINTER(Bn), vp, vp, f, vp, vp,
                                                   ctypes.POINTER(i32), vp]
    L.dt_upd_bn_finish.argtypes = [ctypes.c_int64, i32, vp, ctypes.POINTER(Bn), vp, vp]
    return L


def timeit(torch, fn, reps):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def run(n, reps, variants=''):
    import torch
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    s = torch.cuda.current_stream().cuda_stream
    names = variants.split(',') if variants else list(SKIPS) + list(EXTRA)
    for name in names:
        L = load(name)
        row = []
        for layer, (cin, ks, st, ih, iw) in LAYERS.items():
            oh, ow = (ih - ks) // st + 1, (iw - ks) // st + 1
            x = torch.rand(n, ih, iw, cin, device=dev)
            w = torch.randn(32, ks * ks * cin, device=dev) * 0.05
            z = torch.empty(n, oh, ow, 32, device=dev)
            b = torch.zeros(32, device=dev)
            rm, rv = torch.zeros(32, device=dev), torch.ones(32, device=dev)
            mi = torch.empty(64, device=dev)
            work = torch.zeros(int(L.dt_upd_bn_work_floats()), device=dev)
            a = (cin, ks, st, n, ih, iw)

            def fwd_bn():
                rc = L.dt_upd_conv_fwd_bn(*a, x.data_ptr(), w.data_ptr(), b.data_ptr(), 0.01, 1e-5,
                                          0.1, rm.data_ptr(), rv.data_ptr(), None, 1, z.data_ptr(),
                                          mi.data_ptr(), work.data_ptr(), None, s)
                assert rc == 0, rc

            def fwd():
                assert L.dt_upd_conv_fwd(*a, x.data_ptr(), w.data_ptr(), z.data_ptr(), s) == 0
            t = {'fwd_bn': timeit(torch, fwd_bn, reps), 'fwd': timeit(torch, fwd, reps)}
            if name in ('full', 'no_a_loads', 'no_w_stage', 'no_part_loads', 'no_chain_merge',
                        'no_chain_both'):
                # the chain: partials only, and normalise-on-load from a hand-off
                part = torch.zeros(int(L.dt_upd_part_floats()), device=dev)
                pin = torch.zeros(int(L.dt_upd_part_floats()), device=dev).view(-1, 32, 3)
                pin[:, :, 0] = 10.0
                pin[:, :, 2] = 5.0
                parts = ctypes.c_int32(0)
                hand = Bn(pin.data_ptr(), 256, 2560, b.data_ptr(), rv.data_ptr(), rm.data_ptr(),
                          0.01, 1e-5, 0.1, rm.data_ptr(), rv.data_ptr(), None, 1, mi.data_ptr(),
                          None)

                def part_only():
                    assert L.dt_upd_conv_fwd_part(*a, x.data_ptr(), None, w.data_ptr(),
                                                  b.data_ptr(), 0.01, z.data_ptr(),
                                                  part.data_ptr(), ctypes.byref(parts), s) == 0
                t['part'] = timeit(torch, part_only, reps)
                if cin == 32:
                    def part_norm():
                        assert L.dt_upd_conv_fwd_part(*a, x.data_ptr(), ctypes.byref(hand),
                                                      w.data_ptr(), b.data_ptr(), 0.01,
                                                      z.data_ptr(), part.data_ptr(),
                                                      ctypes.byref(parts), s) == 0
                    t['part_norm'] = timeit(torch, part_norm, reps)
                    y = torch.empty_like(z)

                    def finish():
                        assert L.dt_upd_bn_finish(z.numel() // 32, 0, z.data_ptr(),
                                                  ctypes.byref(hand), y.data_ptr(), s) == 0
                    t['finish'] = timeit(torch, finish, reps)
            if name in ('full', 'f32', 'wg_nodb', 'wg_db1'):
                ww = torch.empty(int(L.dt_upd_wgrad_work_floats(*a)), device=dev)
                dw = torch.empty_like(w)

                def wgrad():
                    assert L.dt_upd_conv_wgrad(*a, x.data_ptr(), z.data_ptr(), dw.data_ptr(),
                                               ww.data_ptr(), s) == 0
                t['wgrad+reduce'] = timeit(torch, wgrad, reps)
                if cin == 32:
                    dx = torch.empty_like(x)

                    def dgrad():
                        assert L.dt_upd_conv_dgrad(*a, z.data_ptr(), w.data_ptr(), dx.data_ptr(),
                                                   s) == 0
                    t['dgrad'] = timeit(torch, dgrad, reps)
            row.append('L%d ' % layer + ' '.join('%s %.1f' % kv for kv in t.items()))
        print('%-11s | %s' % (name, ' | '.join(row)), flush=True)


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--build', action='store_true')
    ap.add_argument('--n', type=int, default=64)
    ap.add_argument('--reps', type=int, default=200)
    ap.add_argument('--variants', default='', help='comma-separated names (default: all)')
    args = ap.parse_args()
    if args.build:
        build(args.variants)
    else:
        run(args.n, args.reps, args.variants)
