"""Diagnostic: dt_conv1 at 4096 samples (reference mode: statistics on), timed
for builds of dtconv.hip that skip one phase of the streaming conv1s_kernel
each (DTCONV_SKIP bits, see the source).  `--build` compiles the variants
(here, no GPU needed) into build/conv1_variants/; run without it on the GPU
box.  Extra -D flags for every variant: --defines."""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'diag_so', 'conv1_variants' + os.environ.get('CONV1_TAG', ''))  # travels with gpurun (build/ does not)
SKIPS = {'full': 0, 'no_prefetch': 1, 'no_mma': 2, 'no_store': 4, 'no_stats': 8,
         'no_commit': 16, 'only_mma': 1 | 4 | 8 | 16, 'only_io': 2 | 8 | 16, 'none': 31,
         'no_ldsread': 32}
ONLY = [v for v in os.environ.get('CONV1_ONLY', '').split(',') if v]   # subset of SKIPS


def build(defines):
    sys.path.insert(0, ROOT)
    from aido1_amd import _lib
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, 'aido1_amd', 'csrc', 'dtconv.hip')
    for name, bits in SKIPS.items():
        if ONLY and name not in ONLY:
            continue
        so = os.path.join(OUT, 'libconv1_%s.so' % name)
        subprocess.check_call([_lib.HIPCC] + _lib.HIP_FLAGS + ['-DDTCONV_SKIP=%d' % bits] +
                              ['-D' + d for d in defines] + ['-o', so, src])
        print('built', so)


def run(n, reps):
    import torch
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    ring = torch.rand(n, 3, 120, 160, device=dev)
    wf = (torch.randn(16 * 64 * 8, device=dev) * 0.05).half()
    b = torch.zeros(32, device=dev)
    y = torch.empty(n, 57, 77, 32, dtype=torch.float16, device=dev)
    part = torch.empty(n, 8, 32, 3, device=dev)
    o = (ctypes.c_int32 * 3)(0, 1, 2)
    s = torch.cuda.current_stream().cuda_stream
    if os.environ.get('CONV1_DATA') == 'zero':     # same work, quiet operands
        ring.zero_()
        wf.zero_()
    elif os.environ.get('CONV1_DATA') == 'frames':  # piecewise-constant, like rendered frames
        ring.copy_((ring * 4).floor() / 4)
    byts = n * (3 * 120 * 160 * 4 + 57 * 77 * 32 * 2)
    print('%-12s %9s %9s' % ('variant', 'conv1 us', 'TB/s'))
    for name in SKIPS:
        if ONLY and name not in ONLY:
            continue
        L = ctypes.CDLL(os.path.join(OUT, 'libconv1_%s.so' % name))
        L.dt_conv1.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                               ctypes.POINTER(ctypes.c_int32)] + [ctypes.c_void_p] * 4 + \
            [ctypes.c_float, ctypes.c_void_p]

        def call():
            rc = L.dt_conv1(ring.data_ptr(), n, 3, o, wf.data_ptr(), b.data_ptr(), y.data_ptr(),
                            part.data_ptr(), 0.01, s)
            assert rc == 0, rc
        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print('%-12s %9.1f %9.2f' % (name, us, byts / us / 1e6))


if __name__ == '__main__':
    p = argparse.ArgumentParser()
    p.add_argument('--build', action='store_true')
    p.add_argument('--defines', nargs='*', default=[])
    p.add_argument('--n', type=int, default=4096)
    p.add_argument('--reps', type=int, default=20)
    a = p.parse_args()
    build(a.defines) if a.build else run(a.n, a.reps)
