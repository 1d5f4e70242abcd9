"""Diagnostic: dt_conv32 per layer at 4096 samples (reference mode: input norm
+ statistics), timed for builds of dtconv.hip that skip one phase each
(DTCONV_SKIP bits, see the source).  `--build` compiles the variants (here,
no GPU needed) into build/conv_variants/; run without it on the GPU box."""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'build', 'conv_variants')
SKIPS = {'full': 0, 'no_prefetch': 1, 'no_mma': 2, 'no_store': 4, 'no_stats': 8,
         'no_commit': 16, 'only_mma': 1 | 4 | 8 | 16, 'none': 31}


def build():
    sys.path.insert(0, ROOT)
    from aido1_amd import _lib
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(ROOT, 'aido1_amd', 'csrc', 'dtconv.hip')
    for name, bits in SKIPS.items():
        so = os.path.join(OUT, 'libconv_%s.so' % name)
        subprocess.check_call([_lib.HIPCC] + _lib.HIP_FLAGS + ['-DDTCONV_SKIP=%d' % bits,
                                                                '-o', so, src])
        print('built', so)


def run(n, reps):
    import torch
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    shapes = {2: (57, 77, 27, 37), 3: (27, 37, 12, 17), 4: (12, 17, 9, 14)}
    res = {}
    for name in SKIPS:
        L = ctypes.CDLL(os.path.join(OUT, 'libconv_%s.so' % name))
        L.dt_conv32.argtypes = [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 6 + \
            [ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
             ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        for layer, (ih, iw, oh, ow) in shapes.items():
            x = (torch.rand(n, ih, iw, 32, device=dev) * 2).half()
            w = (torch.randn(32 * 64 * 8, device=dev) * 0.05).half()
            b = torch.zeros(32, device=dev)
            pp = torch.rand(n, 32, 3, device=dev) + 0.5
            g = torch.ones(32, device=dev)
            bt = torch.zeros(32, device=dev)
            y = torch.empty(n, oh * ow * 32, dtype=torch.float16, device=dev)
            part = torch.empty(n, 32, 3, device=dev)
            s = torch.cuda.current_stream().cuda_stream
            last = layer == 4

            def call():
                rc = L.dt_conv32(layer, n, x.data_ptr(), w.data_ptr(), b.data_ptr(), pp.data_ptr(),
                                 g.data_ptr(), bt.data_ptr(), 1e-5, y.data_ptr(),
                                 None if last else part.data_ptr(),
                                 g.data_ptr() if last else None, bt.data_ptr() if last else None,
                                 1e-5, 0.01, s)
                assert rc == 0, rc
            for _ in range(3):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            res[(name, layer)] = e0.elapsed_time(e1) / reps * 1e3
    print('%-12s %9s %9s %9s' % ('variant', 'conv2 us', 'conv3 us', 'conv4 us'))
    for name in SKIPS:
        print('%-12s %9.1f %9.1f %9.1f' % (name, res[(name, 2)], res[(name, 3)], res[(name, 4)]))


if __name__ == '__main__':
    p = argparse.ArgumentParser()
    p.add_argument('--build', action='store_true')
    p.add_argument('--n', type=int, default=4096)
    p.add_argument('--reps', type=int, default=20)
    a = p.parse_args()
    build() if a.build else run(a.n, a.reps)
