"""Time dt_mlp_fwd / dt_mlp_bwd (include/dthead.h) on config.json's two tails
against the torch ops they replace.  usage: python tools/mlp_bench.py"""
import ctypes
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from aido1_amd import _lib  # noqa: E402

REPS = 200


def timed(fn):
    for _ in range(10):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / REPS


def main():
    dev = torch.device('cuda', 0)
    L = _lib.lib()
    st = torch.cuda.current_stream(dev).cuda_stream
    for m, k0, k1, n1, n2, a1, a2 in [(64, 256, 2, 128, 1, 1, 0), (64, 512, 0, 2, 0, 2, 0)]:
        g = torch.Generator(device=dev).manual_seed(0)
        r = (lambda *s: torch.randn(*s, device=dev, generator=g))
        x0, x1 = r(m, k0), (r(m, k1) if k1 else None)
        w1, b1 = r(n1, k0 + k1) * 0.05, r(n1)
        w2, b2 = (r(n2, n1) * 0.05, r(n2)) if n2 else (None, None)
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        p = _lib.DtMlp(m, k0, k1, n1, n2, a1, a2, 0.01, w1.data_ptr(), b1.data_ptr(), ptr(w2),
                       ptr(b2))
        h = torch.empty(m, n1, device=dev)
        y = torch.empty(m, n2, device=dev) if n2 else None
        dy = r(m, n2 or n1)
        outs = [torch.empty_like(t) if t is not None else None for t in (x0, x1, w1, b1, w2, b2)]

        def fwd():
            rc = L.dt_mlp_fwd(ctypes.byref(p), x0.data_ptr(), ptr(x1), h.data_ptr(), ptr(y), st)
            assert rc == 0, rc

        def bwd():
            rc = L.dt_mlp_bwd(ctypes.byref(p), x0.data_ptr(), ptr(x1), h.data_ptr(), ptr(y),
                              dy.data_ptr(), *[ptr(t) for t in outs], st)
            assert rc == 0, rc

        x = torch.cat([x0, x1], 1) if k1 else x0

        def tfwd():
            t = F.linear(x, w1, b1)
            t = F.leaky_relu(t, 0.01) if a1 == 1 else torch.tanh(t)
            if n2:
                F.linear(t, w2, b2)

        print('m %d k %d+%d n1 %d n2 %d: dt_mlp_fwd %.1f us, dt_mlp_bwd %.1f us, torch fwd %.1f us'
              % (m, k0, k1, n1, n2, timed(fwd), timed(bwd), timed(tfwd)), flush=True)


if __name__ == '__main__':
    main()
