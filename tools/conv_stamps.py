"""Diagnostic: shader-clock stamps inside a conv32 layer's steps (a
DTCONV_STAMPS=<input height> build, DTSIM_DIAG_LIB; 57 conv2, 27 conv3, 12
conv4; a DTCONV1_STAMPS build for layer 1): dt_conv32 (dt_conv1_index for
layer 1) of that layer (argv[1], default 2) at 4096 samples (reference mode),
then the mean cycles between the stamp points of steps 8-47 of 8 workgroups x
2 waves.
Points: 0 step entry, 1 MFMAs issued, 2 LeakyReLU done (acc ready), 3 stores +
statistics done, 4 commit done, 5 after the barrier."""
import ctypes
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
L = ctypes.CDLL(os.environ['DTSIM_DIAG_LIB'])
L.dt_conv32.argtypes = [ctypes.c_int32, ctypes.c_int32] + [ctypes.c_void_p] * 6 + \
    [ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
     ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
dev = torch.device('cuda', 0)
n = 4096
layer = int(sys.argv[1]) if len(sys.argv) > 1 else 2
if layer == 1:   # conv1 on a palette-index ring (3 slots), the actor's form
    L.dt_conv1_index_split.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32] + \
        [ctypes.c_void_p] * 6 + [ctypes.c_float, ctypes.c_void_p]
    ring = torch.randint(0, 5, (n, 3, 120, 160), dtype=torch.uint8, device=dev)
    order = (ctypes.c_int32 * 3)(0, 1, 2)
    w1 = (torch.randn(16 * 64 * 8, device=dev) * 0.05).half()
    b1 = torch.zeros(32, device=dev)
    y1 = torch.empty(n, 57 * 77 * 32, dtype=torch.float16, device=dev)
    part1 = torch.empty(n, 32, 3, device=dev)
    s1 = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        assert L.dt_conv1_index_split(ring.data_ptr(), n, 3, order, w1.data_ptr(), b1.data_ptr(),
                                      None, y1.data_ptr(), part1.data_ptr(), 0.01, s1) == 0
ih, iw, oh, ow = {1: (57, 77, 27, 37), 2: (57, 77, 27, 37), 3: (27, 37, 12, 17),
                  4: (12, 17, 9, 14)}[layer]
last = layer == 4
x = (torch.rand(n, ih, iw, 32, device=dev) * 2).half()
w = (torch.randn(32 * 64 * 8, device=dev) * 0.05).half()
b = torch.zeros(32, device=dev)
pp = torch.rand(n, 32, 3, device=dev) + 0.5
g = torch.ones(32, device=dev)
bt = torch.zeros(32, device=dev)
y = torch.empty(n, oh * ow * 32, dtype=torch.float16, device=dev)
part = torch.empty(n, 32, 3, device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(5 if layer > 1 else 0):
    assert L.dt_conv32(layer, n, x.data_ptr(), w.data_ptr(), b.data_ptr(), pp.data_ptr(),
                       g.data_ptr(), bt.data_ptr(), 1e-5, y.data_ptr(),
                       None if last else part.data_ptr(), g.data_ptr() if last else None,
                       bt.data_ptr() if last else None, 1e-5, 0.01, s) == 0
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (8 * 2 * 48 * 8))()
assert L.dt_diag_convstamps(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(8, 2, 48, 8).astype(np.int64)[:, :, :, :6]
lo = 8 if layer != 4 else 1        # conv4: one step a sample, ~8 a workgroup
names = ['issue+ld+mfma issue', 'mfma drain+lrelu', 'store+stats', 'commit', 'barrier']
d = [[] for _ in names]
step = []
for w in range(8):
    for v in range(2):
        for t in range(lo, 48):
            r = a[w, v, t]
            if (r == 0).any():
                break
            for i in range(5):
                d[i].append(r[i + 1] - r[i])
            if t + 1 < 48 and (a[w, v, t + 1] != 0).all():
                step.append(a[w, v, t + 1, 0] - r[0])
for i, nm in enumerate(names):
    print('%-22s mean %7.0f  median %7.0f  cycles (%d steps)' % (nm, np.mean(d[i]), np.median(d[i]),
                                                                len(d[i])))
print('%-22s mean %7.0f  median %7.0f' % ('step (entry to entry)', np.mean(step), np.median(step)))
