"""Diagnostic: shader-clock stamps inside conv2's steps (a DTCONV_STAMPS build,
DTSIM_DIAG_LIB): dt_conv32 layer 2 at 4096 samples (reference mode), then the
mean cycles between the stamp points of steps 8-47 of 8 workgroups x 2 waves.
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
x = (torch.rand(n, 57, 77, 32, device=dev) * 2).half()
w = (torch.randn(32 * 64 * 8, device=dev) * 0.05).half()
b = torch.zeros(32, device=dev)
pp = torch.rand(n, 32, 3, device=dev) + 0.5
g = torch.ones(32, device=dev)
bt = torch.zeros(32, device=dev)
y = torch.empty(n, 27 * 37 * 32, dtype=torch.float16, device=dev)
part = torch.empty(n, 32, 3, device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    assert L.dt_conv32(2, n, x.data_ptr(), w.data_ptr(), b.data_ptr(), pp.data_ptr(), g.data_ptr(),
                       bt.data_ptr(), 1e-5, y.data_ptr(), part.data_ptr(), None, None, 1e-5, 0.01,
                       s) == 0
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (8 * 2 * 48 * 8))()
assert L.dt_diag_convstamps(buf) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(8, 2, 48, 8).astype(np.int64)[:, :, 8:48, :6]
d = np.diff(a, axis=3)
step = a[:, :, 1:, 0] - a[:, :, :-1, 0]
names = ['issue+ld+mfma issue', 'mfma drain+lrelu', 'store+stats', 'commit', 'barrier']
for i, nm in enumerate(names):
    print('%-22s mean %7.0f  median %7.0f  cycles' % (nm, d[..., i].mean(), np.median(d[..., i])))
print('%-22s mean %7.0f  median %7.0f' % ('step (entry to entry)', step.mean(), np.median(step)))
