"""Diagnostic: dt_conv12 index mapping with delta weights (conv1 copies input
channel 0 at kernel offset (ky1, kx1), conv2 copies conv1 channel 0 at (ky2, kx2))."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd import _lib  # noqa: E402
from aido1_amd.actor import conv1_fragments, conv32_fragments  # noqa: E402

gpu = torch.device('cuda', 0)
L = _lib.lib()
n = 2
yy = torch.arange(120, device=gpu).view(1, 1, 120, 1).float()
xx = torch.arange(160, device=gpu).view(1, 1, 1, 160).float()
ring = torch.zeros(n, 3, 120, 160, device=gpu)
ring[:, 0] = (yy[0, 0] * 0.25 + xx[0, 0] * 0.001)   # encodes (y, x) in fp16-representable steps
ring[:, 1] = 0.5
for (ky1, kx1, ky2, kx2) in [(0, 0, 0, 0), (3, 5, 0, 0), (0, 0, 2, 3)]:
    w1 = torch.zeros(32, 3, 8, 8, device=gpu)
    w1[0, 0, ky1, kx1] = 1.0
    w1[1, 1, 0, 0] = 1.0
    b1 = torch.zeros(32, device=gpu)
    w2 = torch.zeros(32, 32, 4, 4, device=gpu)
    w2[0, 0, ky2, kx2] = 1.0
    w2[1, 1, 0, 0] = 1.0
    b2 = torch.zeros(32, device=gpu)
    y2 = torch.zeros(n, 27, 37, 32, dtype=torch.float16, device=gpu)
    o = (ctypes.c_int32 * 3)(0, 1, 2)
    w1f, w2f = conv1_fragments(w1), conv32_fragments(w2)
    rc = L.dt_conv12(ring.data_ptr(), n, 3, o, w1f.data_ptr(), b1.data_ptr(),
                     None, None, 1e-5, w2f.data_ptr(), b2.data_ptr(),
                     y2.data_ptr(), None, 0.01, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    g = y2[0, :, :, 0].float()
    # want: y2[oy, ox] = in[2(2oy + ky2) + ky1, 2(2ox + kx2) + kx1]
    oy = torch.arange(27, device=gpu).view(27, 1)
    ox = torch.arange(37, device=gpu).view(1, 37)
    iy = 2 * (2 * oy + ky2) + ky1
    ix = 2 * (2 * ox + kx2) + kx1
    want = (iy * 0.25 + ix * 0.001).half().float()
    print('deltas', (ky1, kx1, ky2, kx2), 'rc', rc, 'max err', (g - want).abs().max().item(),
          'ch1 (0.5?)', y2[0, :, :, 1].float().min().item(), y2[0, :, :, 1].float().max().item())
    for (a, b) in [(0, 0), (0, 1), (1, 0), (5, 7), (26, 36)]:
        v = g[a, b].item()
        print('   y2[%d,%d] got %.4f (row %.2f col %.1f) want %.4f' % (a, b, v, v // 0.25, (v % 0.25) / 0.001, want[a, b].item()))
