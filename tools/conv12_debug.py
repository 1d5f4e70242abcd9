"""Diagnostic: dt_conv12 vs the f32 restatement, error per conv2 output row,
eval and reference mode (tests/test_gpu_actor.py has the pass/fail form)."""
import ctypes
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd import _lib  # noqa: E402
from aido1_amd.actor import conv1_fragments, conv32_fragments  # noqa: E402

gpu = torch.device('cuda', 0)
L = _lib.lib()
torch.manual_seed(11)
n, slots, order = 8, 3, [0, 1, 2]
ring = torch.rand(n, slots, 120, 160, device=gpu)
w1 = torch.randn(32, 3, 8, 8, device=gpu) * 0.08
b1 = torch.randn(32, device=gpu) * 0.2
w2 = (torch.randn(32, 32, 4, 4, device=gpu) * 0.05).half().float()
b2 = torch.randn(32, device=gpu) * 0.1
x = ring[:, order].half().float()
h1 = F.leaky_relu(F.conv2d(x, w1.half().float(), b1, stride=2)).double()
for ident in (True, False):
    w2e = torch.zeros_like(w2)
    if ident:   # conv2 = pick conv1 channel c at kernel offset (0,0): y2[c,oy,ox] = h1[c,2oy,2ox]
        for c in range(32):
            w2e[c, c, 0, 0] = 1.0
        b2e = torch.zeros_like(b2)
    else:
        w2e, b2e = w2, b2
    want = F.leaky_relu(F.conv2d(h1.half().double(), w2e.double(), b2e.double(), stride=2))
    y2 = torch.zeros(n, 27, 37, 32, dtype=torch.float16, device=gpu)
    o = (ctypes.c_int32 * 3)(*order)
    w1f, w2f = conv1_fragments(w1), conv32_fragments(w2e)
    rc = L.dt_conv12(ring.data_ptr(), n, slots, o, w1f.data_ptr(), b1.data_ptr(),
                     None, None, 1e-5, w2f.data_ptr(), b2e.data_ptr(),
                     y2.data_ptr(), None, 0.01, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = y2.permute(0, 3, 1, 2).double()
    err = (got - want).abs()
    print('identity conv2' if ident else 'random conv2', 'rc', rc, 'max err', err.max().item(),
          'max want', want.abs().max().item())
    print('  err per output row:', ['%.2g' % v for v in err.amax((0, 1, 3)).tolist()])
    print('  err per output col:', ['%.2g' % v for v in err.amax((0, 1, 2)).tolist()])
    print('  err per channel:', ['%.2g' % v for v in err.amax((0, 2, 3)).tolist()])
    print('  err per sample:', ['%.2g' % v for v in err.amax((1, 2, 3)).tolist()])
    if ident:
        print('  got[0,:4,0,0]', got[0, :4, 0, 0].tolist(), 'want', want[0, :4, 0, 0].tolist())
        print('  got[0,0,0,:6]', got[0, 0, 0, :6].tolist(), 'want', want[0, 0, 0, :6].tolist())
