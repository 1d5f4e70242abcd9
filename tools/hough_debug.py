"""Diagnostic: dt_hough_lines vs oracle/hough_oracle.c on synthetic images;
for the first mismatching image, the first divergence of the visit traces."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from oracle import linedet_ref as LR  # noqa: E402
from aido1_amd import _lib  # noqa: E402
from aido1_amd.render import hough_lines  # noqa: E402
from test_gpu_hough import _synthetic  # noqa: E402

params = (2, 3, 1)
imgs = _synthetic(48, sum(params))
lines, counts = hough_lines(torch.from_numpy(imgs).to('cuda'), *params)
bad = []
for i in range(48):
    want = LR.hough_lines(imgs[i], *params)
    c = int(counts[i])
    got = lines[i, :max(c, 0)].cpu().numpy()
    if c != len(want) or not np.array_equal(got, want):
        bad.append(i)
print('mismatching images', bad)
if bad:
    i = bad[0]
    L = _lib.lib()
    L.dt_diag_hough_trace.argtypes = [ctypes.c_void_p]
    tr = torch.full((4096, 4), -7, dtype=torch.int32, device='cuda')
    L.dt_diag_hough_trace(tr.data_ptr())
    hough_lines(torch.from_numpy(imgs[i:i + 1]).to('cuda'), *params)
    L.dt_diag_hough_trace(None)
    gt = tr.cpu().numpy()
    ot = np.full((4096, 4), -7, np.int32)
    LR.hough_lines(imgs[i], *params, trace=ot)
    d = np.nonzero(np.any(gt != ot, axis=1))[0]
    print('image', i, 'first trace divergence at visit', d[:1], 'of', len(d))
    if len(d):
        k = d[0]
        for j in range(max(0, k - 2), k + 3):
            print('  visit', j, 'gpu', gt[j].tolist(), 'oracle', ot[j].tolist())
