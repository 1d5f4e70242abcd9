"""Diagnostic: where a dt_conv12 workgroup spends its time (shader-clock stamps
of the -DDTSIM_STAMPS build, tools/step_stamps.sh; run with
DTSIM_DIAG_LIB=aido1_amd/libdtsim_stamps.so)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd import _lib  # noqa: E402
from aido1_amd.actor import ConfigActor, FusedActor  # noqa: E402

gpu = torch.device('cuda', 0)
import json  # noqa: E402
cfg = json.load(open(os.path.join(os.path.dirname(__file__), '..', 'aido1_amd', 'configs',
                                  'reference_config.json')))
a = ConfigActor(cfg['model']['actor']).to(gpu)
mode = os.environ.get('MODE', 'reference')
f = FusedActor(a, dtype=torch.float16, mode=mode)
x = torch.rand(4096, 3, 120, 160, device=gpu)
L = _lib.lib()
L.dt_diag_c12stamps.argtypes = [ctypes.c_void_p]
buf = np.zeros((4096, 8), np.uint64)
recs = []
for it in range(6):
    f(x)
    torch.cuda.synchronize()
    if it >= 2:
        L.dt_diag_c12stamps(buf.ctypes.data_as(ctypes.c_void_p))
        recs.append(buf.astype(np.int64).copy())
b = np.stack(recs)
life = (b[..., 1] - b[..., 0]) / 100.0
cyc = b[..., 7] - b[..., 2]
clk = np.median(cyc / (life * 1e3))
names = ['weights + step-0 rows', 'phase A (conv1, 35 steps)', 'phase B (norm)',
         'C: first row writes', 'C: rest (conv2 8 steps)']
print('mode %s: workgroup life median %.2f us (p10 %.2f p90 %.2f), clock %.2f GHz; launch span %.1f us'
      % (mode, np.median(life), np.percentile(life, 10), np.percentile(life, 90), clk,
         (b[-1, :, 1].max() - b[-1, :, 0].min()) / 100.0))
for i, nm in enumerate(names):
    d = b[..., 3 + i] - b[..., 2 + i]
    print('  %-28s median %7.0f cyc (%.2f us)' % (nm, np.median(d), np.median(d) / clk / 1e3))
