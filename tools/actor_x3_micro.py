"""Time the float32-accurate actor chain (dt_conv1x_split / dt_conv32x_split +
float32 linears) against the fp16 fast chain at 4096 samples, on palette-index
frames, with the exploring / exploiting split (3584 + 512) the rollout uses.

    python tools/actor_x3_micro.py [--n 4096] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--layers', action='store_true', help='per-layer times of the x3 chain')
    args = ap.parse_args()
    from aido1_amd.actor import ConfigActor, FusedActor
    cfg = json.load(open(os.path.join(os.path.dirname(__file__), '..', 'tests', 'golden',
                                      'reference_config.json')))['model']['actor']
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    a, b = ConfigActor(cfg).to(dev), ConfigActor(cfg).to(dev)
    n = args.n
    n0 = n * 7 // 8
    ring = torch.randint(0, 8, (n, 3, 120, 160), dtype=torch.uint8, device=dev)
    order = [2, 0, 1]
    res = {}
    for name, dt in (('fp16', torch.float16), ('x3_f32', torch.float32)):
        fa = FusedActor(a, dtype=dt, mode='reference')
        fb = FusedActor(b, dtype=dt, mode='reference')
        for _ in range(3):
            fa.forward_pair(fb, ring, order, n0)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.iters)]
        for s, e in ev:
            s.record()
            fa.forward_pair(fb, ring, order, n0)
            e.record()
        torch.cuda.synchronize()
        ts = sorted(s.elapsed_time(e) for s, e in ev)
        res[name] = {'median_ms': ts[len(ts) // 2], 'min_ms': ts[0]}
        if name == 'x3_f32' and args.layers:
            import ctypes
            from aido1_amd import _lib
            L = _lib.lib()
            B = fa._x3_buffers(n, dev)
            st = torch.cuda.current_stream().cuda_stream
            o = (ctypes.c_int32 * 3)(*order)
            calls = {
                'conv1x': lambda: L.dt_conv1x_split(ring.data_ptr(), 1, n, 3, o, fa.w0x.data_ptr(),
                                                    fa.bf[0].data_ptr(), None, B['y1'].data_ptr(),
                                                    B['p1'].data_ptr(), 0.01, st)}
            ins = [('y1', 'p1'), ('y2', 'p2'), ('y3', 'p3')]
            outs = [('y2', 'p2'), ('y3', 'p3'), ('flat', None)]
            for layer in range(3):
                last = layer == 2

                def call(layer=layer, last=last):
                    x, pp = ins[layer]
                    y, po = outs[layer]
                    return L.dt_conv32x_split(
                        layer + 2, n, B[x].data_ptr(), fa.wx32[layer].data_ptr(),
                        fa.bf[layer + 1].data_ptr(), B[pp].data_ptr(),
                        fa.gamma[layer].data_ptr(), fa.beta[layer].data_ptr(), 1e-5,
                        B[y].data_ptr(), B[po].data_ptr() if po else None,
                        fa.gamma[3].data_ptr() if last else None,
                        fa.beta[3].data_ptr() if last else None, 1e-5, 0.01, None, st)
                calls['conv%dx' % (layer + 2)] = call
            for k, f in calls.items():
                assert f() == 0
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(args.iters)]
                for s, e in ev:
                    s.record()
                    f()
                    e.record()
                torch.cuda.synchronize()
                ts = sorted(s.elapsed_time(e) for s, e in ev)
                res['layer_' + k + '_ms'] = ts[len(ts) // 2]
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
