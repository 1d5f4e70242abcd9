"""Intermittent non-finite parameters after DDPG updates on the GPU
(tests/test_gpu_distributed.py, tests/test_gpu_trainer.py::test_train_loop_runs
failed so on some boxes).  Each trial is a fresh process (MIOpen's Find runs
once per process and shape): after NaN-filled blocks were freed into the caching allocator, four updates
on the formula batch, with the
update's MIOpen Find mode on or off, reporting the first update and the
parameters that went non-finite.

  python tools/nan_probe.py --trials 6
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def trial(search, graph, poison):
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    sys.path.insert(0, ROOT)
    import torch
    from test_trainer import make_trainer, formula_batch
    dev = torch.device('cuda', 0)
    if poison:
        # leave NaN-filled blocks in the caching allocator, as earlier work in
        # a long-lived process does: a kernel that reads memory it never wrote
        # then sees NaN instead of a fresh allocation's zeros
        for mb in (1, 4, 16, 64, 256):
            junk = [torch.full((mb * 262144,), float('nan'), device=dev) for _ in range(4)]
            del junk
    tr = make_trainer(dev, graph=graph, warmup=1, conv_search=search)
    out = {'search': search, 'graph': graph, 'poison': poison, 'bad': None}
    for k in range(4):
        m, info = tr.update(formula_batch(16))
        torch.cuda.synchronize()
        bad = [n for mod, tag in ((tr.actor, 'actor'), (tr.critic, 'critic'))
               for n, p in mod.named_parameters() if not torch.isfinite(p).all()]
        bad += [tag + ':' + n for mod, tag in ((tr.actor, 'actor'), (tr.critic, 'critic'))
                for n, b in mod.named_buffers() if b.is_floating_point() and not torch.isfinite(b).all()]
        losses = [float(m['critic_loss']), float(m['actor_loss'])]
        if bad or not all(map(lambda v: v == v, losses)):
            out['bad'] = {'update': k, 'params': bad[:12], 'losses': losses}
            break
    print('RESULT ' + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trials', type=int, default=6)
    ap.add_argument('--one', default='')
    args = ap.parse_args()
    if args.one:
        s, g, pz = args.one.split(',')
        trial(s == '1', g == '1', pz == '1')
        return
    for search, graph in (('1', '1'), ('0', '1'), ('1', '0')):
        nbad = 0
        for t in range(args.trials):
            r = subprocess.run([sys.executable, __file__, '--one', search + ',' + graph + ',1'],
                               capture_output=True, text=True, timeout=120)
            line = [x for x in r.stdout.splitlines() if x.startswith('RESULT ')]
            res = json.loads(line[0][7:]) if line else {'error': r.stderr[-800:]}
            nbad += 1 if (res.get('bad') or 'error' in res) else 0
            print('search=%s graph=%s trial %d: %s' % (search, graph, t, json.dumps(res)), flush=True)
        print('search=%s graph=%s: %d of %d poisoned trials non-finite'
              % (search, graph, nbad, args.trials), flush=True)


if __name__ == '__main__':
    main()
