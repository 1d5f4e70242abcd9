"""Diagnostic (GPU): where do the rollout actor's non-finite outputs come from?
Round 4's guards named `actor_out` at tick 0 in 3 tests of one full GPU
suite run (tests/test_gpu_trainer.py, test_gpu_guard.py), i.e. the fp16
reference-mode FusedActor on freshly rendered frames, before any update.

A: the split forward (forward_pair, dropout off) repeated on ONE ring: every
   buffer of the conv chain compared with the first repetition (a race shows
   as a mismatch) and scanned for NaN / Inf.
B: the same with the ring re-rendered from the same poses each time.
C: the loop itself (ActorRollout.step) with every buffer scanned per decision.
Prints the first bad buffer / rows it finds."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aido1_amd.rollout import ActorRollout  # noqa: E402

REPS = int(os.environ.get('REPS', '150'))


def bufs(actor):
    return {k: v for k, v in actor._bufs.items() if v is not None}


def snap(actor, flat, out):
    d = {k: v.clone() for k, v in bufs(actor).items()}
    d['flat'] = flat.clone()
    d['out'] = out.clone()
    return d


def bad_rows(t):
    f = ~torch.isfinite(t.float().reshape(t.shape[0], -1))
    return f.any(1).nonzero().flatten().tolist()


def run_pair(roll):
    a, b = roll.actor, roll.exploit_actor
    flat = a._convs_pair(b, roll.ring, roll.order(), roll.n_explore)
    out = torch.empty(roll.n, 2, device=roll.ring.device)
    a._heads(b, flat, roll.n_explore, out)
    return flat, out


def main():
    with open(os.path.join(os.path.dirname(__file__), '..', 'aido1_amd', 'configs',
                           'reference_config.json')) as f:
        cfg = json.load(f)
    n = int(os.environ.get('ENVS', '128'))
    if os.environ.get('POISON'):
        # the caching allocator's free blocks full of NaN: any buffer read
        # before it is written then shows up as non-finite
        held = []
        for mb in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512):
            for _ in range(3):
                held.append(torch.full((mb << 18,), float('nan'), device='cuda'))
        for kb in (1, 4, 16, 64, 256):
            for _ in range(16):
                held.append(torch.full((kb << 8,), float('nan'), device='cuda'))
        torch.cuda.synchronize()
        del held
        print('poisoned the caching allocator')
    torch.manual_seed(5)
    roll = ActorRollout(cfg, n, device=0, seed=5)
    roll.reset()
    for act in (roll.actor, roll.exploit_actor):
        act.p_drop = 0.0
    torch.cuda.synchronize()
    print('ring finite:', bool(torch.isfinite(roll.ring).all()), 'min/max', roll.ring.min().item(),
          roll.ring.max().item())
    flat, out = run_pair(roll)
    torch.cuda.synchronize()
    ref = snap(roll.actor, flat, out)
    for k, v in ref.items():
        br = bad_rows(v)
        if br:
            print('A rep 0: %s non-finite rows %s' % (k, br[:20]))
    mism = 0
    for rep in range(1, REPS):
        flat, out = run_pair(roll)
        cur = snap(roll.actor, flat, out)
        for k in ref:
            if not torch.equal(cur[k], ref[k]):
                diff = (cur[k].float() - ref[k].float()).abs()
                rows = (diff.reshape(diff.shape[0], -1) > 0).any(1).nonzero().flatten().tolist()
                if mism < 12:
                    print('A rep %d: %s differs in rows %s (max %.3g); non-finite rows %s'
                          % (rep, k, rows[:12], diff.nan_to_num(1e30).max().item(),
                             bad_rows(cur[k])[:12]))
                mism += 1
    print('A: %d buffer mismatches over %d repetitions' % (mism, REPS))
    # C: the loop (dropout live again), every buffer scanned per decision
    for act in (roll.actor, roll.exploit_actor):
        act.p_drop = 0.5
    nbad = 0
    for d in range(40):
        roll.step()
        for k, v in list(bufs(roll.actor).items()) + [('actor_out', roll.actor_out),
                                                        ('ring', roll.ring)]:
            br = bad_rows(v)
            if br and nbad < 12:
                print('C decision %d: %s non-finite rows %s' % (d, k, br[:12]))
                nbad += 1
    torch.cuda.synchronize()
    print('C: %d non-finite findings over 40 decisions' % nbad)


if __name__ == '__main__':
    main()
