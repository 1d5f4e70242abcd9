"""Diagnostic (GPU): reproduce the rollout actor's NaN parameters seen after
an eager DDPG update on a NaN batch (tests/test_gpu_guard.py
test_update_names_the_batch[False] followed by
test_train_loop_names_the_actor_output), checking the rollout actor's
gamma / beta after every stage to find the step that corrupts them."""
import gc
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'tests', 'golden'))
from conftest import golden  # noqa: E402
from test_trainer import formula_batch, make_trainer  # noqa: E402

gpu = torch.device('cuda', 0)
NAN = float('nan')


def bad(t):
    return int((~torch.isfinite(t.float())).sum().item())


def scan(tag, mod):
    vals = {k: bad(v) for k, v in mod.named_parameters()}
    vals.update({k: bad(v) for k, v in mod.named_buffers()})
    nz = {k: v for k, v in vals.items() if v}
    print('   %-14s %s' % (tag, nz or 'finite'), flush=True)


def report(tag, loop):
    torch.cuda.synchronize()
    print(tag, flush=True)
    scan('rollout.actor', loop.rollout.actor)
    scan('exploit_actor', loop.rollout.exploit_actor)
    scan('trainer.actor', loop.trainer.actor)
    scan('target_actor', loop.trainer.target_actor)
    scan('critic', loop.trainer.critic)


def first_test():
    if os.environ.get('SKIP_FIRST'):
        return
    tr = make_trainer(gpu, graph=False, warmup=1)
    clean = formula_batch(16)
    for _ in range(2):
        tr.update(clean)
    obs = torch.as_tensor(clean[0]).clone()
    if not os.environ.get('NO_NAN'):
        obs[2, 0, 10, 10] = NAN
    tr.update((obs,) + tuple(clean[1:]))
    try:
        tr.check()
    except Exception as e:  # noqa: BLE001
        print('first test guard:', str(e)[:120])
    if os.environ.get('KEEP'):
        return tr
    del tr
    if os.environ.get('GC'):
        gc.collect()
    torch.cuda.synchronize()
    return None


def main():
    keep = first_test()
    from aido1_amd.actor import ConfigActor
    torch.manual_seed(5)
    fresh = ConfigActor(golden('reference_config.json')['model']['actor'])
    scan('fresh CPU actor', fresh)
    scan('fresh on GPU', fresh.to(gpu))
    from aido1_amd.train_loop import TrainLoop
    loop = TrainLoop(golden('reference_config.json'), n_envs=128, device=0, seed=5,
                     buffer_size=1024, batch_size=32, graph=True)
    report('after TrainLoop()', loop)
    ea = loop.rollout.exploit_actor
    g0 = ea.gamma[0].detach()
    print('exploit gamma.0 bits[12:24]', [hex(v & 0xffffffff) for v in g0.view(torch.int32)[12:24].tolist()])
    print('exploit gamma.0 ptr %x beta.0 ptr %x' % (g0.data_ptr(), ea.beta[0].data_ptr()))
    print('trainer guard ptr %x' % loop.guard.words.data_ptr())
    for tag, fa, src in (('rollout', loop.rollout.actor, loop.trainer.actor),
                         ('exploit', ea, loop.trainer.target_actor)):
        bns = src.layers()[1]
        for i in range(4):
            eq_g = torch.equal(fa.gamma[i].detach(), bns[i].weight.detach())
            eq_b = torch.equal(fa.beta[i].detach(), bns[i].bias.detach())
            if not (eq_g and eq_b):
                print('%s layer %d gamma equal %s beta equal %s: %s' % (
                    tag, i, eq_g, eq_b, fa.gamma[i].detach()[:3].tolist()))
    ea.refresh(loop.trainer.target_actor)
    torch.cuda.synchronize()
    scan('exploit after 2nd refresh', ea)
    loop.reset()
    report('after reset', loop)
    loop.rollout.step()
    report('after rollout step', loop)
    del keep


if __name__ == '__main__':
    main()
