"""Reference-mode (train-mode, batch-of-one BN) FusedActor on the GPU: max
|action error| per dtype against a float64 CPU restatement, on formula frames
and rendered frames, formula and xavier weights."""
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, 'tests'); sys.path.insert(0, 'tests/golden')
from conftest import golden
from formulas import formula_input, formula_state_dict
from test_trainer import no_dropout
from aido1_amd.actor import ConfigActor, FusedActor, apply_head
from aido1_amd.rollout import ActorRollout

dev = torch.device('cuda', 0)
cfg = golden('reference_config.json')


def f64_actor(a, x):
    convs, bns, l1, l2 = a.layers()
    h = x.double().cpu()
    for c, b in zip(convs, bns):
        h = F.leaky_relu(F.conv2d(h, c.weight.double().cpu(), c.bias.double().cpu(), stride=c.stride))
        m = h.mean((2, 3), keepdim=True)
        v = (h - m).square().mean((2, 3), keepdim=True)
        h = (h - m) / torch.sqrt(v + b.eps) * b.weight.double().cpu().view(1, -1, 1, 1) + \
            b.bias.double().cpu().view(1, -1, 1, 1)
    h = F.leaky_relu(F.linear(h.flatten(1), l1.weight.double().cpu(), l1.bias.double().cpu()))
    return apply_head(F.linear(h, l2.weight.double().cpu(), l2.bias.double().cpu()), a.head)


roll = ActorRollout(cfg, 64, device=0, seed=3, actor_mode='eval')
roll.reset()
for _ in range(5):
    roll.step()
frames = roll.stack()
for init in ('formula', 'xavier'):
    torch.manual_seed(0)
    a = ConfigActor(no_dropout(cfg['model']['actor']))
    if init == 'formula':
        a.load_state_dict(formula_state_dict(a.state_dict()))
    a = a.to(dev)
    for name, x in (('formula', formula_input(16).to(dev)), ('render', frames)):
        ref = f64_actor(a, x)
        for dt in (torch.float32, torch.float16, torch.bfloat16):
            f = FusedActor(a, dtype=dt, mode='reference')
            err = (f(x).double().cpu() - ref).abs()
            print('%-8s %-8s %-15s max %.3e mean %.3e' % (init, name, dt, err.max(), err.mean()))
