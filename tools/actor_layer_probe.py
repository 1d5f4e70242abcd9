"""Per-layer check of the reference-mode actor on the GPU: torch train-mode
modules (batch of one) and the FusedActor path, each against float64 CPU."""
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, 'tests'); sys.path.insert(0, 'tests/golden')
from conftest import golden
from formulas import formula_input, formula_state_dict
from test_trainer import no_dropout
from aido1_amd.actor import ConfigActor, FusedActor

torch.backends.cudnn.allow_tf32 = False
dev = torch.device('cuda', 0)
cfg = golden('reference_config.json')
a = ConfigActor(no_dropout(cfg['model']['actor']))
a.load_state_dict(formula_state_dict(a.state_dict()))
a.train()
convs, bns, lin1, lin2 = a.layers()
n = 16
x = formula_input(n)


def f64_layers(x):
    outs = []
    h = x.double()
    for c, b in zip(convs, bns):
        h = F.leaky_relu(F.conv2d(h, c.weight.double(), c.bias.double(), stride=c.stride))
        m = h.mean((2, 3), keepdim=True)
        v = (h - m).square().mean((2, 3), keepdim=True)
        h = (h - m) / torch.sqrt(v + b.eps) * b.weight.double().view(1, -1, 1, 1) + \
            b.bias.double().view(1, -1, 1, 1)
        outs.append(h)
    return outs


ref = f64_layers(x)
ag = ConfigActor(no_dropout(cfg['model']['actor']))
ag.load_state_dict(a.state_dict())
ag = ag.to(dev).train()
gc, gb, _, _ = ag.layers()
# torch modules on GPU, batch of one
for i in range(n):
    h = x[i:i + 1].to(dev)
    errs = []
    with torch.no_grad():
        for k, (c, b) in enumerate(zip(gc, gb)):
            h = b(F.leaky_relu(c(h)))
            errs.append((h.double().cpu() - ref[k][i:i + 1]).abs().max().item())
    print('torch-gpu sample %2d' % i, ' '.join('%.1e' % e for e in errs))
f = FusedActor(ag, dtype=torch.float32, mode='reference')
h = x.to(dev).to(memory_format=torch.channels_last)
with torch.no_grad():
    for k in range(4):
        h = F.conv2d(h, f.w[k], f.b[k], stride=f.strides[k])
        h = f._lrelu_sample_norm(h, k)
        e = (h.double().cpu() - ref[k]).abs().amax((1, 2, 3))
        print('fused layer %d' % k, ' '.join('%.1e' % v for v in e.tolist()))
