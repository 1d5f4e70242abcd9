"""Time one batch-64 DDPG update: eager with MIOpen, eager with torch's native
conv/BN kernels, and (last, riskiest) HIP-graph replay with native kernels."""
import sys
import time
import torch
sys.path.insert(0, 'tests'); sys.path.insert(0, 'tests/golden')
from test_trainer import make_trainer
from formulas import formula_batch

dev = torch.device('cuda', 0)
batch = [torch.as_tensor(b).to(dev) for b in formula_batch(64)]


def timed(tr, k=20):
    for _ in range(5):
        tr.update(batch)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(k):
        tr.update(batch)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / k * 1e3


mode = sys.argv[1]
if mode == 'eager_miopen':
    print('eager miopen  %.2f ms' % timed(make_trainer(dev)), flush=True)
elif mode == 'eager_native':
    torch.backends.cudnn.enabled = False
    print('eager native  %.2f ms' % timed(make_trainer(dev)), flush=True)
elif mode == 'graph_miopen':
    print('graph miopen  %.2f ms' % timed(make_trainer(dev, graph=True, warmup=2)), flush=True)
elif mode == 'graph_native':
    torch.backends.cudnn.enabled = False
    print('graph native  %.2f ms' % timed(make_trainer(dev, graph=True, warmup=2)), flush=True)

if mode == 'cmp':
    torch.backends.cudnn.allow_tf32 = False
    runs = {'eager': make_trainer(dev), 'eager_capturable': make_trainer(dev, graph=True, warmup=99),
            'graph_w1': make_trainer(dev, graph=True, warmup=1),
            'graph_w3': make_trainer(dev, graph=True, warmup=3)}
    b16 = [torch.as_tensor(b).to(dev) for b in formula_batch(16)]
    for name, tr in runs.items():
        out = []
        for k in range(5):
            m, info = tr.update(b16)
            out.append('%.6f/%.6f' % (m['critic_loss'].item(), m['actor_loss'].item()))
        print('%-17s' % name, ' '.join(out), flush=True)

if mode == 'adam':
    torch.manual_seed(0)
    for shape in ((32, 3, 8, 8), (32,), (256, 4032)):
        p0 = torch.randn(shape, device=dev) * 0.1
        g = torch.randn(shape, device=dev) * torch.logspace(-12, 0, shape[-1], device=dev)
        outs = []
        for cap in (False, True):
            p = p0.clone().requires_grad_()
            lr = torch.tensor(0.004, device=dev) if cap else 0.004
            opt = torch.optim.Adam([p], lr=lr, capturable=cap, foreach=True)
            for k in range(3):
                p.grad = g * (1 + 0.1 * k)
                opt.step()
            outs.append(p.detach())
        d = (outs[0] - outs[1]).abs()
        print('adam', shape, 'max diff %.3e  rel-to-lr %.3e' % (d.max(), d.max() / 0.004), flush=True)
