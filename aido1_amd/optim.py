"""Optimisers the reference's trainer can be configured with
(training/trainers.py:258-268): "adam" (torch Adam, lr set per step by the
decay), "adamw" (models/adamw.py: Adam followed by p -= p * lr * wd), "sgd"
(momentum 0.9, weight decay 1e-4).  All start at lr 0 as the reference's."""
import math

import torch
from torch.optim.optimizer import Optimizer


class AdamW(Optimizer):
    """models/adamw.py:10-109 (the egg-west variant): Adam moments, step
    lr * sqrt(1 - b2^t) / (1 - b1^t), then decoupled decay p -= p * (lr * wd)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group['betas']
            for p in group['params']:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st['step'] = 0
                    st['exp_avg'] = torch.zeros_like(p)
                    st['exp_avg_sq'] = torch.zeros_like(p)
                st['step'] += 1
                m, v = st['exp_avg'], st['exp_avg_sq']
                m.mul_(b1).add_(p.grad, alpha=1 - b1)
                v.mul_(b2).addcmul_(p.grad, p.grad, value=1 - b2)
                denom = v.sqrt().add_(group['eps'])
                step_size = group['lr'] * math.sqrt(1 - b2 ** st['step']) / (1 - b1 ** st['step'])
                p.addcdiv_(m, denom, value=-step_size)
                p.sub_(p * (group['lr'] * group['weight_decay']))
        return loss


def float64_steps(opt):
    """Pre-create a capturable torch Adam's state with float64 `step` tensors.

    torch keeps a capturable Adam's step count as a float32 device tensor, so
    its bias corrections 1 - b^t are rounded to float32 (1 - 0.999 is off by
    1.3e-5 relative, which moves every update by ~6e-6 relative), while plain
    Adam computes them in float64 from a Python number.  With float64 steps
    the graph path's update is plain Adam's to the last bits."""
    for group in opt.param_groups:
        for p in group['params']:
            st = opt.state[p]
            if not st:
                st['step'] = torch.zeros((), dtype=torch.float64, device=p.device)
                st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
    return opt


def make_optimizer(kind, params, capturable=False, device=None):
    """capturable: Adam with a device-tensor lr and step counters, so the step
    can live inside a HIP graph (the lr is then set with fill_; float64, so a
    float64 update sees the lr the eager path would)."""
    if kind == 'adam':
        if capturable:
            return float64_steps(torch.optim.Adam(
                params, lr=torch.tensor(0.0, dtype=torch.float64, device=device),
                capturable=True, foreach=True))
        return torch.optim.Adam(params, lr=0.)
    if kind == 'adamw':
        return AdamW(params, lr=0., weight_decay=0.0001)
    if kind == 'sgd':
        return torch.optim.SGD(params, lr=0., momentum=0.9, weight_decay=0.0001)
    raise NotImplementedError(kind)
