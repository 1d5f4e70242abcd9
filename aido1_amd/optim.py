"""Optimisers the reference's trainer can be configured with
(training/trainers.py:258-268): "adam" (torch Adam, lr set per step by the
decay), "adamw" (models/adamw.py: Adam followed by p -= p * lr * wd), "sgd"
(momentum 0.9, weight decay 1e-4).  All start at lr 0 as the reference's."""
import ctypes
import math

import numpy as np
import torch
from torch.optim.optimizer import Optimizer

MT_CHUNK = 4096       # DT_MT_CHUNK (include/dttrain.h)


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


class MultiTensorTable:
    """Device tables for include/dttrain.h's multi-tensor kernels: one
    dt_mt_tensor row (up to four float32 tensors of n elements, same strides)
    per entry and the (tensor, chunk) pairs, one workgroup per DT_MT_CHUNK
    elements.  Built eagerly (an H2D copy), so before any graph capture."""

    ROW = np.dtype([('a', '<u8'), ('b', '<u8'), ('c', '<u8'), ('d', '<u8'), ('n', '<i8')])

    def __init__(self, rows, device):
        tab = np.zeros(len(rows), self.ROW)
        chunks = []
        for i, r in enumerate(rows):
            ptrs = [t.data_ptr() for t in r] + [0] * (4 - len(r))
            n = r[0].numel()
            tab[i] = tuple(ptrs) + (n,)
            chunks += [(i, c) for c in range((n + MT_CHUNK - 1) // MT_CHUNK)]
        self.key = self.key_of(rows)
        self.tensors = torch.from_numpy(tab.view(np.uint8).copy()).to(device)
        self.chunks = torch.tensor(chunks, dtype=torch.int32, device=device).reshape(-1)
        self.n_chunks = len(chunks)
        self.sizes = [r[0].numel() for r in rows]

    def refill(self, rows):
        """New pointers for rows of the same sizes, written into the same
        device table (a captured launch that reads it sees them)."""
        if [r[0].numel() for r in rows] != self.sizes:
            raise ValueError('refill needs rows of the same sizes')
        tab = np.zeros(len(rows), self.ROW)
        for i, r in enumerate(rows):
            tab[i] = tuple([t.data_ptr() for t in r] + [0] * (4 - len(r))) + (r[0].numel(),)
        self.tensors.copy_(torch.from_numpy(tab.view(np.uint8).copy()))
        self.key = self.key_of(rows)

    @staticmethod
    def key_of(rows):
        return tuple(t.data_ptr() for r in rows for t in r)

    @staticmethod
    def fits(rows):
        """float32 CUDA tensors, dense, each row's tensors with the same strides."""
        for r in rows:
            t0 = r[0]
            for t in r:
                if (not t.is_cuda or t.dtype != torch.float32 or t.stride() != t0.stride()
                        or t.shape != t0.shape or not (
                            t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(
                                memory_format=torch.channels_last)))):
                    return False
        return True


class DeviceAdam(torch.optim.Adam):
    """Capturable torch Adam whose step is ONE dt_adam launch over all
    parameters (include/dttrain.h) instead of torch's ~10 foreach kernels
    plus a per-parameter division for the float64 bias corrections.  The
    state is torch's (exp_avg, exp_avg_sq per parameter; one shared float64
    step tensor), so state_dict / load_state_dict are Adam's.  The lr is a
    float64 device tensor, set with fill_ (TrainingDecay).  Falls back to
    torch's step for anything dt_adam does not cover (CPU, non-float32,
    weight decay, amsgrad, maximize)."""

    def __init__(self, params, device):
        super().__init__(params, lr=torch.tensor(0.0, dtype=torch.float64, device=device),
                         capturable=True, foreach=True)
        self._step_t = torch.zeros((), dtype=torch.float64, device=device)
        self._counter = torch.zeros(1, dtype=torch.int32, device=device)
        for group in self.param_groups:
            for p in group['params']:
                st = self.state[p]
                st['step'] = self._step_t
                st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
        self._table = None
        self.guard, self.grad_bit, self.param_bit = None, -1, -1

    def set_guard(self, guard, grad_stage, param_stage):
        """Report non-finite gradients / updated parameters into `guard`
        (aido1_amd/guard.py): inside dt_adam, or by scans around torch's step
        when it falls back."""
        from aido1_amd.guard import BIT
        self.guard, self.grad_bit, self.param_bit = guard, BIT[grad_stage], BIT[param_stage]

    def load_state_dict(self, state_dict):
        """Adam's, then the one shared float64 step tensor again (torch restores
        a float32 step per parameter, which would send every later step down
        the torch fallback) and the moments in their parameter's memory format
        (the dt_adam table needs equal strides).  Each group keeps its own
        float64 device lr tensor, filled with the loaded value: torch would
        put a deep copy there (a host tensor after map_location='cpu'), which
        dt_adam cannot read and which HIP graphs captured earlier and
        TrainingDecay's fill_ never see.  Likewise the moments are copied into
        the tensors they replace, so a captured dt_adam keeps reading them."""
        lrs = [g['lr'] for g in self.param_groups]
        old = {p: (st.get('exp_avg'), st.get('exp_avg_sq')) for p, st in self.state.items()}
        super().load_state_dict(state_dict)
        for g, lr in zip(self.param_groups, lrs):
            loaded = g['lr']
            if torch.is_tensor(lr):
                lr.fill_(float(loaded.item() if torch.is_tensor(loaded) else loaded))
                g['lr'] = lr
        step = None
        for group in self.param_groups:
            for p in group['params']:
                st = self.state[p]
                if 'step' in st and step is None:
                    step = st['step']
                for k, prev in zip(('exp_avg', 'exp_avg_sq'), old.get(p, (None, None))):
                    if k not in st:
                        continue
                    if prev is not None and prev.shape == st[k].shape:
                        st[k] = prev.copy_(st[k])
                    elif st[k].stride() != p.stride() or st[k].device != p.device:
                        st[k] = torch.empty_like(p).copy_(st[k])
        if step is not None:
            self._step_t.copy_(torch.as_tensor(step, dtype=torch.float64))
        for group in self.param_groups:
            for p in group['params']:
                self.state[p]['step'] = self._step_t
        self._table = None

    def _rows(self, grads=None):
        rows = []
        params = [p for group in self.param_groups for p in group['params']]
        if grads is not None:
            if len(grads) != len(params):
                raise ValueError('one gradient per parameter')
            for p, gr in zip(params, grads):
                st = self.state[p]
                rows.append((p, gr, st['exp_avg'], st['exp_avg_sq']))
            return rows
        for p in params:
            if p.grad is not None:
                st = self.state[p]
                rows.append((p, p.grad, st['exp_avg'], st['exp_avg_sq']))
        return rows

    def finish_capture(self):
        """After a HIP graph captured step(grads=...): write the captured
        gradients' addresses into the table the captured dt_adam reads."""
        if getattr(self, '_deferred', None) is not None:
            self._table.refill(self._deferred)
            self._deferred = None

    @torch.no_grad()
    def step(self, closure=None, grads=None):
        """grads: the gradients as a list in parameter order (the trainer's
        torch.autograd.grad outputs) instead of .grad, so nothing is copied
        into .grad; inside a graph capture with new addresses the table is
        refilled by finish_capture() (its launch reads the table then)."""
        g = self.param_groups[0]
        rows = self._rows(grads)
        if grads is not None and not (MultiTensorTable.fits(rows) and len(self.param_groups) == 1
                                       and not g['weight_decay'] and not g['amsgrad']
                                       and not g['maximize'] and torch.is_tensor(g['lr'])):
            for p, gr in zip([p for gp in self.param_groups for p in gp['params']], grads):
                if p.grad is None:     # .grad in the parameter's own memory format
                    p.grad = torch.empty_like(p)
                p.grad.copy_(gr)
            grads, rows = None, self._rows()
        if (len(self.param_groups) != 1 or g['weight_decay'] or g['amsgrad'] or g['maximize']
                or not torch.is_tensor(g['lr']) or not rows or not MultiTensorTable.fits(rows)
                or any(self.state[r[0]]['step'] is not self._step_t for r in rows)):
            # torch's step increments every state's step: give each its own
            for group in self.param_groups:
                for p in group['params']:
                    st = self.state[p]
                    if st.get('step') is self._step_t:
                        st['step'] = self._step_t.clone()
            if self.guard is not None:
                self.guard.scan(self.grad_bit, *[r[1] for r in rows])
            out = super().step(closure)
            if self.guard is not None:
                self.guard.scan(self.param_bit, *[r[0] for r in rows])
            return out
        if self._table is None or self._table.key != MultiTensorTable.key_of(rows):
            if (torch.cuda.is_current_stream_capturing() and self._table is not None
                    and self._table.sizes == [r[0].numel() for r in rows]):
                self._deferred = rows          # finish_capture() writes them
            else:
                self._table = MultiTensorTable(rows, self._step_t.device)
        from aido1_amd import _lib
        t = self._table
        b1, b2 = g['betas']
        rc = _lib.lib().dt_adam(t.n_chunks, t.tensors.data_ptr(), t.chunks.data_ptr(),
                                self._step_t.data_ptr(), g['lr'].data_ptr(), float(b1), float(b2),
                                float(g['eps']), self._counter.data_ptr(),
                                self.guard.ptr() if self.guard is not None else None,
                                self.grad_bit, self.param_bit,
                                ctypes.c_void_p(torch.cuda.current_stream(self._step_t.device)
                                                .cuda_stream))
        if rc != 0:
            raise _lib.DtError('dt_adam failed (%d)' % rc)
        return None


class SoftUpdate:
    """models/torch_utils.py:5-9 for a (target, source) module pair: one
    dt_soft_update launch on the GPU, torch foreach ops otherwise."""

    def __init__(self):
        self._tables = {}

    @torch.no_grad()
    def __call__(self, target, source, tau):
        self.many([(target, source)], tau)

    @torch.no_grad()
    def many(self, pairs, tau):
        """Every (target, source) pair of `pairs` in ONE dt_soft_update launch
        (the trainer's target actor and target critic together)."""
        rows = [(t.data, s.data) for target, source in pairs
                for t, s in zip(target.parameters(), source.parameters())]
        if not rows or not MultiTensorTable.fits(rows):
            tp = [r[0] for r in rows]
            a = torch._foreach_mul(tp, 1.0 - tau)
            b = torch._foreach_mul([r[1] for r in rows], tau)
            torch._foreach_add_(a, b)
            torch._foreach_copy_(tp, a)
            return
        key = tuple((id(target), id(source)) for target, source in pairs)
        t = self._tables.get(key)
        if t is None or t.key != MultiTensorTable.key_of(rows):
            t = self._tables[key] = MultiTensorTable(rows, rows[0][0].device)
        from aido1_amd import _lib
        rc = _lib.lib().dt_soft_update(t.n_chunks, t.tensors.data_ptr(), t.chunks.data_ptr(),
                                       float(tau), ctypes.c_void_p(torch.cuda.current_stream(
                                           rows[0][0].device).cuda_stream))
        if rc != 0:
            raise _lib.DtError('dt_soft_update failed (%d)' % rc)


def make_optimizer(kind, params, capturable=False, device=None):
    """capturable: Adam with a device-tensor lr and step counters, so the step
    can live inside a HIP graph (the lr is then set with fill_; float64, so a
    float64 update sees the lr the eager path would)."""
    if kind == 'adam':
        if capturable:
            dev = torch.device(device) if device is not None else None
            if dev is not None and dev.type == 'cuda':
                return DeviceAdam(params, dev)
            return float64_steps(torch.optim.Adam(
                params, lr=torch.tensor(0.0, dtype=torch.float64, device=device),
                capturable=True, foreach=True))
        return torch.optim.Adam(params, lr=0.)
    if kind == 'adamw':
        return AdamW(params, lr=0., weight_decay=0.0001)
    if kind == 'sgd':
        return torch.optim.SGD(params, lr=0., momentum=0.9, weight_decay=0.0001)
    raise NotImplementedError(kind)
