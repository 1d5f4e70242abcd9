"""The DDPG update's train-mode layers on the GPU kernels (include/dttrain.h,
include/dtupd.h).

Every conv block of config.json's actor and critic is conv_2d -> leaky_relu
-> batch_norm_2d (models/ddpg/modules.py MetaNet), and the trainer runs all
four networks in train mode (training/trainers.py:143-237).  On the GPU in
float32 with channels_last activations:
* ``conv_trunk``: a run of such blocks on config.json's four layers as ONE
  chain (dtupd.h): each convolution merges the previous block's BatchNorm
  partials itself and normalises while it loads, so no normalised activation
  is stored; the last block writes the trunk's output in NCHW (the flatten
  after it is a view).  Backward: dt_bn_leaky_bwd per block, the weight
  gradient normalising its input rows again while staging them, the input
  gradient.
* ``conv_leaky_bn``: one block (dt_upd_conv_fwd_bn + dt_bn_leaky_apply on
  dtupd.h's layers; MIOpen + dt_bn_leaky_fwd for any other shape).
* ``linear``: the long-K linear after the trunk (4032 -> 256 / 512) with its
  LeakyReLU, split-K MFMA kernels.
The activation leaky(z + bias) is never stored: every kernel recomputes it
from the convolution output z.  The modules, parameters and state_dict are
the unchanged torch ones; ``applicable`` / ``trunk_len`` /
``linear_applicable`` say when the kernels replace them.

Streams: every BatchNorm module owns its kernels' scratch (the partials and
work buffers, ``_dt_part`` / ``_dt_work``), so ONE module must not be
forwarded on two streams at once.  The trainer's two-stream stages
(trainer._fork) forward different modules on each branch;
tests/test_gpu_trainer.py checks them against the one-stream order bit for
bit, eager and captured.
"""
import contextlib
import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from aido1_amd import _lib

C = 32


def applicable(x, conv, act, bn):
    return (x.is_cuda and x.dtype == torch.float32 and bn.training and bn.track_running_stats
            and bn.affine and bn.momentum is not None and bn.running_mean is not None
            and conv.bias is not None and conv.out_channels == C and conv.groups == 1
            and tuple(conv.padding) == (0, 0) and tuple(conv.dilation) == (1, 1)
            and isinstance(act, nn.LeakyReLU) and bn.num_features == C
            and conv.weight.dtype == torch.float32)


def _work(bn, key, dev):
    """A scratch buffer per BatchNorm and direction, zeroed once (the kernels
    leave their counters and partial counts at zero): plain attributes, not
    state."""
    name = '_dt_work_' + key
    w = getattr(bn, name, None)
    if w is None or w.device != dev:
        L = _lib.lib()
        size = L.dt_upd_bn_work_floats() if key == 'upd' else L.dt_train_work_floats(0)
        w = torch.zeros(int(size), device=dev)
        setattr(bn, name, w)
    return w


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _guard(bn):
    """The guard block the trainer attached (aido1_amd/guard.py), or NULL."""
    g = getattr(bn, '_dt_guard', None)
    return g.ptr() if g is not None else None


def attach_guard(module, guard):
    """Report every fused BatchNorm of `module` into `guard` (DT_GUARD_BN_*)."""
    for m in module.modules():
        if isinstance(m, nn.BatchNorm2d):
            m._dt_guard = guard


class _BnLeaky(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, bias, gamma, beta, bn, slope):
        L = _lib.lib()
        m = z.numel() // C
        y = torch.empty_like(z)
        mi = torch.empty(2 * C, device=z.device)
        nbt = bn.num_batches_tracked
        rc = L.dt_bn_leaky_fwd(m, z.data_ptr(), bias.data_ptr(), slope, gamma.data_ptr(),
                               beta.data_ptr(), bn.eps, bn.momentum, bn.running_mean.data_ptr(),
                               bn.running_var.data_ptr(),
                               nbt.data_ptr() if nbt is not None else None,
                               int(getattr(bn, '_dt_updates', 1)), None,
                               y.data_ptr(), mi.data_ptr(), _work(bn, 'fwd', z.device).data_ptr(),
                               _guard(bn), _stream(z.device))
        if rc != 0:
            raise _lib.DtError('dt_bn_leaky_fwd failed (%d)' % rc)
        # the activation is recomputed from z and bias in the backward (never stored)
        ctx.save_for_backward(z, bias, mi, gamma)
        ctx.bn, ctx.slope = bn, slope
        return y

    @staticmethod
    def backward(ctx, dy):
        z, bias, mi, gamma = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        L = _lib.lib()
        dz = torch.empty_like(z)
        g = torch.empty(3, C, device=z.device)      # dbias, dgamma, dbeta
        rc = L.dt_bn_leaky_bwd(z.numel() // C, dy.data_ptr(), z.data_ptr(), bias.data_ptr(),
                               mi.data_ptr(), gamma.data_ptr(), ctx.slope, dz.data_ptr(),
                               g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(),
                               _work(ctx.bn, 'bwd', z.device).data_ptr(), _guard(ctx.bn),
                               _stream(z.device))
        if rc != 0:
            raise _lib.DtError('dt_bn_leaky_bwd failed (%d)' % rc)
        return dz, g[0], g[1], g[2], None, None


@contextlib.contextmanager
def running_updates(module, k):
    """Inside: each fused train-mode BatchNorm of `module` moves its running
    statistics k times (num_batches_tracked += k), as k train-mode forwards
    over the same batch do; its output is the one forward's."""
    bns = [m for m in module.modules() if isinstance(m, nn.BatchNorm2d)]
    for m in bns:
        m._dt_updates = int(k)
    try:
        yield
    finally:
        for m in bns:
            m._dt_updates = 1


# (C_in, KS, ST, IH, IW) of include/dtupd.h's kernels: config.json's four
# conv_2d layers at 120 x 160 observations
UPD_CONV_LAYERS = {(3, 8, 2, 120, 160), (32, 4, 2, 57, 77), (32, 4, 2, 27, 37),
                   (32, 4, 1, 12, 17)}


def upd_conv_applicable(x, conv):
    """The update's convolution runs on dt_upd_conv_* (f32 MFMA) for these."""
    w = conv.weight
    return (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 4
            and conv.out_channels == C and conv.groups == 1
            and tuple(conv.padding) == (0, 0) and tuple(conv.dilation) == (1, 1)
            and conv.stride[0] == conv.stride[1] and w.shape[2] == w.shape[3]
            and (x.shape[1], w.shape[2], conv.stride[0], x.shape[2], x.shape[3])
            in UPD_CONV_LAYERS)


class _UpdConv(torch.autograd.Function):
    """conv2d(x, w, stride) without bias on include/dtupd.h: NHWC f32, the
    weight in its channels_last memory ([co][kh][kw][ci]); backward = the
    kernels' weight gradient (deterministic chunked sum) and input gradient."""

    @staticmethod
    def forward(ctx, x, w, st):
        cl = torch.channels_last
        x = x.contiguous(memory_format=cl)
        w = w.contiguous(memory_format=cl)
        n, cin, ih, iw = x.shape
        ks = w.shape[2]
        oh, ow = (ih - ks) // st + 1, (iw - ks) // st + 1
        z = torch.empty((n, C, oh, ow), device=x.device, dtype=x.dtype, memory_format=cl)
        rc = _lib.lib().dt_upd_conv_fwd(cin, ks, st, n, ih, iw, x.data_ptr(), w.data_ptr(),
                                        z.data_ptr(), _stream(x.device))
        if rc != 0:
            raise _lib.DtError('dt_upd_conv_fwd failed (%d)' % rc)
        ctx.save_for_backward(x, w)
        ctx.st = st
        return z

    @staticmethod
    def backward(ctx, dz):
        x, w = ctx.saved_tensors
        st = ctx.st
        cl = torch.channels_last
        dz = dz.contiguous(memory_format=cl)
        n, cin, ih, iw = x.shape
        ks = w.shape[2]
        L = _lib.lib()
        dx = dw = None
        if ctx.needs_input_grad[1]:
            work = torch.empty(int(L.dt_upd_wgrad_work_floats(cin, ks, st, n, ih, iw)),
                               device=x.device)
            dw = torch.empty_like(w)
            rc = L.dt_upd_conv_wgrad(cin, ks, st, n, ih, iw, x.data_ptr(), dz.data_ptr(),
                                     dw.data_ptr(), work.data_ptr(), _stream(x.device))
            if rc != 0:
                raise _lib.DtError('dt_upd_conv_wgrad failed (%d)' % rc)
        if ctx.needs_input_grad[0]:
            if cin != C:    # the observation layer: its input never needs one here
                dx = torch.nn.grad.conv2d_input(x.shape, w, dz, stride=st)
            else:
                dx = torch.empty_like(x)
                rc = L.dt_upd_conv_dgrad(cin, ks, st, n, ih, iw, dz.data_ptr(), w.data_ptr(),
                                         dx.data_ptr(), _stream(x.device))
                if rc != 0:
                    raise _lib.DtError('dt_upd_conv_dgrad failed (%d)' % rc)
        return dx, dw, None


def upd_conv(x, conv):
    """conv(x) without its bias on the dtupd.h kernels (upd_conv_applicable)."""
    return _UpdConv.apply(x, conv.weight, int(conv.stride[0]))


class _ConvBnLeaky(torch.autograd.Function):
    """The whole train-mode block bn(leaky(conv(x) + bias)) on the GPU kernels:
    forward dt_upd_conv_fwd_bn (convolution + the batch statistics in its
    epilogue) and dt_bn_leaky_apply; backward dt_bn_leaky_bwd (BatchNorm,
    LeakyReLU and bias gradients), then the convolution's weight and input
    gradients (dt_upd_conv_wgrad / _dgrad).  Four to five kernels each way
    where MIOpen plus the tail ran eight or more."""

    @staticmethod
    def forward(ctx, x, w, bias, gamma, beta, bn, slope, st):
        cl = torch.channels_last
        x = x.contiguous(memory_format=cl)
        w = w.contiguous(memory_format=cl)
        n, cin, ih, iw = x.shape
        ks = w.shape[2]
        oh, ow = (ih - ks) // st + 1, (iw - ks) // st + 1
        L = _lib.lib()
        z = torch.empty((n, C, oh, ow), device=x.device, dtype=x.dtype, memory_format=cl)
        mi = torch.empty(2 * C, device=x.device)
        nbt = bn.num_batches_tracked
        s = _stream(x.device)
        rc = L.dt_upd_conv_fwd_bn(cin, ks, st, n, ih, iw, x.data_ptr(), w.data_ptr(),
                                  bias.data_ptr(), slope, bn.eps, bn.momentum,
                                  bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                                  nbt.data_ptr() if nbt is not None else None,
                                  int(getattr(bn, '_dt_updates', 1)), z.data_ptr(), mi.data_ptr(),
                                  _work(bn, 'upd', x.device).data_ptr(), _guard(bn), s)
        if rc != 0:
            raise _lib.DtError('dt_upd_conv_fwd_bn failed (%d)' % rc)
        y = torch.empty_like(z)
        rc = L.dt_bn_leaky_apply(z.numel() // C, z.data_ptr(), bias.data_ptr(), slope,
                                 mi.data_ptr(), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), s)
        if rc != 0:
            raise _lib.DtError('dt_bn_leaky_apply failed (%d)' % rc)
        ctx.save_for_backward(x, w, z, bias, mi, gamma)
        ctx.bn, ctx.slope, ctx.st = bn, slope, st
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, z, bias, mi, gamma = ctx.saved_tensors
        cl = torch.channels_last
        dy = dy.contiguous(memory_format=cl)
        L = _lib.lib()
        s = _stream(z.device)
        dz = torch.empty_like(z)
        g = torch.empty(3, C, device=z.device)      # dbias, dgamma, dbeta
        rc = L.dt_bn_leaky_bwd(z.numel() // C, dy.data_ptr(), z.data_ptr(), bias.data_ptr(),
                               mi.data_ptr(), gamma.data_ptr(), ctx.slope, dz.data_ptr(),
                               g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(),
                               _work(ctx.bn, 'bwd', z.device).data_ptr(), _guard(ctx.bn), s)
        if rc != 0:
            raise _lib.DtError('dt_bn_leaky_bwd failed (%d)' % rc)
        n, cin, ih, iw = x.shape
        ks, st = w.shape[2], ctx.st
        dx = dw = None
        if ctx.needs_input_grad[1]:
            work = torch.empty(int(L.dt_upd_wgrad_work_floats(cin, ks, st, n, ih, iw)),
                               device=x.device)
            dw = torch.empty_like(w)
            rc = L.dt_upd_conv_wgrad(cin, ks, st, n, ih, iw, x.data_ptr(), dz.data_ptr(),
                                     dw.data_ptr(), work.data_ptr(), s)
            if rc != 0:
                raise _lib.DtError('dt_upd_conv_wgrad failed (%d)' % rc)
        if ctx.needs_input_grad[0]:
            if cin != C:
                dx = torch.nn.grad.conv2d_input(x.shape, w, dz, stride=st)
            else:
                dx = torch.empty_like(x)
                rc = L.dt_upd_conv_dgrad(cin, ks, st, n, ih, iw, dz.data_ptr(), w.data_ptr(),
                                         dx.data_ptr(), s)
                if rc != 0:
                    raise _lib.DtError('dt_upd_conv_dgrad failed (%d)' % rc)
        return dx, dw, g[0], g[1], g[2], None, None, None


def _bn_handoff(bn, slope, part, parts, m, bias, gamma, beta, mi):
    """include/dtupd.h DtUpdBn for block `bn` (pointers into live tensors)."""
    nbt = bn.num_batches_tracked
    g = getattr(bn, '_dt_guard', None)
    return _lib.DtUpdBn(part.data_ptr(), int(parts), int(m), bias.data_ptr(), gamma.data_ptr(),
                        beta.data_ptr(), float(slope), float(bn.eps), float(bn.momentum),
                        bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                        nbt.data_ptr() if nbt is not None else None,
                        int(getattr(bn, '_dt_updates', 1)), mi.data_ptr(),
                        g.ptr() if g is not None else None)


def _part(bn, dev):
    """Block `bn`'s partials buffer for the chain (a plain attribute)."""
    w = getattr(bn, '_dt_part', None)
    if w is None or w.device != dev:
        w = torch.empty(int(_lib.lib().dt_upd_part_floats()), device=dev)
        bn._dt_part = w
    return w


class _ConvTrunk(torch.autograd.Function):
    """A chain of train-mode blocks bn_j(leaky(conv_j(.) + bias_j)) on the
    include/dtupd.h chain kernels: conv j + 1 merges block j's statistics
    itself and normalises z_j while loading it, so neither a last-arrival
    merge nor y_j (a normalisation pass, a full-size tensor) exists except for
    the last block (dt_upd_bn_finish).  Backward: dt_bn_leaky_bwd per block,
    the weight gradient normalising z_j again while staging
    (dt_upd_conv_wgrad_bn), the input gradient (dt_upd_conv_dgrad).  Outputs,
    running statistics and gradients are the block-by-block path's bit for
    bit (tests/test_gpu_upd_conv.py)."""

    @staticmethod
    def forward(ctx, x, meta, *params):
        bns, slopes, strides = meta
        cl = torch.channels_last
        L = _lib.lib()
        dev = x.device
        s = _stream(dev)
        x = x.contiguous(memory_format=cl)
        ws = [params[4 * j].contiguous(memory_format=cl) for j in range(len(bns))]
        zs, mis = [], []
        prev = None          # the previous block's DtUpdBn
        cur = x
        for j, bn in enumerate(bns):
            bias, gamma, beta = params[4 * j + 1: 4 * j + 4]
            n, cin, ih, iw = cur.shape
            ks, st = ws[j].shape[2], strides[j]
            oh, ow = (ih - ks) // st + 1, (iw - ks) // st + 1
            z = torch.empty((n, C, oh, ow), device=dev, dtype=x.dtype, memory_format=cl)
            part = _part(bn, dev)
            parts = ctypes.c_int32(0)
            rc = L.dt_upd_conv_fwd_part(cin, ks, st, n, ih, iw, cur.data_ptr(),
                                        ctypes.byref(prev) if prev is not None else None,
                                        ws[j].data_ptr(), bias.data_ptr(), slopes[j], z.data_ptr(),
                                        part.data_ptr(), ctypes.byref(parts), s)
            if rc != 0:
                raise _lib.DtError('dt_upd_conv_fwd_part failed (%d)' % rc)
            mi = torch.empty(2 * C, device=dev)
            prev = _bn_handoff(bn, slopes[j], part, parts.value, n * oh * ow, bias, gamma, beta,
                               mi)
            zs.append(z)
            mis.append(mi)
            cur = z
        # y in plain NCHW: the flatten after the trunk is a view, not a copy
        y = torch.empty(cur.shape, device=dev, dtype=cur.dtype)
        rc = L.dt_upd_bn_finish(cur.numel() // C, cur.shape[2] * cur.shape[3], cur.data_ptr(),
                                ctypes.byref(prev), y.data_ptr(), s)
        if rc != 0:
            raise _lib.DtError('dt_upd_bn_finish failed (%d)' % rc)
        ctx.save_for_backward(x, *ws, *zs, *mis, *params)
        ctx.meta, ctx.k = meta, len(bns)
        return y

    @staticmethod
    def backward(ctx, dy):
        bns, slopes, strides = ctx.meta
        k = ctx.k
        saved = ctx.saved_tensors
        x, ws, zs, mis, params = (saved[0], saved[1:1 + k], saved[1 + k:1 + 2 * k],
                                  saved[1 + 2 * k:1 + 3 * k], saved[1 + 3 * k:])
        cl = torch.channels_last
        L = _lib.lib()
        dev = x.device
        s = _stream(dev)
        grads = [None] * (4 * k)
        dx = None
        dyj = dy.contiguous(memory_format=cl)
        for j in range(k - 1, -1, -1):
            bias, gamma, beta = params[4 * j + 1: 4 * j + 4]
            z = zs[j]
            dz = torch.empty_like(z)
            g = torch.empty(3, C, device=dev)      # dbias, dgamma, dbeta
            rc = L.dt_bn_leaky_bwd(z.numel() // C, dyj.data_ptr(), z.data_ptr(), bias.data_ptr(),
                                   mis[j].data_ptr(), gamma.data_ptr(), slopes[j], dz.data_ptr(),
                                   g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(),
                                   _work(bns[j], 'bwd', dev).data_ptr(), _guard(bns[j]), s)
            if rc != 0:
                raise _lib.DtError('dt_bn_leaky_bwd failed (%d)' % rc)
            grads[4 * j + 1], grads[4 * j + 2], grads[4 * j + 3] = g[0], g[1], g[2]
            xin = x if j == 0 else zs[j - 1]
            n, cin, ih, iw = xin.shape
            w, st = ws[j], strides[j]
            ks = w.shape[2]
            hand = None
            if j > 0:
                pb, pg, pbt = params[4 * j - 3: 4 * j]
                hand = _bn_handoff(bns[j - 1], slopes[j - 1], _part(bns[j - 1], dev), 1, 1, pb,
                                   pg, pbt, mis[j - 1])
            if ctx.needs_input_grad[2 + 4 * j]:
                work = torch.empty(int(L.dt_upd_wgrad_work_floats(cin, ks, st, n, ih, iw)),
                                   device=dev)
                dw = torch.empty_like(w)
                rc = L.dt_upd_conv_wgrad_bn(cin, ks, st, n, ih, iw, xin.data_ptr(),
                                            ctypes.byref(hand) if hand is not None else None,
                                            dz.data_ptr(), dw.data_ptr(), work.data_ptr(), s)
                if rc != 0:
                    raise _lib.DtError('dt_upd_conv_wgrad_bn failed (%d)' % rc)
                grads[4 * j] = dw
            if j > 0:
                dyj = torch.empty_like(xin)
                rc = L.dt_upd_conv_dgrad(cin, ks, st, n, ih, iw, dz.data_ptr(), w.data_ptr(),
                                         dyj.data_ptr(), s)
                if rc != 0:
                    raise _lib.DtError('dt_upd_conv_dgrad failed (%d)' % rc)
            elif ctx.needs_input_grad[0]:
                dx = torch.nn.grad.conv2d_input(x.shape, w, dz, stride=st)
        return (dx, None) + tuple(grads)


# the chain kernels for runs of >= 2 blocks (False: block by block, for A/B runs)
CHAIN = True


def trunk_len(x, mods, i, k):
    """How many consecutive train-mode blocks (conv, LeakyReLU, BatchNorm) of
    mods[i:k], starting at mods[i] with input shape x.shape, the chain kernels
    take (0 or >= 2): every conv one of include/dtupd.h's layers, every block
    fused-tail applicable."""
    if not (CHAIN and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4):
        return 0
    shape = tuple(x.shape)
    j = i
    while j + 2 < k:
        conv, act, bn = mods[j], mods[j + 1], mods[j + 2]
        c = getattr(conv, 'kernel', None)
        if c is None or not isinstance(bn, nn.BatchNorm2d) or not isinstance(act, nn.LeakyReLU):
            break
        if not applicable(x, c, act, bn):
            break
        w = c.weight
        st = c.stride[0]
        if (c.stride[0] != c.stride[1] or w.shape[2] != w.shape[3] or w.shape[1] != shape[1]
                or (shape[1], w.shape[2], st, shape[2], shape[3]) not in UPD_CONV_LAYERS):
            break
        ks = w.shape[2]
        shape = (shape[0], C, (shape[2] - ks) // st + 1, (shape[3] - ks) // st + 1)
        j += 3
    blocks = (j - i) // 3
    return blocks if blocks >= 2 else 0


def conv_trunk(x, mods, i, blocks):
    """The chain of `blocks` blocks starting at mods[i] (trunk_len) on x."""
    convs = [mods[i + 3 * b].kernel for b in range(blocks)]
    acts = [mods[i + 3 * b + 1] for b in range(blocks)]
    bns = [mods[i + 3 * b + 2] for b in range(blocks)]
    meta = (bns, [float(a.negative_slope) for a in acts], [int(c.stride[0]) for c in convs])
    params = []
    for c, bn in zip(convs, bns):
        params += [c.weight, c.bias, bn.weight, bn.bias]
    return _ConvTrunk.apply(x, meta, *params)


def conv_leaky_bn(x, conv, act, bn):
    """bn(act(conv(x))) for a train-mode block (see the module docstring)."""
    if upd_conv_applicable(x, conv):
        return _ConvBnLeaky.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, bn,
                                  float(act.negative_slope), int(conv.stride[0]))
    z = F.conv2d(x, conv.weight, None, conv.stride)
    z = z.contiguous(memory_format=torch.channels_last)
    return _BnLeaky.apply(z, conv.bias, bn.weight, bn.bias, bn, float(act.negative_slope))


# nn.Linear layers on include/dtupd.h's split-K kernels: long K (the 4032-wide
# flatten of the conv trunk), N a multiple of 32, float32 on the GPU
LINEAR_MIN_K = 1024


def linear_applicable(x, lin):
    w = lin.weight
    return (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 2
            and x.shape[1] == w.shape[1] and w.shape[1] >= LINEAR_MIN_K and w.shape[1] % 32 == 0
            and w.shape[0] % 32 == 0 and lin.bias is not None)


class _UpdLinear(torch.autograd.Function):
    """y = x w^T + b (torch.nn.Linear), optionally through the following
    LeakyReLU (slope not None) and after a dropout folded in (u: uniforms,
    p: the rate; include/dtupd.h *_drop), with K split over waves and summed
    in a fixed order; backward dx and dw / db on their own MFMA kernels, the
    LeakyReLU's gradient taken from the saved output, the dropout mask
    re-read from u.  Where the library GEMM took one tile a workgroup over all
    of K at batch 64."""

    @staticmethod
    def forward(ctx, x, w, b, slope, u, p, grads):
        x = x.contiguous()
        w = w.contiguous()
        m, k = x.shape
        n = w.shape[0]
        L = _lib.lib()
        y = torch.empty(m, n, device=x.device, dtype=x.dtype)
        work = torch.empty(int(L.dt_upd_linear_work_floats(m, n, k)), device=x.device)
        act = slope is not None
        # the dropped input for the weight gradient (written by the forward)
        # (grads: autograd is recording -- Function.forward itself runs with it off)
        want = grads and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        xd = torch.empty_like(x) if (u is not None and want) else None
        rc = L.dt_upd_linear_fwd_drop(m, n, k, x.data_ptr(), u.data_ptr() if u is not None else None,
                                      float(p), xd.data_ptr() if xd is not None else None,
                                      w.data_ptr(), b.data_ptr(), int(act),
                                      float(slope) if act else 0.0, y.data_ptr(), work.data_ptr(),
                                      _stream(x.device))
        if rc != 0:
            raise _lib.DtError('dt_upd_linear_fwd_drop failed (%d)' % rc)
        ctx.save_for_backward(x if u is None else xd, w, y if act else None, u)
        ctx.slope, ctx.p = slope, float(p)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, w, yv, u = ctx.saved_tensors
        yact = yv.data_ptr() if yv is not None else None
        up = u.data_ptr() if u is not None else None
        slope = float(ctx.slope) if ctx.slope is not None else 0.0
        dy = dy.contiguous()
        m, k = dy.shape[0], w.shape[1]
        n = w.shape[0]
        L = _lib.lib()
        s = _stream(dy.device)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(m, k, device=dy.device, dtype=dy.dtype)
            rc = L.dt_upd_linear_dgrad_drop(m, n, k, dy.data_ptr(), w.data_ptr(), yact, slope, up,
                                            ctx.p, dx.data_ptr(), s)
            if rc != 0:
                raise _lib.DtError('dt_upd_linear_dgrad_drop failed (%d)' % rc)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            dw = torch.empty_like(w)
            db = torch.empty(n, device=dy.device, dtype=dy.dtype)
            # xs: the input, or with a dropout the dropped input the forward wrote
            rc = L.dt_upd_linear_wgrad(m, n, k, dy.data_ptr(), xs.data_ptr(), yact, slope,
                                       dw.data_ptr(), db.data_ptr(), s)
            if rc != 0:
                raise _lib.DtError('dt_upd_linear_wgrad failed (%d)' % rc)
        return dx, dw, db, None, None, None, None


# The dropout uniforms of one update drawn in ONE launch: the trainer opens a
# pool of `sites` [m, k] slices (drop_pool) before its stages and every folded
# dropout takes the next slice; outside a pool (or past its end) a site draws
# its own torch.rand.  The slices are static tensors, so a captured graph
# replays the single draw (graph-safe Philox offsets) and the sites read it.
_DROP = {'pool': None, 'next': 0}
FOLD_DROPOUT = True   # fold a dropout into the linear after it (A/B switch, tools/update_only.py)


@contextlib.contextmanager
def drop_pool(sites, m, k, device):
    pool = torch.rand(sites, m, k, device=device)
    saved = dict(_DROP)
    _DROP['pool'], _DROP['next'] = pool, 0
    try:
        yield pool
    finally:
        _DROP.update(saved)


def drop_uniforms(x):
    pool, i = _DROP['pool'], _DROP['next']
    if (pool is not None and i < pool.shape[0] and tuple(pool.shape[1:]) == tuple(x.shape)
            and pool.device == x.device):
        _DROP['next'] = i + 1
        return pool[i]
    return torch.rand(x.shape, device=x.device, dtype=torch.float32)


def linear(x, lin, slope=None, drop=0.0):
    """lin(x), then LeakyReLU(slope) if slope is not None, on the dtupd.h
    kernels (linear_applicable); drop > 0: F.dropout(x, drop) folded in
    (uniforms from drop_uniforms)."""
    u = drop_uniforms(x) if drop > 0.0 else None
    return _UpdLinear.apply(x, lin.weight, lin.bias, slope, u, float(drop) if drop > 0.0 else 0.0,
                            torch.is_grad_enabled())


# ---- the small fully connected tails after the trunk's linear (include/dthead.h) --------
MLP_ACT = {'none': 0, 'leaky': 1, 'tanh': 2, 'sigmoid': 3}


def _act_code(m):
    if m is None:
        return 0, None
    if isinstance(m, nn.LeakyReLU):
        return (1, float(m.negative_slope)) if m.negative_slope >= 0 else (None, None)
    if isinstance(m, nn.Tanh):
        return 2, None
    if isinstance(m, nn.Sigmoid):
        return 3, None
    return None, None


def mlp_plan(seq, parts):
    """(w1, b1, act1, w2, b2, act2, slope) when the output branch `seq`
    (config.json's output MetaNet: linear [-> act] [-> linear [-> act]]) on the
    concatenation of `parts` fits dt_mlp_fwd; None otherwise (torch runs it)."""
    mods = list(seq.internal_modules)
    if not mods or not all(p.is_cuda and p.dtype == torch.float32 and p.dim() == 2 for p in parts):
        return None
    if len(parts) not in (1, 2) or any(p.shape[0] != parts[0].shape[0] for p in parts):
        return None
    lins, acts, i = [], [], 0
    while i < len(mods):
        lin = getattr(mods[i], 'linear', None)
        if lin is None or len(lins) == 2:
            return None
        act = mods[i + 1] if i + 1 < len(mods) and getattr(mods[i + 1], 'linear', None) is None \
            else None
        code, slope = _act_code(act)
        if code is None:
            return None
        lins.append(lin)
        acts.append((code, slope))
        i += 2 if act is not None else 1
    slopes = {s for _, s in acts if s is not None}
    if len(slopes) > 1:
        return None
    m, k = parts[0].shape[0], sum(p.shape[1] for p in parts)
    n1 = lins[0].out_features
    n2 = lins[1].out_features if len(lins) == 2 else 0
    if (lins[0].in_features != k or (n2 and lins[1].in_features != n1) or m > 256 or k > 1024
            or n1 > (512 if n2 else 1024) or n2 > 64 or m * n1 > 8192 or m * n2 > 2048
            or n2 * n1 > 4096
            or any(l.weight.dtype != torch.float32 or not l.weight.is_cuda for l in lins)):
        return None
    slope = slopes.pop() if slopes else 0.0
    w2, b2 = (lins[1].weight, lins[1].bias) if n2 else (None, None)
    return (lins[0].weight, lins[0].bias, acts[0][0], w2, b2, acts[1][0] if n2 else 0, slope)


def _mlp_struct(x0, x1, w1, b1, w2, b2, act1, act2, slope):
    ptr = (lambda t: t.data_ptr() if t is not None else None)
    return _lib.DtMlp(x0.shape[0], x0.shape[1], x1.shape[1] if x1 is not None else 0,
                      w1.shape[0], w2.shape[0] if w2 is not None else 0, act1, act2, slope,
                      w1.data_ptr(), ptr(b1), ptr(w2), ptr(b2))


class _Mlp(torch.autograd.Function):
    """The output branch on [x0 | x1] in one dt_mlp_fwd launch; backward in one
    dt_mlp_bwd launch (only the gradients autograd asks for)."""

    @staticmethod
    def forward(ctx, x0, x1, w1, b1, w2, b2, meta):
        act1, act2, slope = meta
        x0 = x0.contiguous()
        x1 = x1.contiguous() if x1 is not None else None
        w1 = w1.contiguous()
        w2 = w2.contiguous() if w2 is not None else None
        p = _mlp_struct(x0, x1, w1, b1, w2, b2, act1, act2, slope)
        h = torch.empty(p.m, p.n1, device=x0.device)
        y = torch.empty(p.m, p.n2, device=x0.device) if p.n2 else None
        rc = _lib.lib().dt_mlp_fwd(ctypes.byref(p), x0.data_ptr(),
                                   x1.data_ptr() if x1 is not None else None, h.data_ptr(),
                                   y.data_ptr() if y is not None else None,
                                   torch.cuda.current_stream(x0.device).cuda_stream)
        if rc != 0:
            raise _lib.DtError('dt_mlp_fwd failed (%d)' % rc)
        ctx.meta = meta
        ctx.has = (x1 is not None, b1 is not None, w2 is not None, b2 is not None)
        ctx.save_for_backward(x0, x1, w1, b1, w2, b2, h, y)
        return y if y is not None else h

    @staticmethod
    def backward(ctx, dy):
        x0, x1, w1, b1, w2, b2, h, y = ctx.saved_tensors
        act1, act2, slope = ctx.meta
        need = ctx.needs_input_grad
        dy = dy.contiguous()
        new = (lambda t, want: torch.empty_like(t) if (want and t is not None) else None)
        dx0, dx1 = new(x0, need[0]), new(x1, need[1])
        dw1, db1 = new(w1, need[2]), new(b1, need[3])
        dw2, db2 = new(w2, need[4]), new(b2, need[5])
        p = _mlp_struct(x0, x1, w1, b1, w2, b2, act1, act2, slope)
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        rc = _lib.lib().dt_mlp_bwd(ctypes.byref(p), x0.data_ptr(), ptr(x1), h.data_ptr(), ptr(y),
                                   dy.data_ptr(), ptr(dx0), ptr(dx1), ptr(dw1), ptr(db1),
                                   ptr(dw2), ptr(db2),
                                   torch.cuda.current_stream(dy.device).cuda_stream)
        if rc != 0:
            raise _lib.DtError('dt_mlp_bwd failed (%d)' % rc)
        return dx0, dx1, dw1, db1, dw2, db2, None


def mlp(parts, plan):
    """The output branch of mlp_plan on `parts` (1 or 2 [m, k] tensors)."""
    w1, b1, act1, w2, b2, act2, slope = plan
    x1 = parts[1] if len(parts) == 2 else None
    return _Mlp.apply(parts[0], x1, w1, b1, w2, b2, (act1, act2, slope))


def td_applicable(parts, rew, notdone):
    m = parts[0].shape[0]
    return all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == m
               for t in (rew, notdone))


@torch.no_grad()
def mlp_td(parts, plan, rew, notdone, gamma):
    """The output branch of mlp_plan on `parts` and the TD target
    rew + (notdone * gamma) * y in one dt_mlp_fwd_td launch; returns the
    target [m, n_out] (no autograd: the target networks' pass)."""
    w1, b1, act1, w2, b2, act2, slope = plan
    x0 = parts[0].contiguous()
    x1 = parts[1].contiguous() if len(parts) == 2 else None
    p = _mlp_struct(x0, x1, w1.contiguous(), b1, w2.contiguous() if w2 is not None else None, b2,
                    act1, act2, slope)
    dev = x0.device
    h = torch.empty(p.m, p.n1, device=dev)
    y = torch.empty(p.m, p.n2, device=dev) if p.n2 else None
    target = torch.empty(p.m, p.n2 or p.n1, device=dev)
    rc = _lib.lib().dt_mlp_fwd_td(ctypes.byref(p), x0.data_ptr(),
                                  x1.data_ptr() if x1 is not None else None, h.data_ptr(),
                                  y.data_ptr() if y is not None else None, rew.data_ptr(),
                                  notdone.data_ptr(), float(gamma), target.data_ptr(),
                                  torch.cuda.current_stream(dev).cuda_stream)
    if rc != 0:
        raise _lib.DtError('dt_mlp_fwd_td failed (%d)' % rc)
    return target


# ---- the DDPG losses (include/dthead.h dt_loss) ------------------------------------------
class _Loss(torch.autograd.Function):
    """kind 0: F.mse_loss(a, b) (mean); kind 1: -mean(a).  One launch forward,
    one backward (gradient for `a` only: b is the detached target)."""

    @staticmethod
    def forward(ctx, a, b, kind):
        a = a.contiguous()
        b = b.contiguous() if b is not None else None
        loss = torch.empty((), device=a.device)
        rc = _lib.lib().dt_loss(kind, a.numel(), a.data_ptr(),
                                b.data_ptr() if b is not None else None, loss.data_ptr(),
                                torch.cuda.current_stream(a.device).cuda_stream)
        if rc != 0:
            raise _lib.DtError('dt_loss failed (%d)' % rc)
        ctx.kind = kind
        ctx.save_for_backward(a, b)
        return loss

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous()
        da = torch.empty_like(a)
        rc = _lib.lib().dt_loss_bwd(ctx.kind, a.numel(), a.data_ptr(),
                                    b.data_ptr() if b is not None else None, g.data_ptr(),
                                    da.data_ptr(), torch.cuda.current_stream(a.device).cuda_stream)
        if rc != 0:
            raise _lib.DtError('dt_loss_bwd failed (%d)' % rc)
        return da, None, None


def _loss_applicable(*ts):
    """The fused loss kernels take float32 GPU tensors of ONE shape: F.mse_loss
    broadcasts [m] against [m, 1] to [m, m], which an element-wise kernel over
    equal numel would silently not do."""
    return all(t.is_cuda and t.dtype == torch.float32 for t in ts) and \
        len({tuple(t.shape) for t in ts}) == 1


def mse_loss(a, b):
    """F.mse_loss(a, b) (b without gradient) in one launch each way on the GPU."""
    if _loss_applicable(a, b) and not b.requires_grad:
        return _Loss.apply(a, b.detach(), 0)
    return F.mse_loss(a, b)


def neg_mean(a):
    """-1.0 * torch.mean(a) (the actor loss) in one launch each way on the GPU."""
    if _loss_applicable(a):
        return _Loss.apply(a, None, 1)
    return -1.0 * torch.mean(a)
