"""Which layer's fp16 rounding sets the reference-mode actor's action error:
the f32 path (MIOpen f32 convs, per-sample BatchNorm) with ONE stage's fp16
effects emulated at a time -- its conv input (post-BatchNorm values) and
weights rounded to fp16 (the MFMA operands), its output stored in fp16 the
way the HIP chain stores it (LeakyReLU output centred on pixel 0) -- on live
frames of 4096 envs, two weight seeds.  Also all stages at once, and the
real HIP chain, for comparison.  usage: python tools/actor_layer_error.py"""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, 'tests')
from conftest import golden  # noqa: E402
from aido1_amd.actor import ConfigActor, FusedActor, apply_head  # noqa: E402
from aido1_amd.rollout import ActorRollout  # noqa: E402

dev = torch.device('cuda', 0)
cfg = golden('reference_config.json')
roll = ActorRollout(cfg, 4096, device=0, seed=1234, actor_mode='reference',
                    dtype=torch.float16)
roll.reset()
for _ in range(12):
    roll.step()
torch.cuda.synchronize()
stack = roll.stack()
h16 = lambda t: t.half().float()   # noqa: E731


def forward(a, x, emu, parts=('in', 'w', 'out')):
    """emu: set of stages with fp16 effects: 0..3 convs, 'lin1', 'head';
    parts: which effects of conv 0 are emulated (the others get all three)."""
    convs, bns, l1, l2 = a.layers()
    h = x.float().contiguous(memory_format=torch.channels_last)
    for i, (c, b) in enumerate(zip(convs, bns)):
        w = c.weight
        pp = parts if i == 0 else ('in', 'w', 'out')
        if i in emu and 'in' in pp:
            h = h16(h)
        if i in emu and 'w' in pp:
            w = h16(w)
        z = F.leaky_relu(F.conv2d(h, w.contiguous(memory_format=torch.channels_last), c.bias,
                                  stride=c.stride))
        if i in emu and i < 3 and 'out' in pp:     # stored fp16, centred on the sample's pixel 0
            cen = z[:, :, :1, :1]
            z = h16(z - cen) + cen
        m = z.mean((2, 3), keepdim=True)
        v = (z - m).square().mean((2, 3), keepdim=True)
        h = (z - m) / torch.sqrt(v + b.eps) * b.weight.view(1, -1, 1, 1) + b.bias.view(1, -1, 1, 1)
    h = h.contiguous().flatten(1)
    w1 = l1.weight
    if 'lin1' in emu:
        h, w1 = h16(h), h16(w1)
    h = F.linear(h, w1, l1.bias)
    if 'lin1' in emu:
        h = h16(h)
    h = F.leaky_relu(h)
    if 'head' in emu:
        h = h16(h)
    o = F.linear(h, l2.weight if 'head' not in emu else h16(l2.weight), l2.bias)
    if 'head' in emu:
        o = h16(o)
    return apply_head(o, a.head)


with torch.no_grad(), torch.backends.cudnn.flags(enabled=True, benchmark=False,
                                                 deterministic=True, allow_tf32=False):
    for seed in (11, 1234):
        torch.manual_seed(seed)
        actor = ConfigActor(cfg['model']['actor']).to(dev)
        ref = forward(actor, stack, set())
        a16 = FusedActor(actor, dtype=torch.float16, mode='reference')
        a16.p_drop = 0.0
        hip = a16(roll.ring, roll.order())
        print('seed %d: HIP chain max %.3e' % (seed, (hip - ref).abs().max()))
        for emu in ({0}, {1}, {2}, {3}, {'lin1'}, {'head'}, {0, 1, 2, 3, 'lin1', 'head'}):
            e = (forward(actor, stack, emu) - ref).abs()
            print('   emulated %-30s max %.3e p99 %.3e' % (sorted(map(str, emu)), e.max(),
                                                         torch.quantile(e.flatten(), 0.99)))
        for parts in (('in',), ('w',), ('out',)):
            e = (forward(actor, stack, {0}, parts) - ref).abs()
            print('   conv1 only %-12s max %.3e' % (parts, e.max()))
        allbut = {1, 2, 3, 'lin1', 'head'}
        for label, emu, parts in (('conv1 exact weights', allbut | {0}, ('in', 'out')),
                                  ('conv1 exact', allbut, ()),
                                  ('conv1 exact w, lin1+head f32', {0, 1, 2, 3}, ('in', 'out')),
                                  ('convs 1-2 exact weights', {0, 1, 2, 3, 'lin1', 'head'},
                                   ('in', 'out'))):
            e = (forward(actor, stack, emu, parts) - ref).abs()
            print('   %-34s max %.3e p99 %.3e' % (label, e.max(),
                                                  torch.quantile(e.flatten(), 0.99)))
        # per-sample BatchNorm amplification: the smallest std of each conv's output
        convs, bns, _, _ = actor.layers()
        h = stack.float().contiguous(memory_format=torch.channels_last)
        for i, (c, b) in enumerate(zip(convs, bns)):
            z = F.leaky_relu(F.conv2d(h, c.weight, c.bias, stride=c.stride))
            s = z.std((2, 3), unbiased=False)
            mabs = z.abs().amax((2, 3))
            print('   conv%d out: min std %.3e, min std/max|z| %.3e, median std %.3e' % (
                i + 1, s.min(), (s / mabs.clamp_min(1e-30)).min(), s.median()))
            m = z.mean((2, 3), keepdim=True)
            v = (z - m).square().mean((2, 3), keepdim=True)
            h = (z - m) / torch.sqrt(v + b.eps) * b.weight.view(1, -1, 1, 1) + \
                b.bias.view(1, -1, 1, 1)
