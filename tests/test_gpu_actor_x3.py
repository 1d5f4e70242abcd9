"""The float32-accurate actor convolutions on fp16 MFMA (dt_conv1x_split /
dt_conv32x_split, include/dtactor.h; aido1_amd/csrc/dtconvx.hip) against
float64 restatements of each layer, and the whole reference-mode float32
FusedActor against the float64 actor (bench.actor_f64) on rendered frames:
the reference acts in float32 (models/ddpg/model.py:79-88,
duckietown_rl/ddpg.py:44-62), and the bar is |da| <= 1e-4."""
import ctypes
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from formulas import formula_state_dict  # noqa: E402

pytestmark = pytest.mark.gpu


def stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize('index,slots,order,n', [(True, 3, [0, 1, 2], 37), (True, 4, [2, 3, 0], 600),
                                                 (False, 4, [1, 2, 3], 300), (True, 3, [1, 0, 2], 1)])
def test_conv1x_matches_float64(gpu, index, slots, order, n):
    """conv1 + bias + LeakyReLU from the ring (palette-index or grey) vs a
    float64 conv2d of the same frames and weights: the stored (hi, lo) pairs
    plus the centre carry the f64 result to f32 rounding; the per-sample
    statistics (mean of the centred values, M2) likewise."""
    from aido1_amd import _lib
    from aido1_amd.actor import conv1_fragments, hlb_decode, hlb_shape, split_hl
    from aido1_amd.render import decode_index
    L = _lib.lib()
    torch.manual_seed(n + slots)
    if index:
        ring = torch.randint(0, 8, (n, slots, 120, 160), dtype=torch.uint8, device=gpu)
        grey = decode_index(ring)
    else:
        ring = grey = torch.rand(n, slots, 120, 160, device=gpu)
    w = torch.randn(32, 3, 8, 8, device=gpu) * 0.08
    b = torch.randn(32, device=gpu) * 0.2
    ref = F.leaky_relu(F.conv2d(grey[:, order].double(), w.double(), b.double(), stride=2))
    wf = split_hl(conv1_fragments(w, torch.float32)).contiguous()
    y = torch.empty(hlb_shape(n, 57, 77, 2), dtype=torch.float16, device=gpu)
    part = torch.empty(n, 32, 3, device=gpu)
    o = (ctypes.c_int32 * 3)(*order)
    assert L.dt_conv1x_split(ring.data_ptr(), int(index), n, slots, o, wf.data_ptr(),
                             b.data_ptr(), None, y.data_ptr(), part.data_ptr(), 0.01,
                             stream()) == 0
    c = part[..., 2].double()
    scale = max(1.0, ref.abs().max().item())
    assert (c - ref[:, :, 0, 0]).abs().max().item() < 2e-6 * scale
    got = hlb_decode(y, 57, 77, 2).permute(0, 3, 1, 2) + c[:, :, None, None]
    err = (got - ref).abs().max().item()
    assert err < 2e-6 * scale, err
    mean = ref.mean((2, 3))
    m2 = ((ref - mean[:, :, None, None]) ** 2).sum((2, 3))
    assert torch.allclose(part[..., 0].double() + c, mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(part[..., 1].double(), m2, rtol=1e-4, atol=1e-4)


def _layer_case(gpu, layer, n, seed):
    """A conv2..4 case: HLB input (centred-like values) with its exact
    per-sample statistics, BatchNorm parameters, weights; the float64
    reference of the BatchNorm'd input's conv + LeakyReLU."""
    from aido1_amd.actor import hlb_decode, hlb_encode
    shape, stride = {2: ((57, 77), 2), 3: ((27, 37), 2), 4: ((12, 17), 1)}[layer]
    g = torch.Generator(device=gpu).manual_seed(seed)
    ih, iw = shape
    # per-sample channel offsets and spreads, some channels nearly flat
    spread = torch.exp(torch.randn(n, 1, 1, 32, device=gpu, generator=g) * 2.0)
    x = torch.randn(n, ih, iw, 32, device=gpu, generator=g) * spread + \
        torch.randn(n, 1, 1, 32, device=gpu, generator=g) * spread
    xh = hlb_encode(x, stride)
    xt = hlb_decode(xh, ih, iw, stride)                  # the values the kernel sees
    mean = xt.mean((1, 2))
    m2 = ((xt - mean[:, None, None, :]) ** 2).sum((1, 2))
    prev = torch.stack([mean.float(), m2.float(), torch.zeros_like(mean).float()], -1).contiguous()
    gamma = torch.rand(32, device=gpu, generator=g) + 0.5
    beta = torch.rand(32, device=gpu, generator=g) - 0.5
    w = torch.randn(32, 32, 4, 4, device=gpu, generator=g) * 0.05
    b = torch.randn(32, device=gpu, generator=g) * 0.1
    pm, pv = prev[..., 0].double(), prev[..., 1].double() / (ih * iw)
    xn = (xt - pm[:, None, None, :]) / torch.sqrt(pv[:, None, None, :] + 1e-5) * \
        gamma.double() + beta.double()
    ref = F.leaky_relu(F.conv2d(xn.permute(0, 3, 1, 2), w.double(), b.double(), stride=stride))
    return xh, prev, gamma, beta, w, b, ref


@pytest.mark.parametrize('n', [7, 700])
@pytest.mark.parametrize('layer', [2, 3, 4])
def test_conv32x_layers_match_float64(gpu, layer, n):
    """conv2..conv4 with the previous per-sample BatchNorm folded into the
    weights vs float64: layers 2 / 3 write centred HLB pairs and their
    statistics, layer 4 its own BatchNorm's output flattened NCHW in f32.
    Some input channels are nearly flat (spreads e^(2 N(0,1))), the case the
    per-sample norm amplifies.  n = 700 exceeds the resident grid."""
    from aido1_amd import _lib
    from aido1_amd.actor import conv32_fragments, hlb_decode, hlb_shape
    L = _lib.lib()
    xh, prev, gamma, beta, w, b, ref = _layer_case(gpu, layer, n, 10 * layer + n)
    oh, ow = ref.shape[2:]
    wf = conv32_fragments(w, torch.float32)
    g4 = (torch.rand(32, device=gpu) + 0.5) if layer == 4 else None
    b4 = (torch.rand(32, device=gpu) - 0.5) if layer == 4 else None
    if layer == 4:
        y = torch.empty(n, 32 * oh * ow, device=gpu)
        part = None
    else:
        y = torch.empty(hlb_shape(n, oh, ow, 2 if layer == 2 else 1), dtype=torch.float16,
                        device=gpu)
        part = torch.empty(n, 32, 3, device=gpu)
    ptr = (lambda t: t.data_ptr() if t is not None else None)
    assert L.dt_conv32x_split(layer, n, xh.data_ptr(), wf.data_ptr(), b.data_ptr(),
                              prev.data_ptr(), gamma.data_ptr(), beta.data_ptr(), 1e-5,
                              y.data_ptr(), ptr(part), ptr(g4), ptr(b4), 1e-5, 0.01, None,
                              stream()) == 0
    if layer == 4:
        m = ref.mean((2, 3), keepdim=True)
        v = ((ref - m) ** 2).mean((2, 3), keepdim=True)
        want = ((ref - m) / torch.sqrt(v + 1e-5) * g4.double().view(1, -1, 1, 1) +
                b4.double().view(1, -1, 1, 1)).flatten(1)
        err = (y.double() - want).abs().max().item()
        assert err < 2e-5 * max(1.0, want.abs().max().item()), err
        return
    c = part[..., 2].double()
    scale = max(1.0, ref.abs().max().item())
    got = hlb_decode(y, oh, ow, 2 if layer == 2 else 1).permute(0, 3, 1, 2) + \
        c[:, :, None, None]
    err = (got - ref).abs().max().item()
    assert err < 1e-5 * scale, err
    mean = ref.mean((2, 3))
    m2 = ((ref - mean[:, :, None, None]) ** 2).sum((2, 3))
    assert torch.allclose(part[..., 0].double() + c, mean, rtol=1e-5, atol=1e-5 * scale)
    assert torch.allclose(part[..., 1].double(), m2, rtol=1e-4, atol=1e-4 * scale)


@pytest.mark.parametrize('n,n0', [(600, 525), (97, 1), (4096, 3584)])
def test_x3_split_launch_matches_separate_actors(gpu, n, n0):
    """One launch per convolution over two weight sets (the exploring /
    exploiting explorers, config.json:183-186) gives every sample bit for bit
    what a launch with its own set gives."""
    from aido1_amd.actor import ConfigActor, FusedActor
    cfg = golden('reference_config.json')['model']['actor']
    torch.manual_seed(17)
    fa = FusedActor(ConfigActor(cfg).to(gpu), dtype=torch.float32, mode='reference')
    fb = FusedActor(ConfigActor(cfg).to(gpu), dtype=torch.float32, mode='reference')
    with torch.no_grad():
        for f in (fa, fb):
            for p in list(f.gamma) + list(f.beta):
                p.uniform_(0.5, 1.5)
    g = torch.Generator(device=gpu).manual_seed(n)
    ring = torch.randint(0, 8, (n, 3, 120, 160), dtype=torch.uint8, device=gpu, generator=g)
    order = [2, 0, 1]
    flat = fa._convs_x3(ring, order, fb, n0).clone()
    assert torch.equal(flat[:n0], fa._convs_x3(ring[:n0].contiguous(), order))
    assert torch.equal(flat[n0:], fb._convs_x3(ring[n0:].contiguous(), order))
    fa.p_drop = fb.p_drop = 0.0
    out = fa.forward_pair(fb, ring, order, n0)
    ref = torch.cat([fa(ring[:n0].contiguous(), order), fb(ring[n0:].contiguous(), order)])
    assert torch.equal(out, ref)


def test_x3_index_ring_equals_grey_ring(gpu):
    """Palette-index frames give bit for bit what their grey frames give."""
    from aido1_amd.actor import ConfigActor, FusedActor
    from aido1_amd.render import decode_index
    torch.manual_seed(3)
    f = FusedActor(ConfigActor(golden('reference_config.json')['model']['actor']).to(gpu),
                   dtype=torch.float32, mode='reference')
    idx = torch.randint(0, 8, (300, 4, 120, 160), dtype=torch.uint8, device=gpu)
    a = f._convs_x3(idx, [1, 2, 3]).clone()
    assert torch.equal(a, f._convs_x3(decode_index(idx), [1, 2, 3]))


@pytest.mark.parametrize('seed', [1234, 11])
def test_f32_actor_within_1e4_of_float64_on_rendered_frames(gpu, seed):
    """The reference-mode float32 FusedActor (the x3 chain + float32 linears)
    on 1024 envs' live rendered frames vs the float64 actor, dropout off:
    max |da| <= 1e-4 on every env (the fp16 fast mode is ~1e-2 here)."""
    from aido1_amd.actor import ConfigActor
    from aido1_amd.rollout import ActorRollout
    from bench import actor_f64
    from test_trainer import no_dropout
    cfg = golden('reference_config.json')
    torch.manual_seed(seed)
    actor = ConfigActor(no_dropout(cfg['model']['actor'])).to(gpu)
    roll = ActorRollout(cfg, 1024, maps=('small_loop', 'zigzag'), device=0, seed=seed,
                        actor=actor, dtype=torch.float32)
    assert roll.actor.x3
    roll.reset()
    for _ in range(6):
        roll.step()
    got = roll.actor(roll.ring, roll.order()).double().cpu()
    ref = actor_f64(actor, roll.stack(), 'reference', device=gpu)
    err = (got - ref).abs().max().item()
    roll.close()
    assert torch.isfinite(got).all()
    assert err <= 1e-4, err


def test_f32_actor_matches_formula_weights_per_sample(gpu):
    """Formula weights and frames (tests/golden/formulas.py) through the x3
    chain vs the reference modules run one sample at a time in train mode
    (models/ddpg/model.py:74-88) in float64."""
    from aido1_amd.actor import ConfigActor, FusedActor
    from formulas import formula_input
    from test_trainer import no_dropout
    a = ConfigActor(no_dropout(golden('reference_config.json')['model']['actor']))
    a.load_state_dict(formula_state_dict(a.state_dict()))
    a = a.double().train()
    x = formula_input(4)
    with torch.no_grad():
        ref = torch.cat([a(x[i:i + 1].double()) for i in range(4)])
    f = FusedActor(a.float().to(gpu), dtype=torch.float32, mode='reference')
    got = f(x.to(gpu).contiguous()).double().cpu()
    assert (got - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize('n,n0', [(300, 300), (300, 257), (4096, 3584), (33, 1)])
def test_head_x3_matches_float64(gpu, n, n0):
    """dt_actor_head_x3 (lin1 on x3 MFMA, LeakyReLU, lin2, tanh in one launch
    over both weight sets) vs float64 on the same inputs, dropout off."""
    from aido1_amd.actor import FLAT, ConfigActor, FusedActor
    from test_trainer import no_dropout
    cfg = no_dropout(golden('reference_config.json')['model']['actor'])
    torch.manual_seed(n + n0)
    a, b = ConfigActor(cfg).to(gpu), ConfigActor(cfg).to(gpu)
    fa = FusedActor(a, dtype=torch.float32, mode='reference')
    fb = FusedActor(b, dtype=torch.float32, mode='reference')
    assert fa._head_x3_ok(torch.zeros(1, FLAT, device=gpu), fb)
    x = torch.randn(n, FLAT, device=gpu) * 0.7
    out = torch.full((n, 2), float('nan'), device=gpu)
    fa._heads_x3(fb, x, n0, out)
    want = []
    for net, sl in ((a, slice(0, n0)), (b, slice(n0, n))):
        _, _, l1, l2 = net.layers()
        h = F.leaky_relu(x[sl].double() @ l1.weight.double().t() + l1.bias.double())
        want.append(torch.tanh(h @ l2.weight.double().t() + l2.bias.double()))
    want = torch.cat(want)
    assert torch.isfinite(out).all()
    assert (out.double() - want).abs().max().item() < 2e-6


def _drop_hash(x):
    x = x.astype(np.uint64) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def _drop_uniforms(n, k, seed):
    """dt_actor_head_x3_drop's uniforms restated: one two-round hash a pair of
    elements keyed by the seed, 16 bits each (csrc/dtconvx.hip drop_hash)."""
    idx = np.arange(n * k, dtype=np.uint64).reshape(n, k)
    pair = idx[:, 0::2]
    mix = _drop_hash(np.array([seed ^ 0x9E3779B9], dtype=np.uint64))[0]
    hh = _drop_hash((_drop_hash(pair ^ mix) + seed) & 0xFFFFFFFF)
    u = np.empty((n, k))
    u[:, 0::2] = (hh & 0xFFFF) / 65536.0
    u[:, 1::2] = (hh >> 16) / 65536.0
    return u


@pytest.mark.parametrize('n,n0,p,seed', [(300, 257, 0.5, 12345), (64, 64, 0.25, 7)])
def test_head_x3_dropout_folded(gpu, n, n0, p, seed):
    """The dropout folded into lin1's staging (dt_actor_head_x3_drop) against
    float64 of F.dropout with the kernel's mask restated in numpy: every
    element kept where u >= p, scaled by 1 / (1 - p); about 1 - p of them."""
    import ctypes

    from aido1_amd import _lib
    from aido1_amd.actor import FLAT, ConfigActor, FusedActor
    cfg = golden('reference_config.json')['model']['actor']
    torch.manual_seed(n + seed)
    a, b = ConfigActor(cfg).to(gpu), ConfigActor(cfg).to(gpu)
    fa = FusedActor(a, dtype=torch.float32, mode='reference')
    fb = FusedActor(b, dtype=torch.float32, mode='reference')
    x = torch.randn(n, FLAT, device=gpu) * 0.7
    out = torch.full((n, 2), float('nan'), device=gpu)
    L = _lib.lib()
    work = torch.empty(int(L.dt_actor_head_x3_work_floats(n)), device=gpu)
    rc = L.dt_actor_head_x3_drop(
        n, n0, FLAT, x.data_ptr(), p, seed, fa.w1x.data_ptr(), fa.b1.data_ptr(),
        fa.w2.data_ptr(), fa.b2.data_ptr(), fb.w1x.data_ptr(), fb.b1.data_ptr(),
        fb.w2.data_ptr(), fb.b2.data_ptr(), fa._HEAD_CODES[fa.head], 0.01, work.data_ptr(),
        out.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream))
    assert rc == 0
    keep = torch.from_numpy(_drop_uniforms(n, FLAT, seed) >= p)
    assert abs(keep.double().mean().item() - (1 - p)) < 0.01
    xd = x.double().cpu() * keep / (1.0 - p)
    want = []
    for net, sl in ((a, slice(0, n0)), (b, slice(n0, n))):
        _, _, l1, l2 = net.layers()
        h = F.leaky_relu(xd[sl] @ l1.weight.double().cpu().t() + l1.bias.double().cpu())
        want.append(torch.tanh(h @ l2.weight.double().cpu().t() + l2.bias.double().cpu()))
    want = torch.cat(want)
    assert torch.isfinite(out).all()
    assert (out.double().cpu() - want).abs().max().item() < 4e-6
