"""Actor in the loop on the GPU: the bf16 BN-folded FusedActor against the fp32
eval-mode actor, ring-order equivalence, and the batched rollout."""
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from formulas import formula_input, formula_state_dict  # noqa: E402

pytestmark = pytest.mark.gpu


def test_fused_bf16_close_to_fp32(gpu):
    from aido1_amd.actor import ConfigActor, FusedActor
    a = ConfigActor(golden('reference_config.json')['model']['actor'])
    a.load_state_dict(formula_state_dict(a.state_dict()))
    a.eval()
    x = formula_input(4)
    with torch.no_grad():
        ref = a(x)
    f = FusedActor(a, dtype=torch.bfloat16).to(gpu)
    y = f(x.to(gpu)).cpu()
    assert torch.max(torch.abs(y - ref)) < 3e-2, (y, ref)
    assert np.max(np.abs(y.numpy() - golden('actor.npz')['config_actor'])) < 3e-2


def test_rollout_runs_and_counts(gpu):
    from aido1_amd.rollout import ActorRollout
    cfg = golden('reference_config.json')
    roll = ActorRollout(cfg, 512, device=0, seed=3)
    roll.reset()
    for _ in range(10):
        r, rm, d = roll.step()
    torch.cuda.synchronize()
    st = roll.stats()
    assert st['decisions'] == 512 * 10
    assert 512 * 10 <= st['sim_steps'] <= 512 * 30
    assert torch.isfinite(r).all() and torch.isfinite(roll.ring).all()
    a = roll.actions
    assert (a.abs() <= 1.0).all()
    roll.close()


@pytest.mark.parametrize('dtype,tol', [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
def test_sample_norm_kernel_matches_two_pass(gpu, dtype, tol):
    """dt_sample_norm (include/dtactor.h) vs a float64 two-pass restatement of
    lrelu -> BatchNorm2d(train) on each sample alone."""
    from aido1_amd.actor import ConfigActor, FusedActor
    f = FusedActor(ConfigActor(golden('reference_config.json')['model']['actor']),
                   dtype=dtype, mode='reference').to(gpu)
    torch.manual_seed(0)
    for i, (h, w) in enumerate([(57, 77), (27, 37), (12, 17), (9, 14)]):
        with torch.no_grad():
            f.gamma[i].uniform_(0.5, 1.5)
            f.beta[i].uniform_(-0.1, 0.1)
        x = (torch.randn(5, 32, h, w, device=gpu) * 2 + 3).to(dtype) \
            .contiguous(memory_format=torch.channels_last)
        xd = torch.nn.functional.leaky_relu(x.double())
        m = xd.mean((2, 3), keepdim=True)
        v = (xd - m).square().mean((2, 3), keepdim=True)
        ref = (xd - m) / torch.sqrt(v + 1e-5) * f.gamma[i].double().view(1, -1, 1, 1) + \
            f.beta[i].double().view(1, -1, 1, 1)
        y = f._lrelu_sample_norm(x.clone(memory_format=torch.channels_last), i)
        err = (y.double() - ref).abs().max().item()
        assert err < tol * max(1.0, ref.abs().max().item()), (i, err)


def test_reference_mode_matches_per_sample_train_mode(gpu):
    from aido1_amd.actor import ConfigActor, FusedActor
    from test_trainer import no_dropout
    a = ConfigActor(no_dropout(golden('reference_config.json')['model']['actor']))
    a.load_state_dict(formula_state_dict(a.state_dict()))
    x = formula_input(4)
    a.train()
    with torch.no_grad():
        ref = torch.cat([a(x[i:i + 1]) for i in range(4)])
    f32 = FusedActor(a.to(gpu), dtype=torch.float32, mode='reference')
    np.testing.assert_allclose(f32(x.to(gpu)).cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    # fp16: per-sample normalisation of nearly flat channels amplifies the
    # conv outputs' fp16 rounding; formula frames are the harsh case
    h = FusedActor(a, dtype=torch.float16, mode='reference')
    assert torch.max(torch.abs(h(x.to(gpu)).cpu() - ref)) < 5e-2
    # rendered frames (what the rollout feeds it)
    from aido1_amd.rollout import ActorRollout
    roll = ActorRollout(golden('reference_config.json'), 32, device=0, seed=3)
    roll.reset()
    for _ in range(4):
        roll.step()
    frames = roll.stack()
    a_cpu = ConfigActor(no_dropout(golden('reference_config.json')['model']['actor']))
    a_cpu.load_state_dict(formula_state_dict(a_cpu.state_dict()))
    a_cpu.train()
    with torch.no_grad():
        ref = torch.cat([a_cpu(frames[i:i + 1].cpu()) for i in range(32)])
    assert torch.max(torch.abs(h(frames).cpu() - ref)) < 1.5e-2


@pytest.mark.parametrize('slots,order,n', [(3, [0, 1, 2], 37), (4, [2, 3, 0], 37),
                                           (4, [1, 2, 3], 1100)])
def test_conv1_kernel_matches_conv2d(gpu, slots, order, n):
    """dt_conv1 (MFMA implicit GEMM on the ring) vs conv2d + LeakyReLU in f32 on
    the same fp16-rounded inputs and weights; band statistics and the merged
    per-sample norm vs float64.  n = 1100 is more samples than the streaming
    kernel's resident workgroups, so each workgroup streams several samples
    through its row ring."""
    import ctypes
    import torch.nn.functional as F
    from aido1_amd import _lib
    from aido1_amd.actor import conv1_fragments
    L = _lib.lib()
    torch.manual_seed(1)
    ring = torch.rand(n, slots, 120, 160, device=gpu)
    w = torch.randn(32, 3, 8, 8, device=gpu) * 0.08
    b = torch.randn(32, device=gpu) * 0.2
    x = ring[:, order].half().float()
    ref = F.leaky_relu(F.conv2d(x, w.half().float(), b, stride=2))      # [n,32,57,77]
    y = torch.empty(n, 57, 77, 32, dtype=torch.float16, device=gpu)
    part = torch.empty(n, 32, 3, device=gpu)
    o = (ctypes.c_int32 * 3)(*order)
    s = torch.cuda.current_stream().cuda_stream
    wf = conv1_fragments(w)     # held: a temporary's memory could be reused before the launch
    assert L.dt_conv1(ring.data_ptr(), n, slots, o, wf.data_ptr(), b.data_ptr(),
                      y.data_ptr(), part.data_ptr(), 0.01, s) == 0
    # reference mode stores the outputs centred on the sample's pixel 0
    c = part[..., 2]
    tol = 2e-3 * max(1.0, ref.abs().max().item())
    assert (c - ref[:, :, 0, 0]).abs().max().item() < tol
    got = y.permute(0, 3, 1, 2).float() + c[:, :, None, None]
    err = (got - ref).abs().max().item()
    assert err < tol, err
    # per-sample statistics (mean, M2) of the f32 outputs
    r64 = ref.double()
    mean = r64.mean((2, 3))
    m2 = ((r64 - mean[:, :, None, None]) ** 2).sum((2, 3))
    assert torch.allclose(part[..., 0].double() + c.double(), mean, rtol=1e-3, atol=1e-3)
    assert torch.allclose(part[..., 1].double(), m2, rtol=2e-3, atol=1e-2)
    gamma = torch.rand(32, device=gpu) + 0.5
    beta = torch.rand(32, device=gpu) - 0.5
    y16 = y.permute(0, 3, 1, 2).double() + c.double()[:, :, None, None]   # what it normalises
    assert L.dt_conv1_norm(y.data_ptr(), n, part.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                           1e-5, s) == 0
    m = r64.mean((2, 3), keepdim=True)
    v = ((r64 - m) ** 2).mean((2, 3), keepdim=True)
    want = (y16 - m) / torch.sqrt(v + 1e-5) * gamma.double().view(1, -1, 1, 1) + \
        beta.double().view(1, -1, 1, 1)
    err = (y.permute(0, 3, 1, 2).double() - want).abs().max().item()
    assert err < 5e-3 * max(1.0, want.abs().max().item()), err    # fp16 output rounding


@pytest.mark.parametrize('n', [19, 1100])
@pytest.mark.parametrize('layer,shape,stride', [(2, (57, 77), 2), (3, (27, 37), 2), (4, (12, 17), 1)])
def test_conv32_layers_match_conv2d(gpu, layer, shape, stride, n):
    """dt_conv32 without statistics (the eval-mode layer) vs conv2d + LeakyReLU
    on the same fp16 data; layer 4 writes the NCHW flatten.  n = 1100 exceeds
    the resident grid, so workgroups stream several samples through the ring."""
    import torch.nn.functional as F
    from aido1_amd import _lib
    from aido1_amd.actor import conv32_fragments
    L = _lib.lib()
    torch.manual_seed(layer)
    x = (torch.rand(n, 32, *shape, device=gpu) * 2 - 0.5).half()
    w = (torch.randn(32, 32, 4, 4, device=gpu) * 0.05).half()
    b = (torch.randn(32, device=gpu) * 0.1).half().float()
    ref = F.leaky_relu(F.conv2d(x.float(), w.float(), b, stride=stride))
    xh = x.permute(0, 2, 3, 1).contiguous()                        # NHWC
    oh, ow = ref.shape[2:]
    y = torch.empty(n, 32 * oh * ow if layer == 4 else oh * ow * 32, dtype=torch.float16,
                    device=gpu)
    s = torch.cuda.current_stream().cuda_stream
    wf = conv32_fragments(w.float())   # held across the launch
    assert L.dt_conv32(layer, n, xh.data_ptr(), wf.data_ptr(),
                       b.data_ptr(), None, None, None, 0.0, y.data_ptr(), None, None, None,
                       0.0, 0.01, s) == 0
    got = y.view(n, 32, oh, ow) if layer == 4 else y.view(n, oh, ow, 32).permute(0, 3, 1, 2)
    err = (got.float() - ref).abs().max().item()
    assert err < 3e-3 * max(1.0, ref.abs().max().item()), err


def test_fp16_eval_mode_close_to_fp32(gpu):
    from aido1_amd.actor import ConfigActor, FusedActor
    a = ConfigActor(golden('reference_config.json')['model']['actor'])
    a.load_state_dict(formula_state_dict(a.state_dict()))
    a.eval()
    x = formula_input(4)
    with torch.no_grad():
        ref = a(x)
    f = FusedActor(a.to(gpu), dtype=torch.float16, mode='eval')
    assert torch.max(torch.abs(f(x.to(gpu)).cpu() - ref)) < 1e-2


def test_hip_convs_reference_mode_many_samples(gpu):
    """The fp16 HIP conv chain in reference mode (every per-sample BatchNorm
    applied by the next kernel) vs the f32 MIOpen + dt_sample_norm path, for
    more samples than the persistent grid holds at once."""
    from aido1_amd.actor import ConfigActor, FusedActor
    from test_trainer import no_dropout
    a = ConfigActor(no_dropout(golden('reference_config.json')['model']['actor']))
    a.load_state_dict(formula_state_dict(a.state_dict()))
    torch.manual_seed(5)
    x = torch.rand(1100, 3, 120, 160, device=gpu)
    h = FusedActor(a.to(gpu), dtype=torch.float16, mode='reference')
    f = FusedActor(a, dtype=torch.float32, mode='reference')
    got = h(x)
    want = f(x)
    assert torch.isfinite(got).all()
    assert torch.max(torch.abs(got - want)).item() < 2e-2


def test_rollout_exploiter_block(gpu):
    """config.json:183-186's 7 exploring + 1 exploiting explorers: the last n/8
    envs act with load_exploit_actor's weights, epsilon 0 (explorers.py:116,
    182-184): their stored action is the clipped actor output, mapped by the
    wrapper, with no noise and no random action."""
    from aido1_amd.actor import ConfigActor, FusedActor
    from aido1_amd.rollout import ActorRollout
    cfg = golden('reference_config.json')
    roll = ActorRollout(cfg, 512, device=0, seed=5, actor_mode='eval', dtype=torch.float16)
    assert roll.n_exploit == 64 and roll.n_explore == 448
    torch.manual_seed(21)
    other = ConfigActor(cfg['model']['actor']).to(gpu)
    roll.load_exploit_actor(other)
    ref = FusedActor(other, dtype=torch.float16, mode='eval').to(gpu)
    roll.reset()
    for _ in range(3):
        roll.step()
    ne = roll.n_explore
    # the next decision, recomputed from the frames it sees (the ring before it)
    obs = roll.ring.clone()
    order = roll.order()
    out = ref(obs[ne:], order).float()
    roll.step()
    want = out.clamp(-1.0, 1.0) / 2 + 0.5
    assert torch.equal(roll.actions[ne:], want)
    # exploring envs: noise / random actions make them differ from the plain map
    mine = roll.actor(obs[:ne], order).float().clamp(-1.0, 1.0) / 2 + 0.5
    assert not torch.equal(roll.actions[:ne], mine)
    roll.close()


def test_conv1s_reads_stay_inside_the_ring(gpu):
    """Regression for round 2's conv1s_kernel fault (the last sample's row-free
    step read past the frame ring): the DTCONV_CHECK build checks
    every ring load against n x slots x 120 x 160 and flags any past it.  The
    ring is its own exact-size allocation at the end of a fresh block, the
    1100-sample case where each workgroup streams several samples.  Runs in a
    subprocess because it loads the diagnostic library."""
    import os
    import subprocess
    import sys
    from aido1_amd import _lib
    assert os.path.exists(_lib.CHECK_LIB_PATH), 'build() makes libdtsim_check.so'
    code = r'''
import ctypes, sys, torch
sys.path.insert(0, %r)
from aido1_amd import _lib
from aido1_amd.actor import conv1_fragments
L = _lib.lib()
L.dt_diag_conv1_oob.argtypes = [ctypes.POINTER(ctypes.c_uint)]
dev = torch.device('cuda', 0)
for slots, order, n in ((4, [1, 2, 3], 1100), (3, [2, 0, 1], 37), (3, [0, 1, 2], 1)):
    ring = torch.rand(n, slots, 120, 160, device=dev)
    w = torch.randn(32, 3, 8, 8, device=dev) * 0.08
    b = torch.randn(32, device=dev) * 0.2
    y = torch.empty(n, 57, 77, 32, dtype=torch.float16, device=dev)
    part = torch.empty(n, 32, 3, device=dev)
    wf = conv1_fragments(w)
    o = (ctypes.c_int32 * 3)(*order)
    assert L.dt_conv1(ring.data_ptr(), n, slots, o, wf.data_ptr(), b.data_ptr(), y.data_ptr(),
                      part.data_ptr(), 0.01, torch.cuda.current_stream().cuda_stream) == 0
    flag = ctypes.c_uint(7)
    assert L.dt_diag_conv1_oob(ctypes.byref(flag)) == 0
    print(n, flag.value)
    assert flag.value == 0, 'conv1s_kernel read past the ring (n=%%d)' %% n
    # the palette-index ring (u8, its own exact-size allocation)
    del ring
    iring = torch.randint(0, 8, (n, slots, 120, 160), dtype=torch.uint8, device=dev)
    assert L.dt_conv1_index_split(iring.data_ptr(), n, slots, o, wf.data_ptr(), b.data_ptr(),
                                  None, y.data_ptr(), part.data_ptr(), 0.01,
                                  torch.cuda.current_stream().cuda_stream) == 0
    flag = ctypes.c_uint(7)
    assert L.dt_diag_conv1_oob(ctypes.byref(flag)) == 0
    assert flag.value == 0, 'conv1s_kernel read past the index ring (n=%%d)' %% n
''' % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),)
    env = dict(os.environ, DTSIM_DIAG_LIB=_lib.CHECK_LIB_PATH)
    r = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]


@pytest.mark.parametrize('mode', ['reference', 'eval'])
@pytest.mark.parametrize('n,n0', [(600, 525), (97, 1), (97, 96), (4096, 3584)])
def test_split_launch_matches_separate_actors(gpu, mode, n, n0):
    """dt_conv1_split / dt_conv32_split (include/dtactor.h): one launch per
    convolution over two weight sets gives every sample exactly (bit for bit)
    what a launch with its own set gives -- the exploring / exploiting split of
    rollout.ActorRollout (explorers.py:104-105, config.json:183-186)."""
    from aido1_amd.actor import ConfigActor, FusedActor
    cfg = golden('reference_config.json')['model']['actor']
    torch.manual_seed(7)
    a, b = ConfigActor(cfg), ConfigActor(cfg)
    if mode == 'eval':
        for m in (a, b):
            for bn in [x for x in m.modules() if isinstance(x, torch.nn.BatchNorm2d)]:
                bn.running_mean.uniform_(-0.2, 0.2)
                bn.running_var.uniform_(0.5, 2.0)
    fa = FusedActor(a.to(gpu), dtype=torch.float16, mode=mode)
    fb = FusedActor(b.to(gpu), dtype=torch.float16, mode=mode)
    if mode == 'reference':
        with torch.no_grad():
            for f in (fa, fb):
                for p in list(f.gamma) + list(f.beta):
                    p.uniform_(0.5, 1.5)
    g = torch.Generator(device=gpu).manual_seed(n)
    ring = torch.rand(n, 3, 120, 160, device=gpu, generator=g)
    order = [2, 0, 1]
    flat = fa._convs_pair(fb, ring, order, n0).clone()
    fa_flat = fa._convs_hip(ring[:n0].contiguous(), order)
    fb_flat = fb._convs_hip(ring[n0:].contiguous(), order)
    assert torch.equal(flat[:n0], fa_flat)
    assert torch.equal(flat[n0:], fb_flat)
    fa.p_drop = fb.p_drop = 0.0
    out = fa.forward_pair(fb, ring, order, n0)
    ref = torch.cat([fa(ring[:n0].contiguous(), order), fb(ring[n0:].contiguous(), order)])
    assert torch.allclose(out, ref, atol=1e-3), (out - ref).abs().max()


@pytest.mark.parametrize('mode', ['reference', 'eval'])
@pytest.mark.parametrize('n,n0,slots,order', [(1100, 1100, 4, [1, 2, 3]), (600, 525, 3, [2, 0, 1]),
                                              (37, 36, 3, [0, 1, 2])])
def test_index_ring_equals_grey_ring(gpu, mode, n, n0, slots, order):
    """dt_conv1_index_split on palette-index frames (u8) gives bit for bit
    what dt_conv1_split gives on their grey frames (render.decode_index), for
    one weight set and for the exploring / exploiting split, through the whole
    conv chain; n = 1100 streams several samples per workgroup."""
    from aido1_amd.actor import ConfigActor, FusedActor
    from aido1_amd.render import decode_index
    cfg = golden('reference_config.json')['model']['actor']
    torch.manual_seed(n)
    fa = FusedActor(ConfigActor(cfg).to(gpu), dtype=torch.float16, mode=mode)
    fb = FusedActor(ConfigActor(cfg).to(gpu), dtype=torch.float16, mode=mode)
    g = torch.Generator(device=gpu).manual_seed(n + 1)
    idx = torch.randint(0, 8, (n, slots, 120, 160), dtype=torch.uint8, device=gpu, generator=g)
    grey = decode_index(idx)
    assert torch.equal(fa._convs_hip(idx, order), fa._convs_hip(grey, order))
    if n0 < n:
        assert torch.equal(fa._convs_pair(fb, idx, order, n0).clone(),
                           fa._convs_pair(fb, grey, order, n0))


@pytest.mark.parametrize('n,n0', [(300, 300), (300, 257), (64, 1), (4096, 3584)])
def test_fused_head_matches_float64(gpu, n, n0):
    """The fast mode's head (dt_actor_head_f16_drop: lin1 on fp16 MFMA with
    f32 accumulation, LeakyReLU, lin2, tanh for both weight sets in one
    launch pair) against float64 of the same fp16 operands (its lin1 weights,
    biases and inputs): the products are exact, the sums f32 (2e-6); and
    against FusedActor._head's torch fp16 ops, which round lin1's output and
    the pre-tanh value to fp16 (2e-3)."""
    from aido1_amd.actor import FLAT, ConfigActor, FusedActor
    from test_trainer import no_dropout
    cfg = golden('reference_config.json')['model']['actor']
    torch.manual_seed(n + n0)
    fa = FusedActor(ConfigActor(no_dropout(cfg)).to(gpu), dtype=torch.float16)
    fb = FusedActor(ConfigActor(no_dropout(cfg)).to(gpu), dtype=torch.float16)
    assert fa._head_fusable(fb)
    flat = (torch.randn(n, FLAT, device=gpu) * 0.5).half()
    out = torch.full((n, 2), float('nan'), device=gpu)
    fa._heads(fb, flat, n0, out)
    assert torch.isfinite(out).all()
    want = []
    for a, sl in ((fa, slice(0, n0)), (fb, slice(n0, n))):
        h = torch.nn.functional.leaky_relu(flat[sl].double() @ a.w1.double().t() + a.b1.double())
        want.append(torch.tanh(h @ a.w2.double().t() + a.b2.double()))
    want = torch.cat(want)
    assert (out.double() - want).abs().max().item() < 2e-6
    ref = torch.cat([fa._head(flat[:n0]), fb._head(flat[n0:])])
    assert torch.allclose(out, ref, rtol=0, atol=2e-3), (out - ref).abs().max()


def test_fused_head_dropout_keeps_the_rate(gpu):
    """Reference mode's dropout folded into the fast-mode head: two calls use
    fresh masks (different outputs), and each differs from the no-dropout
    output (the same folded hash as dt_actor_head_x3_drop, whose mask
    tests/test_gpu_actor_x3.py restates bit for bit)."""
    from aido1_amd.actor import FLAT, ConfigActor, FusedActor
    cfg = golden('reference_config.json')['model']['actor']
    torch.manual_seed(3)
    fa = FusedActor(ConfigActor(cfg).to(gpu), dtype=torch.float16, mode='reference')
    assert fa.p_drop == 0.5 and hasattr(fa, 'w1f')
    flat = (torch.randn(256, FLAT, device=gpu) * 0.5).half()
    outs = []
    for _ in range(2):
        out = torch.empty(256, 2, device=gpu)
        fa._heads(None, flat, 256, out)
        outs.append(out)
    fa.p_drop = 0.0
    plain = torch.empty(256, 2, device=gpu)
    fa._heads(None, flat, 256, plain)
    assert not torch.equal(outs[0], outs[1])
    assert not torch.equal(outs[0], plain)


@pytest.mark.parametrize('channels_last', [False, True])
def test_refresh_copies_every_parameter_exactly(gpu, channels_last):
    """FusedActor.refresh (reference mode, fp16) copies every weight, bias,
    gamma and beta of the source actor, whatever memory the caching allocator
    hands it: free blocks are filled with NaN first.  A single mixed-dtype
    torch._foreach_copy_ wrote the fp16 conversion into the float32 gamma /
    beta on this ROCm build (round 4; actor.copy_grouped)."""
    from aido1_amd.actor import ConfigActor, FusedActor
    held = [torch.full((4096,), float('nan'), device=gpu) for _ in range(64)]
    del held
    torch.manual_seed(9)
    a = ConfigActor(golden('reference_config.json')['model']['actor']).to(gpu)
    with torch.no_grad():
        for p in a.parameters():
            p.add_(torch.randn_like(p) * 0.1)
    if channels_last:
        a = a.to(memory_format=torch.channels_last)
    f = FusedActor(a, dtype=torch.float16, mode='reference')
    torch.cuda.synchronize()
    convs, bns, lin1, lin2 = a.layers()
    for i in range(4):
        assert torch.equal(f.w[i].float(), convs[i].weight.detach().half().float()), i
        assert torch.equal(f.b[i].float(), convs[i].bias.detach().half().float()), i
        assert torch.equal(f.gamma[i], bns[i].weight.detach()), i
        assert torch.equal(f.beta[i], bns[i].bias.detach()), i
    for mine, src in ((f.w1, lin1.weight), (f.b1, lin1.bias), (f.w2, lin2.weight),
                      (f.b2, lin2.bias)):
        assert torch.equal(mine.float(), src.detach().half().float())


@pytest.mark.parametrize('mode,dtype', [('reference', torch.float16), ('eval', torch.float16),
                                        ('reference', torch.float32)])
def test_graph_refresh_follows_in_place_updates(gpu, mode, dtype):
    """FusedActor.refresh on the GPU: one dt_refresh_copy launch through index
    maps built at the first refresh from a source (reference mode), or a HIP
    graph captured then (eval mode): after in-place updates of the source's
    weights (what Adam and the soft update do) every acting tensor equals an
    eager refresh's bit for bit."""
    from aido1_amd.actor import ConfigActor, FusedActor
    torch.manual_seed(13)
    a = ConfigActor(golden('reference_config.json')['model']['actor']).to(gpu)
    f = FusedActor(a, dtype=dtype, mode=mode)
    for k in range(3):
        with torch.no_grad():
            for p in a.parameters():
                p.add_(torch.randn_like(p) * 0.05)
            for bn in [m for m in a.modules() if isinstance(m, torch.nn.BatchNorm2d)]:
                bn.running_mean.uniform_(-0.2, 0.2)
                bn.running_var.uniform_(0.5, 2.0)
        f.refresh(a)
        ref = FusedActor(a, dtype=dtype, mode=mode)
        torch.cuda.synchronize()
        for (name, x), (_, y) in zip(f.state_dict().items(), ref.state_dict().items()):
            if mode == 'eval' and name.startswith(('gamma', 'beta')):
                continue            # folded into the weights: unused (never written) in eval mode
            assert torch.equal(x, y), (k, name)
    # one capture per source: reference mode's gather table, eval mode's graph
    assert len(f._refresh_tables if mode == 'reference' else f._refresh_graphs) == 1
