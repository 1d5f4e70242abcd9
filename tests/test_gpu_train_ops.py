"""The fused conv-block tail of the DDPG update (include/dttrain.h,
aido1_amd/train_ops.py) against float64 torch: bias + LeakyReLU + train-mode
BatchNorm forward (outputs, running statistics, num_batches_tracked) and its
backward (input, bias, gamma and beta gradients); then whole networks with
and without it.  float32 kernels against float64 math: rtol 1e-4 / atol 1e-5
on outputs, 1e-4 relative to the largest element on gradients (reductions of
up to 281k terms in a different order)."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from conftest import golden

pytestmark = pytest.mark.gpu


def _ref_tail(z, bias, bn, slope):
    a = F.leaky_relu(z + bias.view(1, -1, 1, 1), slope)
    return F.batch_norm(a, bn.running_mean, bn.running_var, bn.weight, bn.bias, True,
                        bn.momentum, bn.eps)


@pytest.mark.parametrize('shape', [(64, 32, 57, 77), (64, 32, 9, 14), (3, 32, 5, 7)])
def test_bn_leaky_tail_matches_float64(gpu, shape):
    from aido1_amd.train_ops import _BnLeaky
    torch.manual_seed(sum(shape))
    cl = torch.channels_last
    z = (torch.randn(shape, device=gpu) * 2 + 0.3).contiguous(memory_format=cl)
    bias = torch.randn(32, device=gpu) * 0.5
    bn = nn.BatchNorm2d(32).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    ref_bn = copy.deepcopy(bn).double()
    dy = torch.randn(shape, device=gpu).contiguous(memory_format=cl)

    zl = z.clone().requires_grad_(True)
    bl = bias.clone().requires_grad_(True)
    y = _BnLeaky.apply(zl, bl, bn.weight, bn.bias, bn, 0.01)
    y.backward(dy)

    zr = z.double().requires_grad_(True)
    br = bias.double().requires_grad_(True)
    yr = _ref_tail(zr, br, ref_bn, 0.01)
    yr.backward(dy.double())

    torch.testing.assert_close(y.double(), yr.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_mean.double(), ref_bn.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn.running_var.double(), ref_bn.running_var, rtol=1e-5, atol=1e-6)
    assert int(bn.num_batches_tracked) == 1
    for got, want in ((zl.grad, zr.grad), (bl.grad, br.grad), (bn.weight.grad, ref_bn.weight.grad),
                      (bn.bias.grad, ref_bn.bias.grad)):
        scale = want.abs().max().item()
        assert (got.double() - want).abs().max().item() <= 1e-4 * scale + 1e-6


@pytest.mark.parametrize('kind', ['actor', 'critic'])
def test_networks_with_and_without_fused_tail(gpu, kind):
    """A config.json actor / critic in train mode, f32 channels_last, batch 64:
    forward, every parameter gradient and the BatchNorm running statistics
    with the fused tail match torch's modules."""
    from aido1_amd.actor import ConfigActor, ConfigCritic, _Seq
    cfg = golden('reference_config.json')['model']
    torch.manual_seed(4)
    net = (ConfigActor(cfg['actor']) if kind == 'actor' else ConfigCritic(cfg['critic']))
    for m in net.modules():
        if isinstance(m, nn.Dropout):
            m.p = 0.0
    net = net.to(gpu).to(memory_format=torch.channels_last).train()
    ref = copy.deepcopy(net)
    x = torch.rand(64, 3, 120, 160, device=gpu).contiguous(memory_format=torch.channels_last)
    args = (x,) if kind == 'actor' else (x, torch.rand(64, 2, device=gpu))
    try:
        _Seq.fused_tail = False
        out_ref = ref(*args)
        out_ref.square().mean().backward()
    finally:
        _Seq.fused_tail = True
    out = net(*args)
    out.square().mean().backward()
    torch.testing.assert_close(out, out_ref, rtol=1e-4, atol=1e-5)
    for (name, p), (_, q) in zip(net.named_parameters(), ref.named_parameters()):
        scale = q.grad.abs().max().item()
        assert (p.grad - q.grad).abs().max().item() <= 2e-4 * scale + 1e-7, name
    for (name, b), (_, c) in zip(net.named_buffers(), ref.named_buffers()):
        if b.dtype.is_floating_point:
            torch.testing.assert_close(b, c, rtol=1e-5, atol=1e-6, msg=name)
        else:
            assert torch.equal(b, c), name


def test_device_adam_matches_torch_adam(gpu):
    """dt_adam (one launch over every parameter) against torch.optim.Adam
    (plain, Python-double bias corrections) over five steps with a changing
    lr, on a conv + BatchNorm + linear stack with channels_last weights."""
    from aido1_amd.optim import DeviceAdam
    torch.manual_seed(8)
    net = nn.Sequential(nn.Conv2d(3, 32, 8, stride=2), nn.BatchNorm2d(32), nn.Flatten(),
                        nn.Linear(32 * 3 * 3, 5)).to(gpu).to(memory_format=torch.channels_last)
    ref = copy.deepcopy(net)
    opt = DeviceAdam(net.parameters(), gpu)
    ropt = torch.optim.Adam(ref.parameters(), lr=0.0)
    for k in range(5):
        lr = 1e-3 * (1.0 - 0.1 * k)
        opt.param_groups[0]['lr'].fill_(lr)
        ropt.param_groups[0]['lr'] = lr
        for p, q in zip(net.parameters(), ref.parameters()):
            g = torch.randn_like(p) * (0.1 + k)
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.copy_(g)
            q.grad = g.clone()
        opt.step()
        ropt.step()
    for p, q in zip(net.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-6, atol=1e-7)
        st, rst = opt.state[p], ropt.state[q]
        # torch's lerp kernel contracts to an fma: ulp-level differences
        torch.testing.assert_close(st['exp_avg'], rst['exp_avg'], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(st['exp_avg_sq'], rst['exp_avg_sq'], rtol=1e-6, atol=1e-10)
        assert float(st['step']) == 5.0
    assert opt._table is not None          # the fused path ran


def test_device_adam_load_state_dict_cpu_map_eager_and_graph(gpu, tmp_path):
    """DeviceAdam.load_state_dict from torch.save + torch.load(map_location='cpu',
    weights_only=True): the lr stays the group's float64 device tensor (filled
    with the loaded value), the moments land in the tensors they replace, so
    both an eager step and a HIP graph captured BEFORE the load continue the
    saved optimiser bit for bit."""
    from aido1_amd.optim import DeviceAdam
    torch.manual_seed(10)
    src = nn.Sequential(nn.Linear(64, 32), nn.Linear(32, 8)).to(gpu)
    opt = DeviceAdam(src.parameters(), gpu)
    for lr in (1e-3, 5e-4):
        opt.param_groups[0]['lr'].fill_(lr)
        for p in src.parameters():
            p.grad = torch.randn_like(p)
        opt.step()
    path = tmp_path / 'adam.pt'
    torch.save(opt.state_dict(), path)
    net_e, net_g = copy.deepcopy(src), copy.deepcopy(src)
    grads = [torch.randn_like(p) for p in src.parameters()]
    for p, g in zip(src.parameters(), grads):
        p.grad.copy_(g)
    opt.param_groups[0]['lr'].fill_(2e-4)
    opt.step()
    # eager
    opt_e = DeviceAdam(net_e.parameters(), gpu)
    lr_e = opt_e.param_groups[0]['lr']
    opt_e.load_state_dict(torch.load(path, map_location='cpu', weights_only=True))
    assert opt_e.param_groups[0]['lr'] is lr_e and lr_e.device.type == 'cuda'
    assert lr_e.dtype == torch.float64 and float(lr_e) == 5e-4
    lr_e.fill_(2e-4)
    for p, g in zip(net_e.parameters(), grads):
        p.grad = g.clone()
    opt_e.step()
    assert opt_e._table is not None
    # graph captured before the load
    opt_g = DeviceAdam(net_g.parameters(), gpu)
    lr_g = opt_g.param_groups[0]['lr']
    for p in net_g.parameters():
        p.grad = torch.zeros_like(p)
    opt_g.step()                      # lr 0, zero grads: builds the dt_adam table
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        opt_g.step()
    opt_g.load_state_dict(torch.load(path, map_location='cpu', weights_only=True))
    assert opt_g.param_groups[0]['lr'] is lr_g and float(lr_g) == 5e-4
    lr_g.fill_(2e-4)
    for p, g in zip(net_g.parameters(), grads):
        p.grad.copy_(g)
    graph.replay()
    torch.cuda.synchronize()
    for a, b, c in zip(src.parameters(), net_e.parameters(), net_g.parameters()):
        assert torch.equal(a, b) and torch.equal(a, c)
    for p, q in zip(src.parameters(), net_g.parameters()):
        assert torch.equal(opt.state[p]['exp_avg'], opt_g.state[q]['exp_avg'])
        assert float(opt_g.state[q]['step']) == 3.0


def test_soft_update_gpu_bit_exact(gpu):
    """dt_soft_update = torch's t * (1 - tau) + p * tau, bit for bit."""
    from aido1_amd.trainer import soft_update
    torch.manual_seed(9)
    a = nn.Sequential(nn.Conv2d(3, 32, 4), nn.Linear(7, 3)).to(gpu).to(
        memory_format=torch.channels_last)
    b = copy.deepcopy(a)
    for p in b.parameters():
        p.data.add_(torch.randn_like(p))
    tau = 0.005
    expect = [t.data * (1.0 - tau) + s.data * tau for t, s in zip(a.parameters(), b.parameters())]
    soft_update(a, b, tau)
    for t, e in zip(a.parameters(), expect):
        assert torch.equal(t.data, e)


def test_shared_critic_trunk_equals_two_forwards(gpu):
    """trainer._shared_trunk: trunk(obs) once under running_updates(2) then
    head() twice == two full train-mode forwards of the critic, bit for bit:
    the outputs and every state_dict entry (running statistics moved twice,
    num_batches_tracked += 2).  Dropout p = 0 so the heads are deterministic."""
    from aido1_amd.actor import ConfigCritic
    from aido1_amd.train_ops import running_updates
    from test_trainer import no_dropout
    cfg = golden('reference_config.json')
    torch.manual_seed(3)
    cl = torch.channels_last
    a = ConfigCritic(no_dropout(cfg['model']['critic'])).to(gpu).to(memory_format=cl).train()
    b = copy.deepcopy(a)
    obs = torch.rand(16, 3, 120, 160, device=gpu).contiguous(memory_format=cl)
    act1, act2 = torch.rand(16, 2, device=gpu), torch.rand(16, 2, device=gpu)
    with torch.no_grad():
        q1, q2 = a(obs, act1), a(obs, act2)
        with running_updates(b, 2):
            t = b.trunk(obs)
        s1, s2 = b.head(t, act1), b.head(t, act2)
    assert torch.equal(q1, s1) and torch.equal(q2, s2)
    sa, sb = a.state_dict(), b.state_dict()
    assert list(sa) == list(sb)
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
    assert int(sb['net.input_nets.0.internal_modules.2.num_batches_tracked']) == 2
    with pytest.raises(NotImplementedError):   # the torch BatchNorm path cannot repeat
        with running_updates(b.cpu().double(), 2):
            b.trunk(obs.cpu().double())


@pytest.mark.parametrize('slope', [0.01, -0.2])
def test_linear_leaky_fusion_only_for_nonnegative_slope(gpu, slope):
    """_Seq fuses linear -> LeakyReLU into the split-K kernel (its backward
    takes the gradient from the sign of the saved output) only for a slope
    >= 0; a negative slope runs the unfused linear and torch's leaky_relu.
    Either way: output and gradients as torch's modules (float32 tolerance)."""
    from aido1_amd.actor import _Lin, _Seq
    torch.manual_seed(12)
    seq = _Seq([_Lin(1024, 64), nn.LeakyReLU(slope)]).to(gpu)
    ref = copy.deepcopy(seq)
    ref.fused_tail = False
    x = torch.randn(8, 1024, device=gpu, requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)
    y, yr = seq(x), ref(xr)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-5)
    for p, q in zip(seq.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize('m,k0,k1,n1,n2,acts', [
    (64, 256, 2, 128, 1, ('leaky', 'none')),      # config.json's critic tail
    (64, 512, 0, 2, 0, ('tanh', None)),           # config.json's actor tail
    (1, 40, 3, 17, 5, ('sigmoid', 'tanh')),
    (37, 1024, 0, 64, 2, ('leaky', 'sigmoid')),
    (256, 8, 8, 32, 0, ('none', None))])
def test_mlp_tail_matches_float64(gpu, m, k0, k1, n1, n2, acts):
    """dt_mlp_fwd / dt_mlp_bwd (include/dthead.h) through train_ops.mlp against
    float64 torch: the output and every input / parameter gradient, also with
    only some gradients asked for."""
    from aido1_amd import train_ops
    torch.manual_seed(m + k0 + n1)
    mods = [nn.Linear(k0 + k1, n1)]
    act = {'leaky': nn.LeakyReLU(0.01), 'tanh': nn.Tanh(), 'sigmoid': nn.Sigmoid(), 'none': None}
    if act[acts[0]] is not None:
        mods.append(act[acts[0]])
    if n2:
        mods.append(nn.Linear(n1, n2))
        if act[acts[1]] is not None:
            mods.append(act[acts[1]])

    class _L(nn.Module):   # the config MetaNet's '.linear' wrapper
        def __init__(self, lin):
            super().__init__()
            self.linear = lin

    class _S(nn.Module):
        def __init__(self, ms):
            super().__init__()
            self.internal_modules = nn.ModuleList(
                [_L(x) if isinstance(x, nn.Linear) else x for x in ms])

    seq = _S(mods).to(gpu)
    x0 = torch.randn(m, k0, device=gpu, requires_grad=True)
    x1 = torch.randn(m, k1, device=gpu, requires_grad=True) if k1 else None
    parts = [x0] + ([x1] if k1 else [])
    plan = train_ops.mlp_plan(seq, parts)
    assert plan is not None
    y = train_ops.mlp(parts, plan)
    ref = copy.deepcopy(nn.Sequential(*mods)).double()
    x64 = torch.cat([p.detach().double() for p in parts], 1).requires_grad_(True)
    y64 = ref(x64)
    torch.testing.assert_close(y.double(), y64, rtol=1e-5, atol=1e-6)
    g = torch.randn_like(y)
    y.backward(g)
    y64.backward(g.double())
    gx = torch.cat([p.grad for p in parts], 1)
    torch.testing.assert_close(gx.double(), x64.grad, rtol=1e-5, atol=1e-6)
    for a, b in zip([x for x in seq.parameters()], ref.parameters()):
        torch.testing.assert_close(a.grad.double(), b.grad, rtol=1e-5, atol=1e-5)
    # only the first input's gradient
    for p in seq.parameters():
        p.grad = None
        p.requires_grad_(False)
    x0.grad = None
    y2 = train_ops.mlp(parts, train_ops.mlp_plan(seq, parts))
    (gx0,) = torch.autograd.grad(y2, [x0], g)
    torch.testing.assert_close(gx0, gx[:, :k0], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('m', [1, 64, 300])
def test_fused_losses_match_torch(gpu, m):
    """dt_loss / dt_loss_bwd (train_ops.mse_loss, neg_mean): the DDPG critic
    and actor losses and their input gradients against float64 torch."""
    from aido1_amd import train_ops
    torch.manual_seed(m)
    a = torch.randn(m, 1, device=gpu, requires_grad=True)
    b = torch.randn(m, 1, device=gpu)
    loss = train_ops.mse_loss(a, b)
    a64 = a.detach().double().requires_grad_(True)
    ref = torch.nn.functional.mse_loss(a64, b.double())
    torch.testing.assert_close(loss.double(), ref, rtol=1e-6, atol=1e-7)
    loss.backward()
    ref.backward()
    torch.testing.assert_close(a.grad.double(), a64.grad, rtol=1e-6, atol=1e-8)
    q = torch.randn(m, 1, device=gpu, requires_grad=True)
    lq = train_ops.neg_mean(q)
    q64 = q.detach().double().requires_grad_(True)
    rq = -1.0 * torch.mean(q64)
    torch.testing.assert_close(lq.double(), rq, rtol=1e-6, atol=1e-7)
    lq.backward(torch.tensor(0.5, device=gpu))
    rq.backward(torch.tensor(0.5, dtype=torch.float64, device=gpu))
    torch.testing.assert_close(q.grad.double(), q64.grad, rtol=1e-6, atol=1e-9)


def test_td_target_in_the_critic_head(gpu):
    """ConfigCritic.td_target (dt_mlp_fwd_td: the output branch and
    rew + (notdone * gamma) * Q in one launch) equals the torch expression on
    the critic's forward, with dropout off."""
    from aido1_amd.actor import ConfigCritic
    from test_trainer import no_dropout
    cfg = no_dropout(golden('reference_config.json')['model']['critic'])
    torch.manual_seed(3)
    c = ConfigCritic(cfg).to(gpu).to(memory_format=torch.channels_last).eval()
    obs = torch.rand(64, 3, 120, 160, device=gpu).contiguous(memory_format=torch.channels_last)
    act = torch.rand(64, 2, device=gpu)
    rew = torch.randn(64, 1, device=gpu)
    notdone = (torch.rand(64, 1, device=gpu) > 0.2).float()
    with torch.no_grad():
        got = c.td_target(obs, act, rew, notdone, 0.99)
        want = rew + notdone * 0.99 * c(obs, act)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)
