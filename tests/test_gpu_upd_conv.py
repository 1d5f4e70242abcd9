"""The DDPG update's convolutions (include/dtupd.h, csrc/dtupd.hip): forward,
weight gradient and input gradient of config.json's four conv_2d layers
against a float64 CPU restatement (torch's conv2d and torch.nn.grad), for
batch sizes from 1 to past the persistent grid, and the train-mode conv
blocks through autograd against the MIOpen path.  Tolerance: the gradients
are an exact f32 fma chain per output (v_mfma_f32_32x32x2_f32) summed in
another order; the forward's x3 products (fp16 hi / lo pairs, dtupd.hip
DTUPD_X3) carry ~2^-21 of each product besides, so |err| <= 2e-5 * (sum of
|products|) is the bound written below for both (relative to the f64
result's scale)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

LAYERS = [(3, 8, 2, 120, 160), (32, 4, 2, 57, 77), (32, 4, 2, 27, 37), (32, 4, 1, 12, 17)]
CL = torch.channels_last


def _data(cin, ks, n, ih, iw, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, cin, ih, iw, generator=g, dtype=torch.float64) * 2 - 0.5
    w = torch.randn(32, cin, ks, ks, generator=g, dtype=torch.float64) * (2.0 / (cin * ks * ks)) ** 0.5
    return x, w


def _lib_call(name, *args):
    from aido1_amd import _lib
    rc = getattr(_lib.lib(), name)(*args)
    assert rc == 0, (name, rc)


def _bound(ref_abs):
    return 2e-5 * max(1.0, ref_abs)


@pytest.mark.parametrize('layer', LAYERS)
@pytest.mark.parametrize('n', [1, 5, 64])
def test_forward_matches_f64(gpu, layer, n):
    cin, ks, st, ih, iw = layer
    if cin == 3 and n == 64:
        n = 12                                   # CPU f64 reference time
    x, w = _data(cin, ks, n, ih, iw, seed=n + ks)
    ref = F.conv2d(x, w, stride=st)
    xg = x.float().to(gpu).contiguous(memory_format=CL)
    wg = w.float().to(gpu).contiguous(memory_format=CL)
    z = torch.full(ref.shape, float('nan'), device=gpu).contiguous(memory_format=CL)
    s = torch.cuda.current_stream().cuda_stream
    _lib_call('dt_upd_conv_fwd', cin, ks, st, n, ih, iw, xg.data_ptr(), wg.data_ptr(), z.data_ptr(), s)
    torch.cuda.synchronize()
    scale = F.conv2d(x.abs(), w.abs(), stride=st).max().item()
    err = (z.double().cpu() - ref).abs().max().item()
    assert err <= _bound(scale), (err, scale)


@pytest.mark.parametrize('layer', LAYERS)
@pytest.mark.parametrize('n', [1, 7, 64])
def test_weight_grad_matches_f64(gpu, layer, n):
    cin, ks, st, ih, iw = layer
    if cin == 3 and n == 64:
        n = 12
    x, w = _data(cin, ks, n, ih, iw, seed=3 * n + ks)
    oh, ow = (ih - ks) // st + 1, (iw - ks) // st + 1
    dz = torch.randn(n, 32, oh, ow, dtype=torch.float64, generator=torch.Generator().manual_seed(n))
    ref = torch.nn.grad.conv2d_weight(x, w.shape, dz, stride=st)
    from aido1_amd import _lib
    L = _lib.lib()
    xg = x.float().to(gpu).contiguous(memory_format=CL)
    dzg = dz.float().to(gpu).contiguous(memory_format=CL)
    dw = torch.full(w.shape, float('nan'), device=gpu).contiguous(memory_format=CL)
    work = torch.empty(int(L.dt_upd_wgrad_work_floats(cin, ks, st, n, ih, iw)), device=gpu)
    s = torch.cuda.current_stream().cuda_stream
    _lib_call('dt_upd_conv_wgrad', cin, ks, st, n, ih, iw, xg.data_ptr(), dzg.data_ptr(),
              dw.data_ptr(), work.data_ptr(), s)
    torch.cuda.synchronize()
    scale = torch.nn.grad.conv2d_weight(x.abs(), w.shape, dz.abs(), stride=st).max().item()
    err = (dw.double().cpu() - ref).abs().max().item()
    assert err <= _bound(scale), (err, scale)


@pytest.mark.parametrize('layer', LAYERS[1:])
@pytest.mark.parametrize('n', [1, 6, 64])
def test_input_grad_matches_f64(gpu, layer, n):
    cin, ks, st, ih, iw = layer
    x, w = _data(cin, ks, n, ih, iw, seed=5 * n + ks)
    oh, ow = (ih - ks) // st + 1, (iw - ks) // st + 1
    dz = torch.randn(n, 32, oh, ow, dtype=torch.float64, generator=torch.Generator().manual_seed(n))
    ref = torch.nn.grad.conv2d_input(x.shape, w, dz, stride=st)
    wg = w.float().to(gpu).contiguous(memory_format=CL)
    dzg = dz.float().to(gpu).contiguous(memory_format=CL)
    dx = torch.full(x.shape, float('nan'), device=gpu).contiguous(memory_format=CL)
    s = torch.cuda.current_stream().cuda_stream
    _lib_call('dt_upd_conv_dgrad', cin, ks, st, n, ih, iw, dzg.data_ptr(), wg.data_ptr(),
              dx.data_ptr(), s)
    torch.cuda.synchronize()
    scale = torch.nn.grad.conv2d_input(x.shape, w.abs(), dz.abs(), stride=st).max().item()
    got = dx.double().cpu()
    assert torch.isfinite(got).all()          # every element written (untouched rows: 0)
    err = (got - ref).abs().max().item()
    assert err <= _bound(scale), (err, scale)


def test_rejects_other_geometry(gpu):
    from aido1_amd import _lib
    L = _lib.lib()
    assert L.dt_upd_conv_fwd(32, 3, 1, 1, 12, 17, 0, 0, 0, None) != 0
    assert L.dt_upd_wgrad_work_floats(16, 4, 2, 1, 57, 77) == -1
    assert L.dt_upd_conv_dgrad(3, 8, 2, 1, 120, 160, 0, 0, 0, None) != 0


def test_conv_block_autograd_matches_miopen(gpu):
    """A train-mode config.json critic on the dtupd.h convolutions vs the same
    network on MIOpen (train_ops.UPD_CONV_LAYERS emptied): outputs and every
    parameter gradient."""
    from conftest import golden
    from test_trainer import no_dropout

    from aido1_amd import train_ops
    from aido1_amd.actor import ConfigCritic
    cfg = golden('reference_config.json')
    torch.manual_seed(4)
    crit = ConfigCritic(no_dropout(cfg['model']['critic'])).to(gpu).to(memory_format=CL).train()
    obs = torch.rand(16, 3, 120, 160, device=gpu).contiguous(memory_format=CL)
    act = torch.rand(16, 2, device=gpu)

    def run():
        for p in crit.parameters():
            p.grad = None
        q = crit(obs, act)
        q.sum().backward()
        return q.detach().clone(), [p.grad.detach().clone() for p in crit.parameters()]

    state = {k: v.clone() for k, v in crit.state_dict().items()}
    q1, g1 = run()
    crit.load_state_dict(state)
    saved = set(train_ops.UPD_CONV_LAYERS)
    train_ops.UPD_CONV_LAYERS.clear()
    try:
        q0, g0 = run()
    finally:
        train_ops.UPD_CONV_LAYERS.update(saved)
    assert torch.allclose(q1, q0, rtol=1e-4, atol=1e-5)
    for a, b in zip(g1, g0):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-5 * max(1.0, b.abs().max().item()))


@pytest.mark.parametrize('n,updates', [(5, 1), (64, 2)])
def test_trunk_chain_equals_block_path(gpu, n, updates):
    """The conv trunk as one chain (train_ops.conv_trunk: each conv merges the
    previous block's statistics and normalises on load) against the same
    network block by block (dt_upd_conv_fwd_bn + dt_bn_leaky_apply): output,
    running statistics, num_batches_tracked and every gradient bit for bit
    (same partials, merge order and formulas, include/dtupd.h)."""
    from conftest import golden
    from test_trainer import no_dropout

    from aido1_amd import train_ops
    from aido1_amd.actor import ConfigCritic
    cfg = golden('reference_config.json')
    torch.manual_seed(7)
    crit = ConfigCritic(no_dropout(cfg['model']['critic'])).to(gpu).to(memory_format=CL).train()
    obs = torch.rand(n, 3, 120, 160, device=gpu).contiguous(memory_format=CL)
    act = torch.rand(n, 2, device=gpu)
    mods = crit.net.input_nets[0].internal_modules
    assert train_ops.trunk_len(obs, mods, 0, len(mods)) == 4

    def run():
        for p in crit.parameters():
            p.grad = None
        with train_ops.running_updates(crit, updates):
            q = crit(obs, act)
        q.square().sum().backward()
        return (q.detach().clone(), [p.grad.detach().clone() for p in crit.parameters()],
                [b.detach().clone() for b in crit.buffers()])

    state = {k: v.clone() for k, v in crit.state_dict().items()}
    q1, g1, b1 = run()
    crit.load_state_dict(state)
    train_ops.CHAIN = False
    try:
        q0, g0, b0 = run()
    finally:
        train_ops.CHAIN = True
    assert torch.equal(q1, q0)
    for a, b in zip(g1, g0):
        assert torch.equal(a, b)
    for a, b in zip(b1, b0):
        assert torch.equal(a, b)
    assert int(b1[-1]) == updates                     # num_batches_tracked of the last BN


def test_chain_rejects_bad_handoff(gpu):
    from aido1_amd import _lib
    L = _lib.lib()
    b = _lib.DtUpdBn()                                # all NULL
    import ctypes
    parts = ctypes.c_int32(0)
    x = torch.zeros(1, 57, 77, 32, device=gpu)
    assert L.dt_upd_conv_fwd_part(32, 4, 2, 1, 57, 77, x.data_ptr(), ctypes.byref(b), x.data_ptr(),
                                  x.data_ptr(), 0.01, x.data_ptr(), x.data_ptr(),
                                  ctypes.byref(parts), None) != 0
    assert L.dt_upd_bn_finish(1, 0, x.data_ptr(), ctypes.byref(b), x.data_ptr(), None) != 0


@pytest.mark.parametrize('slope', [None, 0.01])
@pytest.mark.parametrize('m,n,k', [(64, 256, 4032), (5, 256, 4032), (33, 64, 1024)])
def test_linear_matches_f64(gpu, m, n, k, slope):
    """The split-K linear kernels (dt_upd_linear_*) against float64 torch:
    forward with bias, dx, dw and db (the critic's 4032 -> 256 layer at batch
    64, a ragged batch, another shape), alone and with the LeakyReLU after it
    fused (its gradient from the output)."""
    from aido1_amd import train_ops
    g = torch.Generator().manual_seed(m + n)
    x = torch.randn(m, k, generator=g, dtype=torch.float64)
    w = torch.randn(n, k, generator=g, dtype=torch.float64) / k ** 0.5
    b = torch.randn(n, generator=g, dtype=torch.float64)
    dy = torch.randn(m, n, generator=g, dtype=torch.float64)
    xg = x.float().to(gpu).requires_grad_()
    lin = torch.nn.Linear(k, n).to(gpu)
    with torch.no_grad():
        lin.weight.copy_(w)
        lin.bias.copy_(b)
    assert train_ops.linear_applicable(xg, lin)
    y = train_ops.linear(xg, lin, slope)
    y.backward(dy.float().to(gpu))
    ref = x @ w.T + b
    if slope is not None:
        ref = torch.where(ref > 0, ref, ref * slope)
        # the gradient's mask is the f32 output's sign (a pre-activation within
        # rounding of zero may fall either side; its value is then ~0 anyway)
        dy = torch.where(y.detach().double().cpu() > 0, dy, dy * slope)
    assert (y.detach().double().cpu() - ref).abs().max().item() <= _bound((x.abs() @ w.abs().T).max().item())
    assert (xg.grad.double().cpu() - dy @ w).abs().max().item() <= _bound((dy.abs() @ w.abs()).max().item())
    assert (lin.weight.grad.double().cpu() - dy.T @ x).abs().max().item() <= \
        _bound((dy.abs().T @ x.abs()).max().item())
    assert (lin.bias.grad.double().cpu() - dy.sum(0)).abs().max().item() <= \
        _bound(dy.abs().sum(0).max().item())


@pytest.mark.parametrize('m,slope,p', [(64, 0.01, 0.5), (37, None, 0.25)])
def test_linear_dropout_folded_matches_f64(gpu, m, slope, p):
    """Dropout folded into the split-K linear (dt_upd_linear_*_drop): the
    forward, dx, dw and db against float64 torch of x * {u >= p} / (1 - p)
    through the same linear (F.dropout's bernoulli(1 - p) mask made from the
    same uniforms u), at the config's flatten width."""
    from aido1_amd import train_ops
    n, k = 256, 4032
    g = torch.Generator().manual_seed(m)
    x = torch.randn(m, k, generator=g, dtype=torch.float64)
    w = torch.randn(n, k, generator=g, dtype=torch.float64) / k ** 0.5
    b = torch.randn(n, generator=g, dtype=torch.float64)
    dy = torch.randn(m, n, generator=g, dtype=torch.float64)
    u = torch.rand(m, k, generator=g, dtype=torch.float32)
    keep = (u >= p).double() / (1.0 - p)
    xg = x.float().to(gpu).requires_grad_()
    lin = torch.nn.Linear(k, n).to(gpu)
    with torch.no_grad():
        lin.weight.copy_(w)
        lin.bias.copy_(b)
    with train_ops.drop_pool(1, m, k, gpu) as pool:
        pool.copy_(u.to(gpu).unsqueeze(0))
        y = train_ops.linear(xg, lin, slope, drop=p)
    y.backward(dy.float().to(gpu))
    xd = x * keep
    ref = xd @ w.T + b
    if slope is not None:
        ref = torch.where(ref > 0, ref, ref * slope)
        dy = torch.where(y.detach().double().cpu() > 0, dy, dy * slope)
    assert (y.detach().double().cpu() - ref).abs().max().item() <= \
        _bound((xd.abs() @ w.abs().T).max().item())
    assert (xg.grad.double().cpu() - (dy @ w) * keep).abs().max().item() <= \
        _bound((dy.abs() @ w.abs()).max().item() * 2.0)
    assert (lin.weight.grad.double().cpu() - dy.T @ xd).abs().max().item() <= \
        _bound((dy.abs().T @ xd.abs()).max().item())
    assert (lin.bias.grad.double().cpu() - dy.sum(0)).abs().max().item() <= \
        _bound(dy.abs().sum(0).max().item())
    # the dropped elements' gradient is exactly zero, the kept ones scaled
    dx = xg.grad.cpu()
    assert torch.all(dx[u < p] == 0)


def test_linear_dropout_site_draws_fresh_uniforms(gpu):
    """Outside a pool every folded dropout draws its own uniforms; inside one
    the sites take consecutive slices and a site past its end draws its own."""
    from aido1_amd import train_ops
    x = torch.ones(8, 1024, device=gpu)
    a = train_ops.drop_uniforms(x)
    bb = train_ops.drop_uniforms(x)
    assert a.shape == x.shape and not torch.equal(a, bb)
    with train_ops.drop_pool(2, 8, 1024, gpu) as pool:
        s0, s1, s2 = (train_ops.drop_uniforms(x) for _ in range(3))
        assert s0.data_ptr() == pool[0].data_ptr() and s1.data_ptr() == pool[1].data_ptr()
        assert s2.data_ptr() not in (pool[0].data_ptr(), pool[1].data_ptr())
    assert train_ops._DROP['pool'] is None
