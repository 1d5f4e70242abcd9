"""Non-finite guards on the GPU (aido1_amd/guard.py, include/dttrain.h):
dt_guard_scan itself, the fused BatchNorm's in-kernel reports (non-finite
statistics; a lost partial, i.e. the merged pixel count != m), dt_adam's, and
the stage names the graph-mode update and the training loop report.  The CPU
restatement of the stage order is tests/test_guard.py."""
import ctypes

import pytest
import torch

from test_trainer import formula_batch, make_trainer

from aido1_amd.guard import BIT, Guard, NonFiniteError

pytestmark = pytest.mark.gpu
NAN, INF = float('nan'), float('inf')


def _stages(g):
    return [s for s, _ in g.read()['stages']]


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('n,at', [(1, 0), (7, 6), (4099, 4098), (1 << 20, 12345), (1 << 20, None)])
def test_scan_finds_every_position(gpu, dtype, n, at):
    g = Guard(gpu)
    x = torch.randn(n + 1, device=gpu, dtype=dtype)[1:]      # misaligned for float32
    if at is not None:
        x[at] = NAN if at % 2 else INF
    g.scan('batch', x, torch.ones(3, device=gpu))
    assert _stages(g) == ([] if at is None else ['batch'])


def test_scan_many_tensors_one_bit_each(gpu):
    g = Guard(gpu)
    ts = [torch.zeros(100, device=gpu) for _ in range(11)]     # two launches (8 + 3)
    ts[9][50] = NAN
    g.scan('td', *ts)
    g.scan('actor_loss', *ts[:9])
    assert _stages(g) == ['td']
    g.clear()
    assert _stages(g) == []


def _bn_call(gpu, z, work, guard):
    from aido1_amd import _lib
    L = _lib.lib()
    c = 32
    bias, gamma, beta = (torch.zeros(c, device=gpu), torch.ones(c, device=gpu),
                         torch.zeros(c, device=gpu))
    rm, rv = torch.zeros(c, device=gpu), torch.ones(c, device=gpu)
    y = torch.empty_like(z)
    mi = torch.empty(2 * c, device=gpu)
    rc = L.dt_bn_leaky_fwd(z.numel() // c, z.data_ptr(), bias.data_ptr(), 0.01, gamma.data_ptr(),
                           beta.data_ptr(), 1e-5, 0.1, rm.data_ptr(), rv.data_ptr(), None, 1, None,
                           y.data_ptr(), mi.data_ptr(), work.data_ptr(), guard.ptr(),
                           ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream))
    assert rc == 0
    return y, mi


def test_bn_reports_nonfinite_statistics(gpu):
    from aido1_amd import _lib
    g = Guard(gpu)
    work = torch.zeros(int(_lib.lib().dt_train_work_floats(0)), device=gpu)
    z = torch.randn(64 * 57 * 77, 32, device=gpu)
    _bn_call(gpu, z, work, g)
    assert _stages(g) == []
    z[1000, 5] = NAN
    _bn_call(gpu, z, work, g)
    assert _stages(g) == ['bn_fwd']


def test_bn_reports_a_lost_partial(gpu):
    """A counter left at grid - 1 makes the FIRST workgroup to finish the
    merger: the other partials are missing (their counts were zeroed by the
    previous merge), and the merged count != m is reported."""
    from aido1_amd import _lib
    g = Guard(gpu)
    work = torch.zeros(int(_lib.lib().dt_train_work_floats(0)), device=gpu)
    m = 64 * 57 * 77
    z = torch.randn(m, 32, device=gpu)
    y0, mi0 = _bn_call(gpu, z, work, g)               # a clean launch first
    assert _stages(g) == []
    grid = min(256, (m * 8 + 2047) // 2048)
    counters = work.view(torch.int32)[256 * 32 * 3:]
    counters[0] = grid - 1
    _bn_call(gpu, z, work, g)
    assert 'bn_count' in _stages(g)


def test_adam_reports_grad_and_param(gpu):
    from aido1_amd.optim import DeviceAdam
    g = Guard(gpu)
    p = torch.nn.Parameter(torch.randn(5000, device=gpu))
    opt = DeviceAdam([p], gpu)
    opt.set_guard(g, 'critic_grad', 'critic_param')
    opt.param_groups[0]['lr'].fill_(1e-3)
    p.grad = torch.randn_like(p)
    opt.step()
    assert _stages(g) == []
    p.grad[4097] = INF
    opt.step()
    assert _stages(g) == ['critic_grad', 'critic_param']


@pytest.mark.parametrize('graph', [False, True])
def test_update_names_the_batch(gpu, graph):
    """A NaN observation in a graph-replayed update: 'batch' comes first at
    its tick, and the fused BatchNorm reports its statistics too."""
    torch.backends.cudnn.allow_tf32 = False
    tr = make_trainer(gpu, graph=graph, warmup=1)
    clean = formula_batch(16)
    for _ in range(2):
        tr.update(clean)
    assert tr.check()['tick'] == 2
    obs = torch.as_tensor(clean[0]).clone()
    obs[2, 0, 10, 10] = NAN
    tr.update((obs,) + tuple(clean[1:]))
    with pytest.raises(NonFiniteError) as e:
        tr.check()
    msg = str(e.value)
    assert msg.split('non-finite values at ')[1].startswith('batch (first at tick 3)')
    assert 'bn_fwd (first at tick 3)' in msg


def test_train_loop_names_the_actor_output(gpu):
    """NaN acting weights: the rollout's actor outputs are named first (the
    tanh clip of DDPG.act would otherwise turn NaN into -1)."""
    from conftest import golden

    from aido1_amd.train_loop import TrainLoop
    loop = TrainLoop(golden('reference_config.json'), n_envs=128, device=0, seed=5,
                     buffer_size=1024, batch_size=32, graph=True)
    loop.reset()
    for _ in range(3):
        loop.step()
    try:
        rec = loop.check()
    except NonFiniteError:
        _report_rollout_state(loop)
        raise
    assert rec['tick'] == 3
    bad = loop.trainer.actor.net.input_nets[0].internal_modules[0].kernel.weight.detach().clone()
    bad[0, 0, 0, 0] = NAN
    loop.rollout.actor.refresh(_with_conv1(loop.trainer.actor, bad))
    loop.step()
    with pytest.raises(NonFiniteError) as e:
        loop.check()
    assert str(e.value).split('non-finite values at ')[1].startswith('actor_out')
    assert BIT['actor_out'] == 0


def _report_rollout_state(loop):
    """Which of the rollout's tensors hold NaN / Inf (printed on failure)."""
    r = loop.rollout
    named = [('ring', r.ring), ('actor_out', r.actor_out), ('actions', r.actions)]
    for tag, a in (('actor', r.actor), ('exploit', r.exploit_actor)):
        if a is None:
            continue
        named += [(tag + '.' + k, v) for k, v in a.named_parameters()]
        named += [(tag + '.' + k, v) for k, v in a.named_buffers()]
        named += [(tag + '._bufs.' + k, v) for k, v in (getattr(a, '_bufs', None) or {}).items()
                  if v is not None]
    named += [('trainer.actor.' + k, v) for k, v in loop.trainer.actor.named_parameters()]
    for k, v in named:
        bad = (~torch.isfinite(v.float())).sum().item()
        if bad:
            rows = (~torch.isfinite(v.float().reshape(v.shape[0], -1))).any(1).nonzero()
            print('NONFINITE %s shape %s: %d elements, rows %s' % (k, tuple(v.shape), bad,
                                                                 rows.flatten()[:16].tolist()))


def _with_conv1(actor, w):
    import copy
    a = copy.deepcopy(actor)
    with torch.no_grad():
        a.net.input_nets[0].internal_modules[0].kernel.weight.copy_(w)
    return a
