"""Non-finite guards (aido1_amd/guard.py, SURVEY.md §5 failure detection) on
the CPU trainer: a NaN injected at each stage of the DDPG update
(training/trainers.py:143-237) is reported under that stage's name, and it is
the first stage named at the earliest tick.  The GPU kernels' own reports
(fused BatchNorm, dt_adam, dt_guard_scan) are tests/test_gpu_guard.py."""
import math

import pytest
import torch

from test_trainer import formula_batch, make_trainer

from aido1_amd.guard import STAGES, Guard, NonFiniteError

NAN = float('nan')


def _first_stage(err):
    """The stage the message names first at its earliest tick."""
    msg = str(err)
    parts = msg.split('non-finite values at ')[1].split('; earliest tick ')
    earliest = int(parts[1].split(',')[0])
    named = [p.strip() for p in parts[0].split('),')]
    for n in named:
        name, tick = n.split(' (first at tick ')
        if int(tick.rstrip(')')) == earliest:
            return name
    raise AssertionError(msg)


def _poison(p):
    with torch.no_grad():
        p[(0,) * p.dim()] = NAN


def _batch_with(**nan):
    obs, act, rew, nxt, done = formula_batch(8)
    obs, act, rew, nxt = (torch.as_tensor(v, dtype=torch.float64).clone()
                          for v in (obs, act, rew, nxt))
    if nan.get('obs'):
        obs[3, 1, 7, 9] = NAN
    return obs, act, rew, nxt, done


def _run(tr, batch, updates=2):
    for _ in range(updates):
        tr.update(batch)
    with pytest.raises(NonFiniteError) as e:
        tr.check()
    return _first_stage(e.value)


def _trainer():
    return make_trainer('cpu', double=True)


def test_clean_update_passes():
    tr = _trainer()
    for _ in range(2):
        tr.update(_batch_with())
    r = tr.check()
    assert r['stages'] == [] and r['tick'] == 2


def test_batch_nan_named():
    assert _run(_trainer(), _batch_with(obs=True)) == 'batch'


def test_target_nan_named():
    tr = _trainer()
    _poison(next(tr.target_critic.parameters()))
    assert _run(tr, _batch_with()) == 'target'


def test_critic_loss_nan_named():
    tr = _trainer()
    _poison(list(tr.critic.parameters())[-1])     # the output bias
    assert _run(tr, _batch_with()) == 'critic_loss'


@pytest.mark.parametrize('net', ['critic', 'actor'])
def test_grad_nan_named(net):
    tr = _trainer()
    p = next(getattr(tr, net).parameters())
    p.register_hook(lambda g: g * NAN)
    assert _run(tr, _batch_with()) == net + '_grad'


@pytest.mark.parametrize('net', ['critic', 'actor'])
def test_param_nan_named(net):
    """A NaN learning rate: finite gradients, non-finite parameters."""
    tr = _trainer()
    getattr(tr, net + '_decay').decays['lr'] = lambda step: NAN
    assert _run(tr, _batch_with(), updates=1) == net + '_param'


def test_actor_loss_nan_named():
    tr = _trainer()
    _poison(list(tr.actor.parameters())[-1])
    assert _run(tr, _batch_with(), updates=1) == 'actor_loss'


def test_td_nan_named():
    """The TD-error forward (no_grad, trainers.py:223-229) alone made NaN."""
    tr = _trainer()
    tr.critic.register_forward_hook(
        lambda m, i, out: out * NAN if not torch.is_grad_enabled() else None)
    assert _run(tr, _batch_with(), updates=1) == 'td'


def test_first_tick_recorded():
    tr = _trainer()
    tr.update(_batch_with())
    tr.update(_batch_with(obs=True))
    with pytest.raises(NonFiniteError) as e:
        tr.check()
    assert 'batch (first at tick 2)' in str(e.value)
    assert 'critic_param (first at tick 2)' in str(e.value)
    # check() cleared the block: the poisoned networks report from tick 3 on
    tr.update(_batch_with())
    with pytest.raises(NonFiniteError) as e:
        tr.check()
    assert 'earliest tick 3' in str(e.value) and 'batch' not in str(e.value)


def test_guard_names_every_stage():
    g = Guard('cpu')
    for bit in STAGES:
        g.scan(bit, torch.tensor([1.0, math.inf]))
    r = g.read()
    assert [s for s, _ in r['stages']] == [STAGES[b] for b in sorted(STAGES)]
    assert r['count'] == len(STAGES)
