"""DDPG update and the full training loop on the GPU.

The update is compared with the reference's own DDPGTrainer.update
(tests/golden/ddpg_update.json, run on CPU in float32).  Tolerance: the GPU
convolutions (MIOpen) sum in a different order than CPU ones, so losses and
TD errors agree to ~1e-5 relative; parameters after three Adam steps agree to
rtol 1e-3 / atol 1e-3 (Adam's first steps move each weight by ~lr * sign(g),
so a gradient within rounding noise of zero may step the other way)."""
import pytest
import torch

from conftest import golden
from test_trainer import check_against_reference, formula_batch, make_trainer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('graph', [False, True])
def test_update_matches_reference_gpu(gpu, graph):
    """graph=True: update 1 eager, updates 2-3 replay the captured HIP graph."""
    torch.backends.cudnn.allow_tf32 = False
    tr = make_trainer(gpu, graph=graph, warmup=1)
    check_against_reference(tr, formula_batch(16), rtol=1e-3, atol=1e-3)
    if graph:
        assert tr._graphs is not None and len(tr._graphs) == 1


@pytest.mark.parametrize('prioritized,graph,size', [(True, True, 1000), (False, False, 1000),
                                                     (True, True, 1024)])
def test_train_loop_runs(gpu, prioritized, graph, size):
    """size 1024 = 8 decisions of 128 envs: the frame store (replay.py)."""
    from aido1_amd.train_loop import TrainLoop
    cfg = golden('reference_config.json')
    loop = TrainLoop(cfg, n_envs=128, device=0, seed=5, buffer_size=size, batch_size=32,
                     prioritized=prioritized, graph=graph)
    assert (loop.replay.frame_envs is not None) == (size == 1024)
    w0 = loop.trainer.actor.net.input_nets[0].internal_modules[0].kernel.weight.detach().clone()
    t0 = loop.rollout.actor.w[1].detach().clone()
    loop.reset()
    for _ in range(12):
        loop.step()
    # the guards name the first stage that produced NaN / Inf (and the
    # replay's rejected priorities), before any assertion on the results
    try:
        rec = loop.check()
    except Exception:
        from test_gpu_guard import _report_rollout_state
        _report_rollout_state(loop)
        raise
    assert rec['tick'] == 12
    assert len(loop.replay) == size and loop.updates == 12 and loop.decisions == 12
    assert torch.isfinite(loop.metrics['critic_loss']) and torch.isfinite(loop.metrics['actor_loss'])
    w1 = loop.trainer.actor.net.input_nets[0].internal_modules[0].kernel.weight
    assert not torch.equal(w0, w1)
    # the exploring envs act with the online actor, the exploiters with the
    # target actor (train_loop._refresh)
    assert not torch.equal(t0, loop.rollout.actor.w[1])
    for mine, src in ((loop.rollout.actor, loop.trainer.actor),
                      (loop.rollout.exploit_actor, loop.trainer.target_actor)):
        k = src.net.input_nets[0].internal_modules[0].kernel.weight
        assert torch.equal(mine.w[0].float(), k.detach().to(mine.w[0].dtype).float())
    st = loop.replay.storage
    if size == 1024:
        obs, act, rew, nxt, done = loop.replay._encode_sample(torch.arange(size, device=gpu))
        p = loop.replay._next_idx          # 12 decisions of 128 rows: 512
        assert p == 512
        # the last decision's next_obs is the rollout's current stack
        assert torch.equal(nxt[p - 128:p], loop.rollout.stack())
        # obs of a decision = next_obs of the env's previous decision
        assert torch.equal(obs[p - 128:p], nxt[p - 256:p - 128])
        assert obs.shape == (size, 3, 120, 160) and st['action'].shape == (size, 2)
    else:
        assert st['obs'].shape == (1000, 3, 120, 160) and st['action'].shape == (1000, 2)
    assert float(st['action'].min()) >= 0.0                  # mapped a/2 + 0.5 stored
    if prioritized:
        loop.replay.check()
        _, _, mp = loop.replay.trees()
        assert mp.item() >= 1.0
    assert loop.rollout.stats()['decisions'] == 128 * 12


@pytest.mark.parametrize('graph', [False, True])
def test_two_stream_stages_equal_one_stream(gpu, graph):
    """The update's side-stream branches (trainer._fork: the targets' forward
    beside the critic's, the stepped critic's trunk beside the actor's
    forward, the TD forward beside the actor step and soft updates) against
    the same update with every stage on one stream: losses, TD errors and
    every state_dict entry (weights, BatchNorm running statistics) bit for
    bit over three updates, eager and captured as HIP graphs (two graph
    branches vs a chain).  Holds because no BatchNorm module is forwarded on
    both branches (its kernels' scratch is per module, train_ops)."""
    torch.backends.cudnn.allow_tf32 = False
    two = make_trainer(gpu, graph=graph, warmup=1)
    one = make_trainer(gpu, graph=graph, warmup=1)
    one._fork = lambda: None
    batch = formula_batch(16)
    for _ in range(3):
        m2, i2 = two.update(batch)
        m1, i1 = one.update(batch)
        torch.cuda.synchronize()
        for k in ('critic_loss', 'actor_loss'):
            assert torch.equal(m1[k], m2[k]), k
        assert torch.equal(i1['td_error'], i2['td_error'])
    for a, b in ((two.actor, one.actor), (two.critic, one.critic),
                 (two.target_actor, one.target_actor), (two.target_critic, one.target_critic)):
        sa, sb = a.state_dict(), b.state_dict()
        for k in sa:
            assert torch.equal(sa[k], sb[k]), k
    if graph:
        assert two._graphs is not None and one._graphs is not None
