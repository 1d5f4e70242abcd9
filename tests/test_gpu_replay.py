"""GPU prioritized replay (csrc/dtreplay.hip through include/dtreplay.h) against
the reference's PrioritizedReplayBuffer (golden op sequences) and the oracle
at full size.  Sampled indices must be identical for the same uniforms; the
trees are compared bit for bit."""
import math

import numpy as np
import pytest
import torch

from conftest import golden
from oracle.per_ref import PrioritizedReplayRef

pytestmark = pytest.mark.gpu


def _payload(items, dev):
    k = torch.tensor(items, dtype=torch.float32, device=dev)
    n = k.numel()
    return k.view(n, 1), torch.stack([k, -k], 1), k.double(), (k + 1).view(n, 1), \
        (k.long() % 5 == 0)


def _inf(v):
    return math.inf if v is None else v


def assert_trees(st, mt, ref_sum, ref_min):
    st, mt = st.cpu().numpy(), mt.cpu().numpy()
    ref_sum = np.asarray(ref_sum, np.float64)
    ref_min = np.asarray([_inf(v) for v in ref_min], np.float64)
    cap = st.size // 2
    leaf = slice(cap, 2 * cap)
    np.testing.assert_allclose(st[leaf], ref_sum[leaf], rtol=4.5e-16, atol=0)
    np.testing.assert_allclose(mt[leaf], ref_min[leaf], rtol=4.5e-16, atol=0)
    node = np.arange(1, cap)
    assert np.array_equal(st[node], st[2 * node] + st[2 * node + 1])          # exact recurrence
    l, r = mt[2 * node], mt[2 * node + 1]
    assert np.array_equal(mt[node], np.where(r < l, r, l))                    # Python min(l, r)
    np.testing.assert_allclose(st[1:cap], ref_sum[1:cap], rtol=1e-15)
    np.testing.assert_allclose(mt[1:cap], ref_min[1:cap], rtol=4.5e-16)


def test_per_matches_reference_op_sequences(gpu):
    from aido1_amd.replay import PrioritizedReplayBuffer
    for case in golden('prioritized_replay.json'):
        rb = PrioritizedReplayBuffer(case['size'], case['alpha'], device=gpu)
        assert rb.capacity == case['capacity']
        for op in case['ops']:
            rb.add_batch(*_payload(op['add'], gpu))
            if 'sample' in op:
                s = op['sample']
                obs, act, rew, nxt, done, w, idx = rb.sample(s['batch'], beta=s['beta'], u=s['u'])
                assert idx.tolist() == s['idx']
                assert obs.view(-1).long().tolist() == s['obs']
                np.testing.assert_allclose(w.cpu().numpy(), s['weights'], rtol=1e-13, atol=0)
                rb.update_priorities(op['update']['idx'], op['update']['priorities'])
            rb.check()
            st, mt, mp = rb.trees()
            assert len(rb) == op['len'] and rb._next_idx == op['next_idx']
            assert mp.item() == op['max_priority']
            assert_trees(st, mt, op['sum_tree'], op['min_tree'])
        rb.close()


def test_per_full_size_against_oracle(gpu):
    """BASELINE config 5 shape: 4096 transitions per add, batched updates with
    duplicate indices, 4096-wide samples; capacity 2^17."""
    from aido1_amd.replay import PrioritizedReplayBuffer
    size, alpha, beta, n = 100_000, 0.6, 0.4, 4096
    rb = PrioritizedReplayBuffer(size, alpha, device=gpu)
    ref = PrioritizedReplayRef(size, alpha)
    rng = np.random.default_rng(5)
    obs = torch.zeros(n, 1, device=gpu)
    act = torch.zeros(n, 2, device=gpu)
    rew = torch.zeros(n, dtype=torch.float64, device=gpu)
    done = torch.zeros(n, dtype=torch.bool, device=gpu)
    for it in range(30):                      # 122880 adds: wraps the 100000 ring
        rb.add_batch(obs, act, rew, obs, done)
        ref.add(n)
        u = rng.random(n)
        *_, w, idx = rb.sample(n, beta=beta, u=u)
        ridx, rw = ref.sample(u.tolist(), beta)
        assert idx.tolist() == ridx, it
        np.testing.assert_allclose(w.cpu().numpy(), rw, rtol=1e-13)
        upd = idx[torch.from_numpy(rng.integers(0, n, n)).to(gpu)]   # duplicates included
        pr = rng.random(n) * (2.0 + it) + 1e-6
        rb.update_priorities(upd, pr)
        ref.update_priorities(upd.tolist(), pr.tolist())
    rb.check()
    st, mt, mp = rb.trees()
    assert mp.item() == ref.max_priority
    assert_trees(st, mt, ref.it_sum.value, [None if v == math.inf else v for v in ref.it_min.value])
    rb.close()


@pytest.mark.parametrize('size,n,batch', [(131072, 4096, 64), (1000, 96, 128), (4096, 300, 7)])
def test_per_fast_paths_against_oracle(gpu, size, n, batch):
    """The config-5 shapes of add / sample / update: whole-block adds (the
    closed-form add walk; 1000 and 4096 also wrap mid-batch: the level walk),
    batch-64 updates with duplicate indices (the LDS ancestor walk; 128 its
    largest batch), samples through the LDS-staged top levels -- the trees bit
    for bit against the reference's restatement."""
    from aido1_amd.replay import PrioritizedReplayBuffer
    alpha, beta = 0.6, 0.4
    rb = PrioritizedReplayBuffer(size, alpha, device=gpu)
    ref = PrioritizedReplayRef(size, alpha)
    rng = np.random.default_rng(size + n)
    obs = torch.zeros(n, 1, device=gpu)
    act = torch.zeros(n, 2, device=gpu)
    rew = torch.zeros(n, dtype=torch.float64, device=gpu)
    done = torch.zeros(n, dtype=torch.bool, device=gpu)
    for it in range(40):
        rb.add_batch(obs, act, rew, obs, done)
        ref.add(n)
        u = rng.random(batch)
        *_, w, idx = rb.sample(batch, beta=beta, u=u)
        ridx, rw = ref.sample(u.tolist(), beta)
        assert idx.tolist() == ridx, it
        np.testing.assert_allclose(w.cpu().numpy(), rw, rtol=1e-13)
        upd = idx[torch.from_numpy(rng.integers(0, batch, batch)).to(gpu)]   # duplicates
        pr = rng.random(batch) * (2.0 + it) + 1e-6
        rb.update_priorities(upd, pr)
        ref.update_priorities(upd.tolist(), pr.tolist())
        if it % 13 == 12:
            st, mt, mp = rb.trees()
            assert mp.item() == ref.max_priority
            assert_trees(st, mt, ref.it_sum.value,
                         [None if v == math.inf else v for v in ref.it_min.value])
    rb.check()
    st, mt, mp = rb.trees()
    assert_trees(st, mt, ref.it_sum.value, [None if v == math.inf else v for v in ref.it_min.value])
    rb.close()


def test_per_rejects_like_reference_asserts(gpu):
    from aido1_amd._lib import DtError
    from aido1_amd.replay import PrioritizedReplayBuffer
    rb = PrioritizedReplayBuffer(16, 0.6, device=gpu)
    rb.add_batch(*_payload(list(range(4)), gpu))
    rb.update_priorities([1, 2], [0.5, -1.0])          # p <= 0: buffers.py:254
    with pytest.raises(DtError, match='priority'):
        rb.check()
    rb.update_priorities([7], [0.5])                   # idx >= len: buffers.py:255
    with pytest.raises(DtError, match='index'):
        rb.check()
    rb.update_priorities([0, 3, 2], [float('nan'), 0.25, 0.0])   # NaN: counted, not dropped
    with pytest.raises(DtError, match='2 offending entries'):
        rb.check()
    rb.check()                                         # cleared
    st, _, _ = rb.trees()
    assert st[16 + 1].item() == pytest.approx(0.5 ** 0.6, rel=1e-15)   # valid entries applied
    assert st[16 + 3].item() == pytest.approx(0.25 ** 0.6, rel=1e-15)
    one = PrioritizedReplayBuffer(16, 0.6, device=gpu)
    one.add_batch(*_payload([0], gpu))
    with pytest.raises(DtError, match='at least 2'):
        one.sample(4, beta=0.4)


@pytest.mark.parametrize('index', [False, True])
def test_frame_store_gpu_equals_stacked_per(gpu, index):
    """dt_frame_add (include/dtreplay.h) behind PrioritizedReplayBuffer's frame
    store: the same sampled indices, weights and stacks as the stacked
    storage, across wraps and respawns; index=True stores palette-index
    frames (u8, copied as 4-byte words) and samples their grey frames."""
    import sys
    sys.path.insert(0, __import__('os').path.dirname(__file__))
    from test_replay import _frame_steps
    from aido1_amd.replay import PrioritizedReplayBuffer
    g = torch.Generator().manual_seed(3)
    n, size = 256, 1024
    a = PrioritizedReplayBuffer(size, 0.6, device=gpu, frame_envs=n)
    b = PrioritizedReplayBuffer(size, 0.6, device=gpu)
    for t in _frame_steps(a, b, n, 9, g, index=index):
        u = torch.rand(64, generator=g, dtype=torch.float64)
        ra, rb = a.sample(64, 0.4, u=u), b.sample(64, 0.4, u=u)
        for x, y in zip(ra, rb):
            assert torch.equal(x, y)
        pr = torch.rand(64, generator=g, dtype=torch.float64) + 0.1
        a.update_priorities(ra[-1], pr)
        b.update_priorities(rb[-1], pr)
    idx = torch.arange(size, device=gpu)
    for x, y in zip(a._encode_sample(idx), b._encode_sample(idx)):
        assert torch.equal(x, y)


@pytest.mark.parametrize('index', [False, True])
def test_frame_gather_equals_encode_and_trainer_inputs(gpu, index):
    """dt_frame_gather (replay.gather_into) writes exactly what _encode_sample
    followed by DDPGTrainer._inputs makes of the same indices: channels_last
    float32 obs / next_obs, actions, float32 rewards, notdone; also for the
    stacked storage (torch fallback) and indices of every row.  index=True:
    palette-index frames, decoded in the gather (frame_kind 1)."""
    import sys
    sys.path.insert(0, __import__('os').path.dirname(__file__))
    from test_replay import _frame_steps
    from test_trainer import make_trainer
    from aido1_amd.replay import PrioritizedReplayBuffer
    g = torch.Generator().manual_seed(4)
    n, size = 256, 1024
    a = PrioritizedReplayBuffer(size, 0.6, device=gpu, frame_envs=n)
    b = PrioritizedReplayBuffer(size, 0.6, device=gpu)
    for _ in _frame_steps(a, b, n, 7, g, index=index):
        pass
    assert a.frames.dtype == (torch.uint8 if index else torch.float32)
    tr = make_trainer(gpu)
    for buf in (a, b):
        for idx in (torch.arange(size, device=gpu), torch.randint(0, size, (64,), device=gpu)):
            tr._in = None
            tr._inputs(buf._encode_sample(idx))
            want = {k: v.clone() for k, v in tr._in.items()}
            tr._in = None
            got = buf.gather_into(idx, tr.static_inputs(idx.shape[0],
                                                        tuple(want['obs'].shape[1:])))
            for k in want:
                assert torch.equal(got[k], want[k]), k
            assert got['obs'].is_contiguous(memory_format=torch.channels_last)


def test_update_priorities_td_equals_explicit_priorities(gpu):
    """dt_per_update_td (|td| + eps formed in the tree kernel, what TrainLoop
    uses) leaves the trees bit for bit as update_priorities(abs(td) + eps)."""
    from aido1_amd.replay import PrioritizedReplayBuffer
    size, n = 4096, 1024
    bufs = [PrioritizedReplayBuffer(size, 0.6, device=gpu) for _ in range(2)]
    obs = torch.zeros(n, 1, device=gpu)
    act = torch.zeros(n, 2, device=gpu)
    rew = torch.zeros(n, dtype=torch.float64, device=gpu)
    done = torch.zeros(n, dtype=torch.bool, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(7)
    for _ in range(3):
        for b in bufs:
            b.add_batch(obs, act, rew, obs, done)
        idx = torch.randint(0, n, (64,), device=gpu, generator=g)
        td = torch.randn(64, 1, device=gpu, generator=g)
        bufs[0].update_priorities_td(idx, td, 1e-6)
        bufs[1].update_priorities(idx, td.detach().abs().reshape(-1).double() + 1e-6)
    ta, tb = bufs[0].trees(), bufs[1].trees()
    for x, y in zip(ta, tb):
        assert torch.equal(x, y)
    for b in bufs:
        b.check()
        b.close()
