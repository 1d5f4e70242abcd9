"""Host logic of the replay buffers on CPU tensors (uniform ReplayBuffer:
utils/buffers.py:12-137), checked against the oracle's index restatement."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle.per_ref import uniform_indices


def _batch(k0, n):
    k = torch.arange(k0, k0 + n, dtype=torch.float32)
    return k.view(n, 1, 1).expand(n, 3, 4).contiguous(), torch.stack([k, -k], 1), k.double(), \
        k.view(n, 1, 1).expand(n, 3, 4) + 1, (k.long() % 5 == 0)


def test_uniform_buffer_add_wrap_and_sample():
    from aido1_amd.replay import ReplayBuffer
    rb = ReplayBuffer(10, device='cpu')
    rb.add_batch(*_batch(0, 4))
    rb.add(*[t[0] for t in _batch(4, 1)])       # single add, reference signature
    assert len(rb) == 5 and rb._next_idx == 5
    rb.add_batch(*_batch(5, 23))                 # wraps twice, later adds win
    assert len(rb) == 10 and rb._next_idx == 8
    # slot s holds the last item k with k % 10 == s among 0..27
    expect = {s: max(k for k in range(28) if k % 10 == s) for s in range(10)}
    assert [int(v) for v in rb.storage['reward']] == [expect[s] for s in range(10)]
    u = np.random.default_rng(0).random(64)
    obs, act, rew, nxt, done = rb.sample(64, u=u)
    idx = uniform_indices(u, len(rb))
    assert [int(v) for v in rew] == [expect[i] for i in idx]
    assert torch.equal(nxt, obs + 1) and torch.equal(act[:, 1], -act[:, 0])
    assert torch.equal(done, rew.long() % 5 == 0)
    assert obs.shape == (64, 3, 4)


def test_obs_dtype_narrowing():
    from aido1_amd.replay import ReplayBuffer
    rb = ReplayBuffer(8, device='cpu', obs_dtype=torch.bfloat16)
    rb.add_batch(*_batch(0, 3))
    assert rb.storage['obs'].dtype == torch.bfloat16 and rb.storage['action'].dtype == torch.float32


def test_create_buffer_reads_config():
    from aido1_amd.replay import ReplayBuffer, create_buffer
    cfg = golden('reference_config.json')
    rb = create_buffer(cfg, device='cpu')
    assert isinstance(rb, ReplayBuffer) and rb._maxsize == cfg['training']['buffer_size']


def test_sample_empty_raises():
    from aido1_amd.replay import ReplayBuffer
    with pytest.raises(ValueError):
        ReplayBuffer(4, device='cpu').sample(2)


def test_add_batch_ring_equals_add_batch():
    """add_batch_ring (next_obs straight from a frame ring in stack order, the
    returned rows chained as the next obs) stores what add_batch of the
    stacked copies stores, across the wrap of the buffer."""
    from aido1_amd.replay import ReplayBuffer
    g = torch.Generator().manual_seed(0)
    n, size = 3, 8
    a, b = ReplayBuffer(size, device='cpu'), ReplayBuffer(size, device='cpu')
    ring = torch.rand(n, 3, 2, 2, generator=g)
    obs_a = obs_b = ring[:, [0, 1, 2]].clone()
    for t in range(7):
        order = [(t + 1 + k) % 3 for k in range(3)]
        ring[:, order[-1]] = torch.rand(n, 2, 2, generator=g)   # the newest frame
        act = torch.rand(n, 2, generator=g)
        rew = torch.rand(n, generator=g, dtype=torch.float64)
        done = torch.rand(n, generator=g) < 0.3
        nxt = ring[:, order]
        b.add_batch(obs_b, act, rew, nxt, done)
        obs_b = nxt
        obs_a = a.add_batch_ring(obs_a, act, rew, ring, order, done)
        assert torch.equal(obs_a, obs_b)
    assert a._next_idx == b._next_idx and len(a) == len(b)
    for k in a.storage:
        assert torch.equal(a.storage[k], b.storage[k]), k


def _frame_steps(a, b, n, steps, g, per=False, index=False):
    """Feed a (frame store) and b (stacked storage) the same decisions of a
    frame ring with the rollout's semantics: one new frame a decision in the
    slot order advances, and a respawned env's whole stack is its new frame
    (the renderer's fresh refill).  index=True: a ring of palette-index
    frames (u8 [4, 8]; b gets their grey frames).  Yields after every
    decision."""
    from aido1_amd.render import as_gray
    dev = a.device
    shape = (4, 8) if index else (2, 4)

    def frames(*lead):
        if index:
            return torch.randint(0, 8, lead + shape, generator=g, dtype=torch.uint8)
        return torch.rand(lead + shape, generator=g)
    ring = frames(n, 3).to(dev)
    obs_a = ring[:, [0, 1, 2]].clone()
    obs_b = as_gray(obs_a)
    for t in range(steps):
        order = [(t + 1 + k) % 3 for k in range(3)]
        done = (torch.rand(n, generator=g) < 0.3).to(dev)
        new = frames(n).to(dev)
        ring[:, order[-1]] = new
        ring[done] = new[done, None]
        act = torch.rand(n, 2, generator=g).to(dev)
        rew = torch.rand(n, generator=g, dtype=torch.float64).to(dev)
        nxt = as_gray(ring[:, order].clone())
        b.add_batch(obs_b, act, rew, nxt, done)
        obs_b = nxt
        obs_a = a.add_batch_ring(obs_a, act, rew, ring, order, done)
        assert obs_a is None
        yield t


@pytest.mark.parametrize('index', [False, True])
def test_frame_store_samples_equal_stacked_storage(index):
    """The frame store (frame_envs: one frame per env a decision plus frame
    indices) returns the stacks the stacked storage (buffers.py:29-52) returns
    for the same indices, across many wraps of the buffer and respawns; a
    palette-index ring is stored as bytes and sampled as its grey frames."""
    from aido1_amd.replay import ReplayBuffer
    g = torch.Generator().manual_seed(1)
    n, size = 3, 9
    a = ReplayBuffer(size, device='cpu', frame_envs=n)
    b = ReplayBuffer(size, device='cpu')
    for _ in _frame_steps(a, b, n, 13, g, index=index):
        assert len(a) == len(b) and a._next_idx == b._next_idx
        u = torch.rand(32, generator=g, dtype=torch.float64)
        for x, y in zip(a.sample(32, u=u), b.sample(32, u=u)):
            assert torch.equal(x, y)
    # every row, not only sampled ones
    idx = torch.arange(size)
    for x, y in zip(a._encode_sample(idx), b._encode_sample(idx)):
        assert torch.equal(x, y)
    assert a.frames.shape[0] == (size // n + 6) * n   # 2k blocks beyond the transitions'


def test_frame_store_rejects():
    from aido1_amd.replay import ReplayBuffer
    with pytest.raises(ValueError):
        ReplayBuffer(10, device='cpu', frame_envs=3)          # must divide size
    with pytest.raises(ValueError):
        ReplayBuffer(9, device='cpu', frame_envs=3, obs_dtype=torch.bfloat16)
    rb = ReplayBuffer(9, device='cpu', frame_envs=3)
    with pytest.raises(ValueError):
        rb.add_batch(*_batch(0, 3))
    ring = torch.zeros(3, 3, 2, 2)
    with pytest.raises(ValueError):                            # the first add needs obs_t
        rb.add_batch_ring(None, torch.zeros(3, 2), torch.zeros(3), ring, [0, 1, 2],
                          torch.zeros(3, dtype=torch.bool))


def _begin_steps(a, b, n, begins, g):
    """As _frame_steps, but a new observation chain (a rollout reset: obs_t
    given again, a fresh stack) at every decision in `begins`."""
    ring = torch.rand(n, 3, 2, 4, generator=g)
    obs_b = ring[:, [0, 1, 2]].clone()
    for t in range(max(begins) + 4):
        if t in begins:
            ring = torch.rand(n, 3, 2, 4, generator=g)
            obs_b = ring[:, [(t + k) % 3 for k in range(3)]].clone()
        order = [(t + 1 + k) % 3 for k in range(3)]
        new = torch.rand(n, 2, 4, generator=g)
        ring[:, order[-1]] = new
        done = torch.zeros(n, dtype=torch.bool)
        act, rew = torch.rand(n, 2, generator=g), torch.rand(n, generator=g, dtype=torch.float64)
        nxt = ring[:, order].clone()
        b.add_batch(obs_b, act, rew, nxt, done)
        a.add_batch_ring(obs_b if (t in begins or t == 0) else None, act, rew, ring, order, done)
        obs_b = nxt
        idx = torch.arange(len(b))
        for x, y in zip(a._encode_sample(idx), b._encode_sample(idx)):
            assert torch.equal(x, y), t


@pytest.mark.parametrize('begins,raises_at', [
    ((0, 1, 2), 2),          # 3 chains in 3 decisions, buffer not full: would wrap
    ((0, 1), None),          # within the 2k spare blocks
    ((0, 4, 8, 12), None),   # one chain per size / n decisions: always safe
    ((0, 4, 5), 5),          # full buffer: the reset before still referenced
    ((0, 2, 3), 3),
])
def test_frame_store_chain_begins_checked_against_live_frames(begins, raises_at):
    """A new chain writes k frame blocks; the store refuses one that would
    overwrite blocks that stored transitions still reference, whether or not
    the buffer is full (size 12, n 3: 4 decisions, 4 + 2k = 10 blocks), and
    every accepted pattern samples what the stacked storage holds."""
    from aido1_amd.replay import ReplayBuffer
    g = torch.Generator().manual_seed(3)
    a = ReplayBuffer(12, device='cpu', frame_envs=3)
    b = ReplayBuffer(12, device='cpu')
    if raises_at is None:
        _begin_steps(a, b, 3, begins, g)
        return
    with pytest.raises(ValueError, match='still reference'):
        _begin_steps(a, b, 3, begins, g)
    assert a._decisions == raises_at
