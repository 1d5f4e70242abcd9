"""HBM-resident replay buffers with the reference's API (utils/buffers.py).

* ``ReplayBuffer`` — buffers.py:12-137 (what ``create_buffer`` returns,
  buffers.py:7-9): ring of ``size`` transitions, uniform ``sample``.
* ``PrioritizedReplayBuffer`` — buffers.py:140-259: the sum/min segment trees
  and the proportional sampling run in the gfx950 kernels of
  csrc/dtreplay.hip (include/dtreplay.h); nothing leaves the GPU.

Transitions are stored field by field in preallocated device tensors of
``size`` rows, allocated on the first add from the shapes / dtypes it brings
(``obs_dtype`` may narrow the two observation fields, e.g. bfloat16, halving
their footprint).  ``add`` takes one transition as the reference does;
``add_batch`` takes a leading batch dimension — one row per env of a batched
rollout — and equals that many ``add`` calls in order.  ``sample`` returns
device tensors in the reference's order; ``random.random`` / ``random.randint``
are replaced by float64 uniforms (``u``, or drawn from ``generator``).
"""
import ctypes

import torch

from aido1_amd import _lib

FIELDS = ('obs', 'action', 'reward', 'next_obs', 'done')


class ReplayBuffer:
    def __init__(self, size, device=None, obs_dtype=None, generator=None):
        if size < 1:
            raise ValueError('size must be >= 1')
        self._maxsize = int(size)
        self._next_idx = 0
        self._len = 0
        self.device = torch.device('cuda', torch.cuda.current_device()) if device is None \
            else torch.device(device)
        if self.device.type == 'cuda' and self.device.index is None:
            self.device = torch.device('cuda', torch.cuda.current_device())
        self.obs_dtype = obs_dtype
        self.gen = generator
        self.storage = None

    def __len__(self):
        return self._len

    # ---- storage -----------------------------------------------------------------
    def _alloc(self, fields):
        self.storage = {}
        for name, t in zip(FIELDS, fields):
            dt = self.obs_dtype if (name in ('obs', 'next_obs') and self.obs_dtype) else t.dtype
            self.storage[name] = torch.zeros((self._maxsize,) + tuple(t.shape[1:]), dtype=dt,
                                             device=self.device)

    def _fields(self, obs_t, action, reward, obs_tp1, done, batched):
        out = []
        for name, x in zip(FIELDS, (obs_t, action, reward, obs_tp1, done)):
            t = torch.as_tensor(x, device=self.device)
            if name == 'done':
                t = t.to(torch.bool)
            elif not t.is_floating_point():
                t = t.to(torch.float32)
            out.append(t if batched else t.unsqueeze(0))
        n = out[0].shape[0]
        if any(t.shape[0] != n for t in out):
            raise ValueError('add_batch: fields disagree on the batch size')
        return out

    def _slots(self, n):
        return (self._next_idx + torch.arange(n, device=self.device)) % self._maxsize

    def _write(self, fields, slots, start):
        """Rows `slots` (= start, start+1, ... mod size) of every field."""
        n = slots.shape[0]
        if n > self._maxsize:        # later adds overwrite earlier ones
            fields = [f[n - self._maxsize:] for f in fields]
            slots = slots[n - self._maxsize:]
            start = (start + n - self._maxsize) % self._maxsize
            n = self._maxsize
        if self.storage is None:
            self._alloc(fields)
        for name, f in zip(FIELDS, fields):
            if start + n <= self._maxsize:   # one contiguous block: a plain copy
                self.storage[name][start:start + n].copy_(f)
            else:
                self.storage[name].index_copy_(0, slots, f.to(self.storage[name].dtype))

    def _reserve(self, n):
        """Device slots of the next n adds (before _advance)."""
        return self._slots(n)

    def _advance(self, n):
        self._next_idx = (self._next_idx + n) % self._maxsize
        self._len = min(self._len + n, self._maxsize)

    # ---- reference API -----------------------------------------------------------
    def add(self, obs_t, action, reward, obs_tp1, done):
        """buffers.py:29-36 (one transition)."""
        self.add_batch(obs_t, action, reward, obs_tp1, done, _batched=False)

    def add_batch(self, obs_t, action, reward, obs_tp1, done, _batched=True):
        fields = self._fields(obs_t, action, reward, obs_tp1, done, _batched)
        n = fields[0].shape[0]
        start = self._next_idx
        self._write(fields, self._reserve(n), start)
        self._advance(n)

    def add_batch_ring(self, obs_t, action, reward, ring, order, done):
        """add_batch with obs_tp1 = ring[:, order] (a rollout's frame ring in its
        stack order), copied from the ring straight into the buffer rows.
        Returns obs_tp1 as stored: a view of the buffer rows (the next
        decision's obs_t, valid until the buffer comes round to them), or a copy
        where the rows would not be one block or would be overwritten by the
        next add."""
        n = ring.shape[0]
        p = self._next_idx
        if self.storage is None or p + n > self._maxsize or 2 * n > self._maxsize:
            nxt = ring[:, list(order)]
            self.add_batch(obs_t, action, reward, nxt, done)
            return nxt
        self._reserve(n)
        st = self.storage
        st['obs'][p:p + n].copy_(torch.as_tensor(obs_t, device=self.device))
        st['action'][p:p + n].copy_(torch.as_tensor(action, device=self.device))
        st['reward'][p:p + n].copy_(torch.as_tensor(reward, device=self.device))
        for k, sl in enumerate(order):
            st['next_obs'][p:p + n, k].copy_(ring[:, sl])
        st['done'][p:p + n].copy_(torch.as_tensor(done, device=self.device).to(torch.bool))
        self._advance(n)
        return st['next_obs'][p:p + n]
    def _encode_sample(self, idxes):
        """buffers.py:38-52: (obs, actions, rewards, next_obs, dones) rows."""
        return tuple(self.storage[name].index_select(0, idxes) for name in FIELDS)

    def uniforms(self, batch_size):
        return torch.rand(batch_size, dtype=torch.float64, device=self.device, generator=self.gen)

    def sample(self, batch_size, u=None):
        """buffers.py:114-137: idx = randint(0, len - 1) = floor(u * len)."""
        if self._len < 1:
            raise ValueError('sample from an empty buffer')
        u = self.uniforms(batch_size) if u is None else torch.as_tensor(
            u, dtype=torch.float64, device=self.device)
        idxes = torch.clamp((u * self._len).floor().long(), max=self._len - 1)
        return self._encode_sample(idxes)


class PrioritizedReplayBuffer(ReplayBuffer):
    """buffers.py:140-259 on the GPU (segment trees in csrc/dtreplay.hip)."""

    def __init__(self, size, alpha=0.5, device=None, obs_dtype=None, generator=None):
        super().__init__(size, device, obs_dtype, generator)
        if not alpha > 0:
            raise ValueError('alpha must be > 0')   # buffers.py:158
        self._alpha = alpha
        self._L = _lib.lib()
        h = ctypes.c_void_p()
        rc = self._L.dt_per_create(self._maxsize, float(alpha), self.device.index, ctypes.byref(h))
        if rc != 0:
            raise _lib.DtError('dt_per_create failed (%d): %s' %
                               (rc, (self._L.dt_per_last_error(None) or b'').decode()))
        self._h = h
        self.capacity = int(self._L.dt_per_capacity(h))

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, rc, what):
        if rc != 0:
            msg = self._L.dt_per_last_error(self._h) or b''
            raise _lib.DtError('%s failed (%d): %s' % (what, rc, msg.decode()))

    def _reserve(self, n):
        """n consecutive add() calls' tree updates (buffers.py:169-174): every
        new leaf gets max_priority**alpha; returns the slots."""
        slots = torch.empty(n, dtype=torch.int64, device=self.device)
        with torch.cuda.device(self.device):
            self._check(self._L.dt_per_add(self._h, n, ctypes.c_void_p(slots.data_ptr()),
                                           self._stream()), 'dt_per_add')
        return slots

    def _advance(self, n):
        super()._advance(n)
        assert self._next_idx == self._L.dt_per_next_idx(self._h)

    def sample(self, batch_size, beta=0.5, u=None):
        """buffers.py:185-235 -> (obs, act, rew, next_obs, done, weights, idxes)."""
        if not beta > 0:
            raise ValueError('beta must be > 0')     # buffers.py:221
        u = self.uniforms(batch_size) if u is None else torch.as_tensor(
            u, dtype=torch.float64, device=self.device).contiguous()
        idxes = torch.empty(batch_size, dtype=torch.int64, device=self.device)
        weights = torch.empty(batch_size, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            self._check(self._L.dt_per_sample(self._h, batch_size, ctypes.c_void_p(u.data_ptr()),
                                              float(beta), ctypes.c_void_p(idxes.data_ptr()),
                                              ctypes.c_void_p(weights.data_ptr()),
                                              self._stream()), 'dt_per_sample')
        return self._encode_sample(idxes) + (weights, idxes)

    def update_priorities(self, idxes, priorities):
        """buffers.py:237-259.  Invalid entries (the reference's asserts) are
        skipped on the GPU and reported by check()."""
        idx = torch.as_tensor(idxes, dtype=torch.int64, device=self.device).reshape(-1).contiguous()
        pr = torch.as_tensor(priorities, dtype=torch.float64, device=self.device).reshape(-1) \
            .contiguous()
        if idx.numel() != pr.numel():
            raise ValueError('len(idxes) != len(priorities)')   # buffers.py:252
        with torch.cuda.device(self.device):
            self._check(self._L.dt_per_update(self._h, idx.numel(), ctypes.c_void_p(idx.data_ptr()),
                                              ctypes.c_void_p(pr.data_ptr()), self._stream()),
                        'dt_per_update')

    def check(self):
        """Synchronise and raise if an update held an entry the reference rejects."""
        with torch.cuda.device(self.device):
            self._check(self._L.dt_per_check(self._h), 'update_priorities')

    def trees(self):
        """(sum tree, min tree, max_priority) copies — float64 [2*capacity] x2, [1]."""
        s = torch.empty(2 * self.capacity, dtype=torch.float64, device=self.device)
        m = torch.empty_like(s)
        mp = torch.empty(1, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            self._check(self._L.dt_per_read(self._h, ctypes.c_void_p(s.data_ptr()),
                                            ctypes.c_void_p(m.data_ptr()),
                                            ctypes.c_void_p(mp.data_ptr()), self._stream()),
                        'dt_per_read')
        return s, m, mp

    def close(self):
        if getattr(self, '_h', None):
            self._L.dt_per_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def create_buffer(config, device=None, prioritized=False, **kw):
    """utils/buffers.py:7-9 (uniform ReplayBuffer(buffer_size); the reference
    keeps the prioritized constructor commented out — ``prioritized=True``
    selects it with the config's alpha)."""
    t = config['training'] if 'training' in config else config
    if prioritized:
        return PrioritizedReplayBuffer(t['buffer_size'], t['alpha'], device=device, **kw)
    return ReplayBuffer(t['buffer_size'], device=device, **kw)
