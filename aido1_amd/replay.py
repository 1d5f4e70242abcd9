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

Frame store (``frame_envs=n``, what TrainLoop uses): a batched rollout of n
envs adds n transitions a decision whose observations are Transformer stacks
of k frames, and consecutive stacks of an env share k - 1 frames
(obs_t = next_obs of the env's previous transition).  Storing both stacks
per transition moves 2k frames an env a decision; the frame store keeps each
decision's ONE new frame per env in a ring of frame blocks (n rows a block,
``size / n + 2k`` blocks) and gives every transition two int32 [k] rows of
frame indices, written by dt_frame_add (include/dtreplay.h) in one kernel
with the frame copy.  ``sample`` gathers the stacks through them, so it
returns what the stacked storage returns.  Needs ``size % n == 0`` and
float32 observations; only ``add_batch_ring`` adds to it.  The frames keep the
ring's dtype: a ring of palette-index frames (u8, render.py) is stored as
such -- a quarter of the grey bytes, 4x the transitions per GiB of HBM -- and
decoded to the grey float32 observations by ``sample`` / ``gather_into``
(bit for bit the grey ring's).
"""
import collections
import ctypes

import torch

from aido1_amd import _lib
from aido1_amd.render import as_gray

FIELDS = ('obs', 'action', 'reward', 'next_obs', 'done')


class ReplayBuffer:
    def __init__(self, size, device=None, obs_dtype=None, generator=None, frame_envs=None):
        if size < 1:
            raise ValueError('size must be >= 1')
        if frame_envs is not None:
            if frame_envs < 1 or size % frame_envs:
                raise ValueError('frame_envs must divide size')
            if obs_dtype not in (None, torch.float32):
                raise ValueError('the frame store holds float32 observations')
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
        self.frame_envs = int(frame_envs) if frame_envs else None
        self.frames = None          # frame store: [blocks * n, H, W] float32
        self._fblock = 0            # frame blocks written so far
        self._begun = False         # a chain of stacks has begun (first add_batch_ring)
        self._stack_lo = 0          # oldest frame block (absolute) the current stacks reference
        self._group_lo = collections.deque()   # the same for every live decision's rows
        self._decisions = 0

    def __len__(self):
        return self._len

    # ---- storage -----------------------------------------------------------------
    def _alloc(self, fields):
        self.storage = {}
        for name, t in zip(FIELDS, fields):
            dt = self.obs_dtype if (name in ('obs', 'next_obs') and self.obs_dtype) else t.dtype
            self.storage[name] = torch.zeros((self._maxsize,) + tuple(t.shape[1:]), dtype=dt,
                                             device=self.device)

    def _field(self, name, x):
        t = torch.as_tensor(x, device=self.device)
        if name == 'done':
            return t.to(torch.bool)
        return t if t.is_floating_point() else t.to(torch.float32)

    def _fields(self, obs_t, action, reward, obs_tp1, done, batched):
        out = []
        for name, x in zip(FIELDS, (obs_t, action, reward, obs_tp1, done)):
            t = self._field(name, x)
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
        if self.frame_envs is not None:
            raise ValueError('the frame store adds through add_batch_ring only')
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
        if self.frame_envs is not None:
            return self._frame_add(obs_t, action, reward, ring, order, done)
        n = ring.shape[0]
        p = self._next_idx
        if self.storage is None or p + n > self._maxsize or 2 * n > self._maxsize:
            nxt = as_gray(ring[:, list(order)])
            self.add_batch(obs_t, action, reward, nxt, done)
            return nxt
        self._reserve(n)
        st = self.storage
        st['obs'][p:p + n].copy_(torch.as_tensor(obs_t, device=self.device))
        st['action'][p:p + n].copy_(torch.as_tensor(action, device=self.device))
        st['reward'][p:p + n].copy_(torch.as_tensor(reward, device=self.device))
        for k, sl in enumerate(order):
            st['next_obs'][p:p + n, k].copy_(as_gray(ring[:, sl]))
        st['done'][p:p + n].copy_(torch.as_tensor(done, device=self.device).to(torch.bool))
        self._advance(n)
        return st['next_obs'][p:p + n]

    # ---- frame store ---------------------------------------------------------------
    def _frame_block(self, frames):
        """Write frames [n, H, W] (any strides) as the next frame block; returns
        the block's first row."""
        n = self.frame_envs
        b = self._fblock % (self.frames.shape[0] // n)
        self.frames[b * n:(b + 1) * n].copy_(frames)
        self._fblock += 1
        return b * n

    def _frame_add(self, obs_t, action, reward, ring, order, done):
        n, k = self.frame_envs, len(order)
        if ring.shape[0] != n:
            raise ValueError('add_batch_ring: the frame store holds %d envs, got %d'
                             % (n, ring.shape[0]))
        if self.frames is None:
            blocks = self._maxsize // n + 2 * k
            self.frames = torch.zeros((blocks * n,) + tuple(ring.shape[2:]), dtype=ring.dtype,
                                      device=self.device)
            self._stack = torch.zeros(n, k, dtype=torch.int32, device=self.device)
            self.storage = {
                'obs_ptr': torch.zeros(self._maxsize, k, dtype=torch.int32, device=self.device),
                'next_ptr': torch.zeros(self._maxsize, k, dtype=torch.int32, device=self.device)}
        if obs_t is None and not self._begun:
            raise ValueError('frame store: the first add_batch_ring needs obs_t')
        # The blocks this add writes (k for a new chain, then the newest frame)
        # overwrite the blocks `blocks` earlier; no live transition may still
        # reference one of those.  Live: every stored decision's rows except
        # the oldest one's when the buffer is full (this add overwrites them).
        blocks = self.frames.shape[0] // n
        live = list(self._group_lo)
        if len(live) == self._maxsize // n:
            live = live[1:]
        last = self._fblock + (k if obs_t is not None else 0)      # absolute, inclusive
        if live and last - blocks >= min(live):
            raise ValueError('frame store: a new observation chain would overwrite frames that '
                             'stored transitions still reference (chains begun too often: '
                             'allow about size / n decisions between resets)')
        if obs_t is not None:
            # a new chain (the first add, or a rollout reset): obs_t's k frames
            # become k frame blocks
            obs_t = torch.as_tensor(obs_t, device=self.device)
            if obs_t.dtype != self.frames.dtype:
                raise ValueError('frame store: obs_t must be in the ring\'s frame dtype (%s)'
                                 % self.frames.dtype)
            ar = torch.arange(n, dtype=torch.int32, device=self.device)
            self._stack_lo = self._fblock
            for j in range(k):
                self._stack[:, j] = ar + self._frame_block(obs_t[:, j])
            self._begun = True
        p = self._next_idx
        self._reserve(n)
        st = self.storage
        # device tensors only: a host tensor here would be a blocking copy
        # that drains the stream every decision
        fields = {name: self._field(name, x)
                  for name, x in (('action', action), ('reward', reward), ('done', done))}
        if any(f.shape[0] != n for f in fields.values()):
            raise ValueError('add_batch_ring: fields disagree on the batch size')
        if 'action' not in st:
            for name, f in fields.items():
                st[name] = torch.zeros((self._maxsize,) + tuple(f.shape[1:]), dtype=f.dtype,
                                       device=self.device)
        st['action'][p:p + n].copy_(fields['action'])
        st['reward'][p:p + n].copy_(fields['reward'])
        st['done'][p:p + n].copy_(fields['done'])
        newest = ring[:, order[-1]]
        b = self._fblock % (self.frames.shape[0] // n)
        dn = fields['done']
        if self.device.type == 'cuda':
            L = _lib.lib()
            if (not newest[0].is_contiguous() or ring.dtype != self.frames.dtype
                    or ring.dtype not in (torch.float32, torch.uint8)):
                raise ValueError('frame store: the ring must hold float32 or uint8 frames, '
                                 'contiguous')
            # dt_frame_add copies 4-byte words
            sz = ring.element_size()
            fe, stride = newest[0].numel() * sz // 4, newest.stride(0) * sz // 4
            with torch.cuda.device(self.device):
                rc = L.dt_frame_add(n, fe, newest.data_ptr(), stride,
                                    self.frames[b * n].data_ptr(), k, self._stack.data_ptr(),
                                    dn.view(torch.uint8).data_ptr(), b * n,
                                    st['obs_ptr'][p].data_ptr(), st['next_ptr'][p].data_ptr(),
                                    ctypes.c_void_p(torch.cuda.current_stream(self.device)
                                                    .cuda_stream))
            if rc != 0:
                raise _lib.DtError('dt_frame_add failed (%d)' % rc)
            self._fblock += 1
        else:   # CPU tensors (tests): the same bookkeeping in torch
            row0 = self._frame_block(newest)
            rows = torch.arange(n, dtype=torch.int32) + row0
            st['obs_ptr'][p:p + n].copy_(self._stack)
            nxt = torch.cat([self._stack[:, 1:], rows[:, None]], 1)
            nxt[dn] = rows[dn, None]
            st['next_ptr'][p:p + n].copy_(nxt)
            self._stack.copy_(nxt)
        # this decision's rows reference the stacks before the add (and the
        # newest block); afterwards the stacks drop their oldest block (an env
        # that respawned references only the newest: a later block)
        self._group_lo.append(self._stack_lo)
        if len(self._group_lo) > self._maxsize // n:
            self._group_lo.popleft()
        self._stack_lo = min(self._stack_lo + 1, self._fblock - 1) if k > 1 else self._fblock - 1
        self._decisions += 1
        self._advance(n)
        return None

    def _encode_sample(self, idxes):
        """buffers.py:38-52: (obs, actions, rewards, next_obs, dones) rows."""
        st = self.storage
        if self.frames is not None:
            shp = (idxes.shape[0], st['obs_ptr'].shape[1]) + tuple(self.frames.shape[1:])
            obs = as_gray(self.frames.index_select(
                0, st['obs_ptr'].index_select(0, idxes).reshape(-1)))
            nxt = as_gray(self.frames.index_select(
                0, st['next_ptr'].index_select(0, idxes).reshape(-1)))
            return (obs.view(shp), st['action'].index_select(0, idxes),
                    st['reward'].index_select(0, idxes), nxt.view(shp),
                    st['done'].index_select(0, idxes))
        return tuple(st[name].index_select(0, idxes) for name in FIELDS)

    def gather_into(self, idxes, out):
        """_encode_sample(idxes) written straight into a trainer's inputs `out`
        (DDPGTrainer.static_inputs: obs / nxt float32 channels_last [b, k, h, w],
        act [b, 2], rew [b, 1], notdone [b, 1]): one dt_frame_gather launch with
        the frame store on the GPU (include/dtreplay.h), torch copies otherwise."""
        st = self.storage
        b = idxes.shape[0]
        if (self.frames is not None and self.frames.is_cuda and out['obs'].dtype == torch.float32
                and out['obs'].is_contiguous(memory_format=torch.channels_last)
                and out['nxt'].is_contiguous(memory_format=torch.channels_last)
                and st['action'].dtype == torch.float32 and st['reward'].dtype == torch.float64
                and st['done'].dtype == torch.bool and idxes.dtype == torch.int64):
            k = st['obs_ptr'].shape[1]
            hw = self.frames[0].numel()
            idxes = idxes.contiguous()
            kind = 1 if self.frames.dtype == torch.uint8 else 0
            rc = _lib.lib().dt_frame_gather(
                b, idxes.data_ptr(), self.frames.data_ptr(), kind, hw, k, st['obs_ptr'].data_ptr(),
                st['next_ptr'].data_ptr(), st['action'].data_ptr(), st['reward'].data_ptr(),
                st['done'].data_ptr(), out['obs'].data_ptr(), out['nxt'].data_ptr(),
                out['act'].data_ptr(), out['rew'].data_ptr(), out['notdone'].data_ptr(),
                ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
            if rc != 0:
                raise _lib.DtError('dt_frame_gather failed (%d)' % rc)
            return out
        obs, act, rew, nxt, done = self._encode_sample(idxes)
        out['obs'].copy_(obs)
        out['nxt'].copy_(nxt)
        out['act'].copy_(act)
        out['rew'].copy_(rew.reshape(-1, 1))
        out['notdone'].copy_((~done.bool()).reshape(-1, 1))
        return out

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

    def __init__(self, size, alpha=0.5, device=None, obs_dtype=None, generator=None,
                 frame_envs=None):
        super().__init__(size, device, obs_dtype, generator, frame_envs)
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
        idxes, weights = self.sample_indices(batch_size, beta, u)
        return self._encode_sample(idxes) + (weights, idxes)

    def sample_indices(self, batch_size, beta=0.5, u=None):
        """sample()'s (idxes, weights) without encoding the rows."""
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
        return idxes, weights

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

    def update_priorities_td(self, idxes, td, eps):
        """update_priorities(idxes, |td| + eps) for float32 TD errors on the
        device, the priorities formed inside the tree kernel (one launch)."""
        idx = torch.as_tensor(idxes, dtype=torch.int64, device=self.device).reshape(-1).contiguous()
        td = td.detach().reshape(-1).contiguous()
        if td.dtype != torch.float32 or td.device != self.device or td.numel() != idx.numel():
            return self.update_priorities(idx, td.abs().double() + eps)
        with torch.cuda.device(self.device):
            self._check(self._L.dt_per_update_td(self._h, idx.numel(),
                                                 ctypes.c_void_p(idx.data_ptr()),
                                                 ctypes.c_void_p(td.data_ptr()), float(eps),
                                                 self._stream()), 'dt_per_update_td')

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
