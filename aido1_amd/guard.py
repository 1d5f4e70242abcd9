"""Non-finite guards on the training path (SURVEY.md §5 "Failure detection":
NaN/Inf guard flags; include/dttrain.h dt_guard_scan).

The reference survives bad values by brute force: its env wrapper retries a
failed step forever (utils/env_wrappers.py:57-68) and an explorer that raises
restarts its episode (training/explorers.py:156-157).  The batched loop here
runs without host synchronisation, so a NaN in one stage would otherwise only
surface many updates later as a NaN loss.  A ``Guard`` is one device block of
DT_GUARD_WORDS int32 that every stage of the loop reports into (a bit per
stage, the tick at which it first fired); nothing is read back until
``check()``, which raises ``NonFiniteError`` naming the stages in pipeline
order, earliest first -- so the first named stage is where a NaN entered.

On the GPU the reports come from the kernels themselves (dt_bn_leaky_fwd /
_bwd, dt_adam) and from dt_guard_scan launches over the stage outputs, all
graph-capturable; on the CPU (the float64 parity path of the tests) the same
bits are set with torch ops.
"""
import ctypes

import torch

from aido1_amd import _lib

WORDS = 36          # DT_GUARD_WORDS
NONE = 0x7fffffff   # DT_GUARD_NONE
MAX_SCAN = 8        # DT_GUARD_MAX

# include/dttrain.h DT_GUARD_*, in pipeline order
STAGES = {
    0: 'actor_out',      # rollout actor outputs (before DDPG.act's clip)
    1: 'env',            # rollout rewards
    2: 'batch',          # the sampled batch
    3: 'target',         # y = r + notdone * gamma * Q'(s', pi'(s'))
    4: 'bn_fwd',         # a train-mode BatchNorm's batch mean / invstd
    5: 'bn_count',       # a BatchNorm's merged pixel count != m (a lost partial)
    6: 'critic_loss',
    7: 'bn_bwd',         # a BatchNorm's dgamma / dbeta / dbias
    8: 'critic_grad',
    9: 'critic_param',
    10: 'actor_loss',
    11: 'actor_grad',
    12: 'actor_param',
    13: 'td',            # the TD error (-> update_priorities)
}
BIT = {v: k for k, v in STAGES.items()}


class NonFiniteError(RuntimeError):
    pass


class DtGuardTensor(ctypes.Structure):
    """include/dttrain.h dt_guard_tensor."""
    _fields_ = [('p', ctypes.c_void_p), ('count', ctypes.c_int64), ('bit', ctypes.c_int32),
                ('dtype', ctypes.c_int32)]


class Guard:
    def __init__(self, device):
        self.device = torch.device(device)
        self.words = torch.zeros(WORDS, dtype=torch.int32, device=self.device)
        self.words[3:] = NONE

    def ptr(self):
        return self.words.data_ptr() if self.words.is_cuda else None

    def tick(self):
        """Advance the sequence number (a device add: captured graphs advance it)."""
        self.words[2:3].add_(1)

    def scan(self, stage, *tensors):
        """Report `stage` if any element of `tensors` is NaN or +-Inf."""
        bit = BIT[stage] if isinstance(stage, str) else int(stage)
        ts = [t for t in tensors if t is not None and t.numel() > 0]
        if not ts:
            return
        if not self.words.is_cuda:
            bad = torch.stack([~torch.isfinite(t).all() for t in ts]).any()
            self._raise_cpu(bit, bad)
            return
        for i in range(0, len(ts), MAX_SCAN):
            part = ts[i:i + MAX_SCAN]
            arr = (DtGuardTensor * len(part))()
            for a, t in zip(arr, part):
                dense = t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(
                    memory_format=torch.channels_last))
                if t.dtype not in (torch.float32, torch.float64) or not dense:
                    raise ValueError('guard scan: dense float32/float64 tensors only')
                a.p, a.count, a.bit = t.data_ptr(), t.numel(), bit
                a.dtype = 0 if t.dtype == torch.float32 else 1
            rc = _lib.lib().dt_guard_scan(len(part), ctypes.cast(arr, ctypes.c_void_p),
                                          self.words.data_ptr(), ctypes.c_void_p(
                torch.cuda.current_stream(self.device).cuda_stream))
            if rc != 0:
                raise _lib.DtError('dt_guard_scan failed (%d)' % rc)

    def _raise_cpu(self, bit, bad):
        w = self.words
        b = bad.to(torch.int32)
        w[0] |= b << bit
        w[1] += b
        if bool(bad):
            w[3 + bit] = min(int(w[3 + bit]), int(w[2]))

    def read(self):
        """{'stages': [(name, first tick), ...] in pipeline order, 'count': n,
        'tick': t} (synchronises with the device)."""
        w = self.words.cpu().tolist()
        bits = w[0] & 0xffffffff
        stages = [(STAGES.get(b, 'bit%d' % b), w[3 + b]) for b in range(32) if bits >> b & 1]
        return {'stages': stages, 'count': w[1], 'tick': w[2]}

    def clear(self):
        self.words[:2].zero_()
        self.words[3:] = NONE

    def check(self, what='training loop'):
        r = self.read()
        if r['stages']:
            first = min(t for _, t in r['stages'])
            msg = ', '.join('%s (first at tick %d)' % s for s in r['stages'])
            self.clear()
            raise NonFiniteError('%s: non-finite values at %s; earliest tick %d, %d detections; '
                                 'the first stage named at the earliest tick is where they '
                                 'entered' % (what, msg, first, r['count']))
        return r
