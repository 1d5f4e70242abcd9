"""Multi-GPU plumbing: one process per GPU, torch.distributed
("nccl" = RCCL over xGMI on MI355X; "gloo" for CPU tests).

* Stepping needs no collective: rank r owns global envs [r*n, (r+1)*n) and keys
  their spawn streams by global id (``env_id_base``), so any GPU count draws
  the streams one big batch would.
* ``reduce_run``: env-step counters summed, wall time maxed (bench.py).
* ``gather_returns``: finished-episode returns of every rank (the explorers'
  per-episode reward log, training/explorers.py:215-240), variable length.
* ``GradAllReduce``: the DDPG gradient all-reduce that replaces the reference's
  barrier + parameter averaging (training/trainers.py:206-213,
  models/torch_utils.py:21-29): gradients flattened into a few large buckets
  (xGMI ring collectives are per-link bound, so few big messages), averaged.
"""
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def env_id_base(rank, n_per_rank):
    return rank * n_per_rank


def reduce_run(counts, elapsed, device='cpu'):
    """counts: dict of numbers summed over ranks; elapsed: max over ranks."""
    keys = sorted(counts)
    t = torch.tensor([float(counts[k]) for k in keys], dtype=torch.float64, device=device)
    e = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    if world()[1] > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
    return dict(zip(keys, t.tolist())), float(e.item())


def gather_returns(returns):
    """All ranks' finished-episode returns, concatenated in rank order: 1-D
    tensors, or [m, c] tables of per-episode records (TrainLoop.poll_episodes:
    rank, env, tick, returns, steps), m varying by rank (padded transfer:
    all_gather needs equal sizes).  The tensors must live where the backend
    can reach them (GPU for nccl, CPU for gloo)."""
    rank, ws = world()
    if ws == 1:
        return returns.clone()
    dev = returns.device
    n = torch.tensor([returns.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(ws)]
    dist.all_gather(sizes, n)
    m = int(max(s.item() for s in sizes))
    buf = torch.full((max(m, 1),) + tuple(returns.shape[1:]), float('nan'), dtype=returns.dtype,
                     device=dev)
    buf[:returns.shape[0]] = returns
    parts = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(parts, buf)
    return torch.cat([p[:int(s.item())] for p, s in zip(parts, sizes)])


def collective_device(device):
    """Where a collective's tensors must live: the rank's GPU under nccl (RCCL),
    the host under gloo."""
    if world()[1] > 1 and dist.get_backend() == 'nccl':
        return torch.device(device)
    return torch.device('cpu')


class GradAllReduce:
    """Average gradients across ranks in buckets of ~bucket_mb MB."""

    def __init__(self, params, bucket_mb=16):
        self.params = [p for p in params if p.requires_grad]
        self.buckets = []
        cur, size = [], 0
        limit = int(bucket_mb * (1 << 20))
        for p in self.params:
            nbytes = p.numel() * p.element_size()
            if cur and size + nbytes > limit:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)

    def __call__(self):
        rank, ws = world()
        if ws == 1:
            return
        for bucket in self.buckets:
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in bucket]
            flat = torch.cat([g.reshape(-1) for g in grads])
            dist.all_reduce(flat, op=dist.ReduceOp.SUM)
            flat /= ws
            off = 0
            for p, g in zip(bucket, grads):
                k = g.numel()
                if p.grad is None:
                    p.grad = flat[off:off + k].view_as(p).clone()
                else:
                    p.grad.copy_(flat[off:off + k].view_as(p))
                off += k
