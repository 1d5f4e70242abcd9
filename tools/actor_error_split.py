"""Where the fp16 reference-mode actor's action error comes from: the
rollout's fp16 chain (dt_conv1 + dt_conv32 x3 + hipBLASLt lin1 + dt_actor_head)
against the f32 path on the same live frames (4096 envs, small_loop/zigzag
after warm-up decisions), split into the trunk's part (the f32 head on the fp16
flatten) and the head's part, for two weight seeds; plus per-layer errors of
the flatten.  usage: python tools/actor_error_split.py [seeds...]"""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, 'tests')
from conftest import golden  # noqa: E402
from aido1_amd.actor import ConfigActor, FusedActor  # noqa: E402
from aido1_amd.rollout import ActorRollout  # noqa: E402

dev = torch.device('cuda', 0)
cfg = golden('reference_config.json')
seeds = [int(s) for s in sys.argv[1:]] or [11, 1234]
roll = ActorRollout(cfg, 4096, device=0, seed=1234, actor_mode='reference',
                    dtype=torch.float16)
roll.reset()
for _ in range(12):
    roll.step()
torch.cuda.synchronize()
ring, order = roll.ring, roll.order()
stack = roll.stack()


def f32_flat(a32, x):
    h = x.to(torch.float32, memory_format=torch.channels_last)
    for i in range(4):
        h = F.conv2d(h, a32.w[i], a32.b[i], stride=a32.strides[i])
        h = a32._lrelu_sample_norm(h, i)
    return h.contiguous().flatten(1)


with torch.no_grad():
    for seed in seeds:
        torch.manual_seed(seed)
        actor = ConfigActor(cfg['model']['actor']).to(dev)
        a16 = FusedActor(actor, dtype=torch.float16, mode='reference')
        a32 = FusedActor(actor, dtype=torch.float32, mode='reference')
        a16.p_drop = a32.p_drop = 0.0
        with torch.backends.cudnn.flags(enabled=True, benchmark=True, deterministic=False,
                                        allow_tf32=False):
            flat32 = f32_flat(a32, stack)
        flat16 = a16._convs_hip(ring, order)
        full16 = a16(ring, order)
        full32 = a32._head(flat32)
        trunk = a32._head(flat16.float())          # f32 head on the fp16 trunk
        # the head in fp16 on the f32 trunk
        head16 = a16._heads(None, flat32.half(), flat32.shape[0],
                            torch.empty(flat32.shape[0], 2, device=dev))
        h32 = F.linear(flat32, a32.w1, a32.b1)
        h16 = F.linear(flat16, a16.w1, a16.b1).float()
        df = (flat16.float() - flat32).abs()
        print('seed %d: |action| total max %.3e p99 %.3e | trunk-only max %.3e | head-only max '
              '%.3e | flatten max %.3e mean %.3e (|flat| max %.2f) | lin1 out max %.3e (|h| max %.2f)'
              % (seed, (full16 - full32).abs().max(),
                 torch.quantile((full16 - full32).abs().flatten(), 0.99),
                 (trunk - full32).abs().max(), (head16 - full32).abs().max(), df.max(), df.mean(),
                 flat32.abs().max(), (h16 - h32).abs().max(), h32.abs().max()))
        worst = (full16 - full32).abs().max(1).values.argmax()
        print('   worst sample %d: full16 %s full32 %s trunk %s head16 %s' % (
            worst, full16[worst].tolist(), full32[worst].tolist(), trunk[worst].tolist(),
            head16[worst].tolist()))
