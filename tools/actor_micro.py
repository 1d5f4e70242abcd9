"""Diagnostic: actor forward time for layout / dtype / MIOpen-search variants."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from aido1_amd.actor import ConfigActor, FusedActor, flops_per_sample

cfg = json.load(open('aido1_amd/configs/reference_config.json'))
n = int(os.environ.get('N', 4096))
dev = torch.device('cuda', 0)
a = ConfigActor(cfg['model']['actor']).eval()
x32 = torch.rand(n, 3, 120, 160, device=dev)

def bench(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps

res = {}
for bench_mode in (False, True):
    torch.backends.cudnn.benchmark = bench_mode
    for dt in (torch.bfloat16, torch.float16):
        f = FusedActor(a, dtype=dt).to(dev)
        res['nchw %s bm=%d' % (dt, bench_mode)] = bench(lambda: f(x32))
        xc = x32.to(dt)
        res['nchw-precast %s bm=%d' % (dt, bench_mode)] = bench(lambda: f(xc))
        fcl = FusedActor(a, dtype=dt).to(dev)
        for i in range(4):
            fcl.w[i].data = fcl.w[i].data.contiguous(memory_format=torch.channels_last)
        xcl = x32.to(dt).contiguous(memory_format=torch.channels_last)
        res['nhwc %s bm=%d' % (dt, bench_mode)] = bench(lambda: fcl(xcl))
# per layer breakdown (bf16 nchw precast)
torch.backends.cudnn.benchmark = True
f = FusedActor(a, dtype=torch.bfloat16).to(dev)
xc = x32.to(torch.bfloat16)
h1 = F.leaky_relu(F.conv2d(xc, f.w[0], f.b[0], stride=2))
h2 = F.leaky_relu(F.conv2d(h1, f.w[1], f.b[1], stride=2))
h3 = F.leaky_relu(F.conv2d(h2, f.w[2], f.b[2], stride=2))
h4 = F.leaky_relu(F.conv2d(h3, f.w[3], f.b[3], stride=1))
res['L conv1'] = bench(lambda: F.conv2d(xc, f.w[0], f.b[0], stride=2))
res['L conv2'] = bench(lambda: F.conv2d(h1, f.w[1], f.b[1], stride=2))
res['L conv3'] = bench(lambda: F.conv2d(h2, f.w[2], f.b[2], stride=2))
res['L conv4'] = bench(lambda: F.conv2d(h3, f.w[3], f.b[3], stride=1))
res['L lin1'] = bench(lambda: F.linear(h4.flatten(1), f.w1, f.b1))
res['L cast'] = bench(lambda: x32.to(torch.bfloat16))
gf = n * flops_per_sample() / 1e9
for k, v in res.items():
    print('%-34s %8.3f ms  %7.1f TFLOP/s' % (k, v, gf / v if not k.startswith('L ') else 0))
