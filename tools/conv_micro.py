"""Microbenchmark of the actor's first two convolutions at 4096 samples, fp16
NHWC: direct vs space-to-depth reformulations (same outputs)."""
import time
import torch
import torch.nn.functional as F

dev = torch.device('cuda', 0)
torch.backends.cudnn.benchmark = True
N = 4096
cl = torch.channels_last
dt = torch.float16


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def s2d(x, b=2):  # NCHW logical -> [N, C*b*b, H/b, W/b] with channel order (c, dy, dx)
    n, c, h, w = x.shape
    return x.view(n, c, h // b, b, w // b, b).permute(0, 1, 3, 5, 2, 4).reshape(n, c * b * b, h // b, w // b)


def w_s2d(w, b=2):  # [co, c, k, k] -> [co, c*b*b, k/b, k/b] matching s2d's channel order
    co, c, k, _ = w.shape
    return w.view(co, c, k // b, b, k // b, b).permute(0, 1, 3, 5, 2, 4).reshape(co, c * b * b, k // b, k // b)


x = torch.rand(N, 3, 120, 160, device=dev)            # f32 ring, NCHW
w1 = (torch.randn(32, 3, 8, 8, device=dev) * 0.05)
b1 = torch.randn(32, device=dev) * 0.1
xh = x.to(dt, memory_format=cl)
w1h = w1.to(dt).contiguous(memory_format=cl)
ref = F.conv2d(xh, w1h, b1.to(dt), stride=2)
xs = s2d(x).to(dt, memory_format=cl)
w1s = w_s2d(w1).to(dt).contiguous(memory_format=cl)
out = F.conv2d(xs, w1s, b1.to(dt), stride=1)
print('conv1 s2d max diff %.3e' % (out.float() - ref.float()).abs().max().item())
print('convert f32 ring -> fp16 NHWC   %.3f ms' % bench(lambda: x.to(dt, memory_format=cl)))
print('convert + s2d                   %.3f ms' % bench(lambda: s2d(x).to(dt, memory_format=cl)))
print('conv1 direct 8x8 s2 (3ch)       %.3f ms' % bench(lambda: F.conv2d(xh, w1h, b1.to(dt), stride=2)))
print('conv1 s2d    4x4 s1 (12ch)      %.3f ms' % bench(lambda: F.conv2d(xs, w1s, b1.to(dt), stride=1)))
xs4 = torch.cat([xs, torch.zeros(N, 4, 60, 80, device=dev, dtype=dt)], 1).contiguous(memory_format=cl)
w1s4 = torch.cat([w1s, torch.zeros(32, 4, 4, 4, device=dev, dtype=dt)], 1).contiguous(memory_format=cl)
print('conv1 s2d    4x4 s1 (16ch pad)  %.3f ms' % bench(lambda: F.conv2d(xs4, w1s4, b1.to(dt), stride=1)))
# conv2: 32 -> 32, 4x4 stride 2 on 57x77
y1 = torch.rand(N, 32, 57, 77, device=dev, dtype=dt).contiguous(memory_format=cl)
w2 = (torch.randn(32, 32, 4, 4, device=dev) * 0.05).to(dt).contiguous(memory_format=cl)
b2 = torch.zeros(32, device=dev, dtype=dt)
print('conv2 direct 4x4 s2 (32ch)      %.3f ms' % bench(lambda: F.conv2d(y1, w2, b2, stride=2)))
y1p = F.pad(y1, (0, 1, 0, 1)).contiguous(memory_format=cl)          # 58 x 78
y1s = s2d(y1p).contiguous(memory_format=cl)                         # 128 x 29 x 39
w2s = w_s2d(w2.float()).to(dt).contiguous(memory_format=cl)         # 32 x 128 x 2 x 2
o2 = F.conv2d(y1s, w2s, b2, stride=1)[:, :, :27, :37]
r2 = F.conv2d(y1, w2, b2, stride=2)
print('conv2 s2d max diff %.3e' % (o2.float() - r2.float()).abs().max().item())
print('conv2 s2d    2x2 s1 (128ch)     %.3f ms' % bench(lambda: F.conv2d(y1s, w2s, b2, stride=1)))
for name, y, ww in (('conv3', torch.rand(N, 32, 27, 37, device=dev, dtype=dt), 2),
                    ('conv4', torch.rand(N, 32, 12, 17, device=dev, dtype=dt), 1)):
    y = y.contiguous(memory_format=cl)
    print('%s direct                    %.3f ms' % (name, bench(lambda: F.conv2d(y, w2, b2, stride=ww))))
