"""torch BatchNorm2d train-mode forward/backward on the GPU vs float64 CPU, by
batch size, memory format and backend (MIOpen vs native)."""
import torch
import torch.nn.functional as F

dev = torch.device('cuda', 0)
torch.manual_seed(0)
for cudnn in (True, False):
    torch.backends.cudnn.enabled = cudnn
    for n, c, h, w in ((1, 32, 57, 77), (4, 32, 57, 77), (64, 32, 57, 77), (64, 32, 9, 14),
                       (1, 32, 9, 14)):
        for fmt in (torch.contiguous_format, torch.channels_last):
            x = (torch.randn(n, c, h, w) * 2 + 3)
            g = torch.rand(c) + 0.5
            b = torch.rand(c) - 0.5
            xd = x.double().requires_grad_()
            yd = F.batch_norm(xd, None, None, g.double(), b.double(), training=True, eps=1e-5)
            gy = torch.randn_like(yd)
            yd.backward(gy)
            xg = x.to(dev).contiguous(memory_format=fmt).requires_grad_()
            rm = torch.zeros(c, device=dev)
            rv = torch.ones(c, device=dev)
            yg = F.batch_norm(xg, rm, rv, g.to(dev), b.to(dev), training=True, eps=1e-5)
            yg.backward(gy.float().to(dev).contiguous(memory_format=fmt))
            ef = (yg.double().cpu() - yd).abs().max().item()
            eb = (xg.grad.double().cpu() - xd.grad).abs().max().item()
            print('cudnn=%d n=%2d hw=%dx%d %-14s fwd %.1e bwd %.1e' % (
                cudnn, n, h, w, 'NHWC' if fmt == torch.channels_last else 'NCHW', ef, eb))
