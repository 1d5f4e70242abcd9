"""The DDPG actor in the loop (BASELINE configs[3]).

Two layouts, parameter names identical to the reference so checkpoints
(`{name}_actor.pth`, `actor_state_dict.pth`) load unchanged:

* ``ActorCNN`` — duckietown_rl/ddpg.py:16-62 (conv1..4, bn1..4, lin1, lin2;
  head: sigmoid * max_action on output 0, tanh on output 1);
* ``ConfigActor`` — the config-driven actor of models/ddpg/modules.py:87-178
  built from config.json's "actor" list (keys
  ``net.input_nets.0.internal_modules.<i>.kernel.*`` etc.; config.json's head
  is tanh on both outputs).

Both compute conv -> LeakyReLU -> BatchNorm x4 -> flatten(4032) -> dropout ->
linear(512) -> LeakyReLU -> linear(2) -> head.  On MI355X the batched forward
runs in bf16 (MFMA through MIOpen/hipBLASLt) with the eval-mode BatchNorms
folded into the following conv / linear, and reads the observation ring
zero-copy: the first conv's input channels are permuted to the ring's slot
order instead of gathering the Transformer stack.
"""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

FLAT = 32 * 9 * 14  # 4032 (120x160 input)


class ActorCNN(nn.Module):
    """duckietown_rl/ddpg.py ActorCNN (same attribute names)."""

    head = 'sigmoid_tanh'

    def __init__(self, action_dim=2, max_action=1.0):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 8, stride=2)
        self.conv2 = nn.Conv2d(32, 32, 4, stride=2)
        self.conv3 = nn.Conv2d(32, 32, 4, stride=2)
        self.conv4 = nn.Conv2d(32, 32, 4, stride=1)
        self.bn1 = nn.BatchNorm2d(32)
        self.bn2 = nn.BatchNorm2d(32)
        self.bn3 = nn.BatchNorm2d(32)
        self.bn4 = nn.BatchNorm2d(32)
        self.dropout = nn.Dropout(.5)
        self.lin1 = nn.Linear(FLAT, 512)
        self.lin2 = nn.Linear(512, action_dim)
        self.max_action = max_action

    def layers(self):
        return ([self.conv1, self.conv2, self.conv3, self.conv4],
                [self.bn1, self.bn2, self.bn3, self.bn4], self.lin1, self.lin2)

    def forward(self, x):
        convs, bns, lin1, lin2 = self.layers()
        for conv, bn in zip(convs, bns):
            x = bn(F.leaky_relu(conv(x)))
        x = self.dropout(x.flatten(1))
        x = lin2(F.leaky_relu(lin1(x)))
        return apply_head(x, self.head, self.max_action)


class _Conv(nn.Module):      # Conv2dWrapper: parameter path ".kernel"
    def __init__(self, cin, cout, k, s):
        super().__init__()
        self.kernel = nn.Conv2d(cin, cout, k, stride=s)


class _Lin(nn.Module):       # LinearWrapper: parameter path ".linear"
    def __init__(self, fin, fout):
        super().__init__()
        self.linear = nn.Linear(fin, fout)


class _Seq(nn.Module):       # MetaNet: ".internal_modules.<i>"
    def __init__(self, mods):
        super().__init__()
        self.internal_modules = nn.ModuleList(mods)


class _Net(nn.Module):
    def __init__(self, inputs, outputs):
        super().__init__()
        self.input_nets = nn.ModuleList(inputs)
        self.output_nets = nn.ModuleList(outputs)


def _build_branch(spec):
    """One branch of config.json's module list -> list of modules (index-aligned
    with the reference's MetaNet so state_dict keys match)."""
    mods = []
    last = None
    for m in spec:
        name = m['name']
        a = m.get('args', {})
        if name == 'input':
            last = m['in_features']
            continue
        if name == 'input_channeled':
            last = m['in_channels']
            continue
        if name == 'conv_2d':
            mods.append(_Conv(last, a['out_channels'], a['kernel_size'], a['stride']))
            if a.get('padding', 0) != 0:
                raise NotImplementedError('padding')
            last = a['out_channels']
        elif name == 'batch_norm_2d':
            mods.append(nn.BatchNorm2d(last))
        elif name == 'leaky_relu':
            mods.append(nn.LeakyReLU())
        elif name == 'flatten':
            mods.append(nn.Flatten())
            last = a['out_features']
        elif name == 'dropout':
            mods.append(nn.Dropout(a['p']))
        elif name == 'linear':
            mods.append(_Lin(last, a['out_features']))
            last = a['out_features']
        elif name == 'tanh':
            mods.append(nn.Tanh())
        elif name == 'sigmoid':
            mods.append(nn.Sigmoid())
        else:
            raise NotImplementedError(name)
    return mods


class ConfigActor(nn.Module):
    """models/ddpg/modules.py Actor built from config.json's "actor" list
    (single input branch, single output branch, as config.json:19-91)."""

    def __init__(self, actor_config):
        super().__init__()
        ins = [s for m in actor_config if m['name'] == 'inputs' for s in m['modules']]
        outs = [s for m in actor_config if m['name'] == 'outputs' for s in m['modules']]
        if len(ins) != 1 or len(outs) != 1:
            raise NotImplementedError('one input and one output branch')
        self.net = _Net([_Seq(_build_branch(ins[0]))], [_Seq(_build_branch(outs[0]))])
        last = outs[0][-1]['name']
        self.head = {'tanh': 'tanh', 'sigmoid': 'sigmoid'}.get(last, 'none')
        self.max_action = 1.0

    def forward(self, x):
        for m in self.net.input_nets[0].internal_modules:
            x = m.kernel(x) if isinstance(m, _Conv) else (m.linear(x) if isinstance(m, _Lin) else m(x))
        for m in self.net.output_nets[0].internal_modules:
            x = m.kernel(x) if isinstance(m, _Conv) else (m.linear(x) if isinstance(m, _Lin) else m(x))
        return x

    def layers(self):
        mods = list(self.net.input_nets[0].internal_modules)
        convs = [m.kernel for m in mods if isinstance(m, _Conv)]
        bns = [m for m in mods if isinstance(m, nn.BatchNorm2d)]
        lins = [m.linear for m in mods if isinstance(m, _Lin)]
        lins += [m.linear for m in self.net.output_nets[0].internal_modules if isinstance(m, _Lin)]
        if len(convs) != 4 or len(bns) != 4 or len(lins) != 2:
            raise NotImplementedError('fused path expects 4 conv/bn pairs and 2 linears')
        return convs, bns, lins[0], lins[1]


def apply_head(x, head, max_action=1.0):
    if head == 'tanh':
        return torch.tanh(x)
    if head == 'sigmoid':
        return torch.sigmoid(x)
    if head == 'sigmoid_tanh':  # ActorCNN: [sigmoid * max_action, tanh]
        return torch.stack([max_action * torch.sigmoid(x[:, 0]), torch.tanh(x[:, 1])], 1)
    return x


class FusedActor(nn.Module):
    """Inference copy of an actor for the batched rollout: eval-mode BatchNorm
    (applied after LeakyReLU) folded into the NEXT conv / the first linear
    (an affine map of that layer's input), weights in `dtype`, and the first
    conv's input channels re-ordered per call to read the frame ring directly.
    Mathematically equal to the source actor in eval mode; numerically within
    bf16 rounding (tests/test_gpu_actor.py).  Convolutions run channels_last."""

    def __init__(self, actor, dtype=torch.bfloat16):
        super().__init__()
        convs, bns, lin1, lin2 = actor.layers()
        self.head = actor.head
        self.max_action = getattr(actor, 'max_action', 1.0)
        self.dtype = dtype
        ws, bs = [], []
        scale = shift = None
        for conv, bn in zip(convs, bns):
            w = conv.weight.detach().double()
            b = conv.bias.detach().double()
            if scale is not None:   # fold previous BN: conv(s*x + t)
                b = b + (w * shift.view(1, -1, 1, 1)).sum((1, 2, 3))
                w = w * scale.view(1, -1, 1, 1)
            ws.append(w)
            bs.append(b)
            scale = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() +
                                                             bn.eps)
            shift = bn.bias.detach().double() - bn.running_mean.detach().double() * scale
        w1 = lin1.weight.detach().double()
        b1 = lin1.bias.detach().double()
        s_flat = scale.repeat_interleave(FLAT // scale.numel())
        t_flat = shift.repeat_interleave(FLAT // shift.numel())
        b1 = b1 + w1 @ t_flat
        w1 = w1 * s_flat.view(1, -1)
        self.strides = [conv.stride for conv in convs]
        # NHWC (channels_last) convolutions: MIOpen's bf16 kernels are ~1.75x
        # faster on these shapes than NCHW (tools/actor_micro.py)
        self.w = nn.ParameterList([nn.Parameter(
            w.to(dtype).contiguous(memory_format=torch.channels_last), requires_grad=False)
            for w in ws])
        self.b = nn.ParameterList([nn.Parameter(b.to(dtype), requires_grad=False) for b in bs])
        self.w1 = nn.Parameter(w1.to(dtype), requires_grad=False)
        self.b1 = nn.Parameter(b1.to(dtype), requires_grad=False)
        self.w2 = nn.Parameter(lin2.weight.detach().to(dtype), requires_grad=False)
        self.b2 = nn.Parameter(lin2.bias.detach().to(dtype), requires_grad=False)

    @torch.no_grad()
    def forward(self, x, order=None):
        """x: [N,3,120,160] stack (oldest first), or the frame ring with
        `order` = ring slots oldest->newest (RenderOutput.order())."""
        w0 = self.w[0]
        if order is not None:
            inv = sorted(range(len(order)), key=lambda c: order[c])
            w0 = w0[:, inv].contiguous(memory_format=torch.channels_last)
        x = x.to(self.dtype, memory_format=torch.channels_last)
        x = F.leaky_relu(F.conv2d(x, w0, self.b[0], stride=self.strides[0]))
        for i in range(1, 4):
            x = F.leaky_relu(F.conv2d(x, self.w[i], self.b[i], stride=self.strides[i]))
        # flatten in NCHW order, as the reference's view(x.size(0), -1)
        x = F.leaky_relu(F.linear(x.contiguous().flatten(1), self.w1, self.b1))
        x = F.linear(x, self.w2, self.b2).float()
        return apply_head(x, self.head, self.max_action)


def flops_per_sample():
    """Multiply-adds x 2 of the actor trunk + head for one 3x120x160 input."""
    shapes = [(3, 32, 8, 57, 77), (32, 32, 4, 27, 37), (32, 32, 4, 12, 17), (32, 32, 4, 9, 14)]
    f = sum(2 * ci * co * k * k * ho * wo for ci, co, k, ho, wo in shapes)
    return f + 2 * FLAT * 512 + 2 * 512 * 2


def clone_eval(actor):
    a = copy.deepcopy(actor)
    a.eval()
    return a
