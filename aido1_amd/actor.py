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
linear(512) -> LeakyReLU -> linear(2) -> head.  On MI355X the batched
forward in the rollout is ``FusedActor``: the four convolutions are
hand-written fp16 MFMA kernels (csrc/dtconv.hip, include/dtactor.h) that read
the observation ring zero-copy (the first conv's input channels follow the
ring's slot order instead of gathering the Transformer stack), with f32
accumulation.  The default mode is 'reference': the reference explorers'
train-mode batch-of-one BatchNorm (per-sample statistics, fused into the
convolution kernels) and live dropout; 'eval' folds the eval-mode
BatchNorms into the following conv / linear.  The linears run as torch fp16
GEMMs (hipBLASLt) and the head in dt_actor_head.
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
    def __init__(self, cin, cout, k, s, weight_init=None):
        super().__init__()
        self.kernel = nn.Conv2d(cin, cout, k, stride=s)
        _init_weight(self.kernel.weight, weight_init, conv=True)

    def forward(self, x):
        return self.kernel(x)


class _Lin(nn.Module):       # LinearWrapper: parameter path ".linear"
    def __init__(self, fin, fout, weight_init=None):
        super().__init__()
        self.linear = nn.Linear(fin, fout)
        _init_weight(self.linear.weight, weight_init, conv=False)

    def forward(self, x):
        return self.linear(x)


def _init_weight(w, mode, conv):
    """LinearWrapper / Conv2dWrapper.init_weights (models/ddpg/modules.py:36-78);
    fanin_init's fan-in is size[0] (the OUTPUT dim, a reference quirk)."""
    with torch.no_grad():
        if mode == 'fanin':
            v = 1.0 / float(w.shape[0]) ** 0.5
            w.uniform_(-v, v)
        elif mode == 'uniform':
            w.uniform_(-3e-3, 3e-3)
        elif mode == 'xavier_normal':
            nn.init.xavier_normal_(w)
        elif mode == 'xavier_uniform':
            nn.init.xavier_uniform_(w)
        elif mode == 'kaiming_normal' and not conv:
            nn.init.kaiming_normal_(w)
        elif mode == 'kaiming_uniform' and not conv:
            nn.init.kaiming_uniform_(w)


class _Seq(nn.Module):       # MetaNet: ".internal_modules.<i>"
    # conv -> LeakyReLU -> BatchNorm blocks in train mode on the GPU (f32) run
    # as one chain (train_ops.conv_trunk, include/dtupd.h) or block by block
    # (train_ops.conv_leaky_bn, include/dttrain.h)
    fused_tail = True

    def __init__(self, mods):
        super().__init__()
        self.internal_modules = nn.ModuleList(mods)

    def forward(self, x):
        return self.run(x, 0, len(self.internal_modules))

    def run(self, x, i, k):
        """Modules [i, k) on x."""
        mods = self.internal_modules
        while i < k:
            m = mods[i]
            if (self.fused_tail and i + 2 < k and isinstance(m, _Conv)
                    and isinstance(mods[i + 2], nn.BatchNorm2d)):
                from aido1_amd import train_ops
                blocks = train_ops.trunk_len(x, mods, i, k)
                if blocks:
                    x = train_ops.conv_trunk(x, mods, i, blocks)
                    i += 3 * blocks
                    continue
                if train_ops.applicable(x, m.kernel, mods[i + 1], mods[i + 2]):
                    x = train_ops.conv_leaky_bn(x, m.kernel, mods[i + 1], mods[i + 2])
                    i += 3
                    continue
            drop = 0.0
            if (self.fused_tail and isinstance(m, nn.Dropout) and i + 1 < k
                    and isinstance(mods[i + 1], _Lin) and x.is_cuda):
                from aido1_amd import train_ops
                if train_ops.FOLD_DROPOUT and train_ops.linear_applicable(x, mods[i + 1].linear):
                    # the dropout folded into the linear's kernels (dtupd.h *_drop)
                    drop = float(m.p) if m.training else 0.0
                    i += 1
                    m = mods[i]
            if self.fused_tail and isinstance(m, _Lin) and x.is_cuda:
                from aido1_amd import train_ops
                if train_ops.linear_applicable(x, m.linear):
                    act = mods[i + 1] if i + 1 < k else None
                    # linear -> leaky_relu in one; its backward reads the
                    # gradient off the sign of the saved output, which is only
                    # the input's sign for a non-negative slope
                    if isinstance(act, nn.LeakyReLU) and act.negative_slope >= 0:
                        x = train_ops.linear(x, m.linear, float(act.negative_slope), drop=drop)
                        i += 2
                    else:
                        x = train_ops.linear(x, m.linear, drop=drop)
                        i += 1
                    continue
            if isinstance(m, nn.BatchNorm2d) and getattr(m, '_dt_updates', 1) != 1:
                raise NotImplementedError('repeated running-statistics updates need the fused '
                                          'train-mode tail (train_ops)')
            x = m(x)
            i += 1
        return x


class _Net(nn.Module):       # Net: input_nets / output_nets (modules.py:86-109)
    def __init__(self, inputs, outputs):
        super().__init__()
        self.input_nets = nn.ModuleList(inputs)
        self.output_nets = nn.ModuleList(outputs)

    def forward(self, *inputs):
        return self.out([net(v) for net, v in zip(self.input_nets, inputs)])

    def out(self, parts):
        """The output branches on the concatenated input branches.  On the GPU
        in float32 a single small output branch (linear [-> act] [-> linear
        [-> act]]) runs as one dt_mlp_fwd launch reading the parts in place
        (train_ops.mlp, include/dthead.h) instead of torch.cat + two library
        GEMMs + activations."""
        if len(self.output_nets) == 1 and self.output_nets[0].fused_tail and parts[0].is_cuda:
            from aido1_amd import train_ops
            plan = train_ops.mlp_plan(self.output_nets[0], parts)
            if plan is not None:
                return [train_ops.mlp(parts, plan)]
        x = torch.cat(parts, dim=1)
        return [net(x) for net in self.output_nets]

    def td_target(self, inputs, rew, notdone, gamma):
        """rew + notdone * gamma * forward(*inputs) (training/trainers.py:166-170)
        without gradients; on the GPU in float32 the output branch and the
        target are one dt_mlp_fwd_td launch (include/dthead.h)."""
        parts = [net(v) for net, v in zip(self.input_nets, inputs)]
        if len(self.output_nets) == 1 and self.output_nets[0].fused_tail and parts[0].is_cuda:
            from aido1_amd import train_ops
            plan = train_ops.mlp_plan(self.output_nets[0], parts)
            if plan is not None and train_ops.td_applicable(parts, rew, notdone):
                return train_ops.mlp_td(parts, plan, rew, notdone, gamma)
        return rew + notdone * gamma * self.out(parts)[0]


def _build_branch(spec):
    """One branch of config.json's module list -> list of modules (index-aligned
    with the reference's MetaNet so state_dict keys match; modules.py:111-142)."""
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
            if a.get('padding', 0) != 0:
                raise NotImplementedError('padding')
            mods.append(_Conv(last, a['out_channels'], a['kernel_size'], a['stride'],
                              a.get('weight_init')))
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
            mods.append(_Lin(last, a['out_features'], a.get('weight_init')))
            last = a['out_features']
        elif name == 'tanh':
            mods.append(nn.Tanh())
        elif name == 'sigmoid':
            mods.append(nn.Sigmoid())
        else:
            raise NotImplementedError(name)
    return mods


def _branches(config, kind):
    return [s for m in config if m['name'] == kind for s in m['modules']]


class ConfigNet(nn.Module):
    """models/ddpg/modules.py Actor / Critic: a Net from a config.json module
    list; forward(*inputs) concatenates the input branches and returns the
    first output branch (modules.py:168-194)."""

    def __init__(self, net_config):
        super().__init__()
        self.net = _Net([_Seq(_build_branch(b)) for b in _branches(net_config, 'inputs')],
                        [_Seq(_build_branch(b)) for b in _branches(net_config, 'outputs')])

    def forward(self, *inputs):
        return self.net(*inputs)[0]


class ConfigActor(ConfigNet):
    """models/ddpg/modules.py Actor built from config.json's "actor" list
    (single input branch, single output branch, as config.json:19-91)."""

    def __init__(self, actor_config):
        super().__init__(actor_config)
        ins, outs = _branches(actor_config, 'inputs'), _branches(actor_config, 'outputs')
        if len(ins) != 1 or len(outs) != 1:
            raise NotImplementedError('one input and one output branch')
        last = outs[0][-1]['name']
        self.head = {'tanh': 'tanh', 'sigmoid': 'sigmoid'}.get(last, 'none')
        self.max_action = 1.0

    def layers(self):
        mods = list(self.net.input_nets[0].internal_modules)
        convs = [m.kernel for m in mods if isinstance(m, _Conv)]
        bns = [m for m in mods if isinstance(m, nn.BatchNorm2d)]
        lins = [m.linear for m in mods if isinstance(m, _Lin)]
        lins += [m.linear for m in self.net.output_nets[0].internal_modules if isinstance(m, _Lin)]
        if len(convs) != 4 or len(bns) != 4 or len(lins) != 2:
            raise NotImplementedError('fused path expects 4 conv/bn pairs and 2 linears')
        return convs, bns, lins[0], lins[1]


class ConfigCritic(ConfigNet):
    """models/ddpg/modules.py Critic from config.json's "critic" list: conv
    trunk -> linear 256 on the observation, the action passed through, both
    concatenated (258) -> linear 128 -> linear 1 (config.json:93-170).

    trunk(obs) + head(t, action) == forward(obs, action): the trunk is the
    observation branch up to its first dropout or linear (the conv stack and
    flatten, a function of obs and the conv weights only), the head the rest
    (dropout draws included).  The trainer shares one trunk between two
    forwards that see the same weights and batch."""

    def _cut(self):
        mods = self.net.input_nets[0].internal_modules
        for j, m in enumerate(mods):
            if isinstance(m, (nn.Dropout, _Lin)):
                return j
        return len(mods)

    def trunk(self, obs):
        return self.net.input_nets[0].run(obs, 0, self._cut())

    def head(self, t, *rest):
        seq = self.net.input_nets[0]
        x0 = seq.run(t, self._cut(), len(seq.internal_modules))
        return self.net.out([x0] + [net(v) for net, v in zip(self.net.input_nets[1:], rest)])[0]

    def td_target(self, obs, action, rew, notdone, gamma):
        """rew + notdone * gamma * forward(obs, action), no gradients (the
        trainer's target y; _Net.td_target)."""
        return self.net.td_target([obs, action], rew, notdone, gamma)


def apply_head(x, head, max_action=1.0):
    if head == 'tanh':
        return torch.tanh(x)
    if head == 'sigmoid':
        return torch.sigmoid(x)
    if head == 'sigmoid_tanh':  # ActorCNN: [sigmoid * max_action, tanh]
        return torch.stack([max_action * torch.sigmoid(x[:, 0]), torch.tanh(x[:, 1])], 1)
    return x


class FusedActor(nn.Module):
    """Inference copy of an actor for the batched rollout, weights in `dtype`
    (fp16 by default in the rollout: under per-sample normalisation bf16's
    8-bit mantissa costs ~5e-2 in the actions vs ~6e-3 for fp16 on rendered
    frames, tools/actor_precision.py; both run on MFMA at the same rate), convolutions channels_last (MIOpen's NHWC bf16 kernels are
    ~1.75x its NCHW ones on these shapes, tools/actor_micro.py), the first
    conv's input channels re-ordered per call so it reads the frame ring in
    place.  Two modes:

    * ``'reference'`` — what the reference's explorers compute: every model is
      in train mode (managers.py:264-268, explorers.py:46) and acts on a batch
      of ONE observation (models/ddpg/model.py:74-88), so each BatchNorm
      normalises a sample with that sample's own per-channel mean and biased
      variance over H x W, and the 0.5 dropout is live.  Batched here as
      per-sample statistics (float32 accumulation) + affine.
    * ``'eval'`` — eval-mode BatchNorm (running statistics) folded into the
      next conv / the first linear: the checkpoint-evaluation policy
      (test-ddpg-cnn.py, DDPG.act after .eval()).

    Numerically within bf16 rounding of the float32 modules
    (tests/test_gpu_actor.py).  ``refresh(actor)`` re-derives the weights in
    place (the acting copy follows the trainer's target actor)."""

    def __init__(self, actor, dtype=torch.bfloat16, mode='eval'):
        super().__init__()
        if mode not in ('eval', 'reference'):
            raise ValueError(mode)
        convs, bns, lin1, lin2 = actor.layers()
        self.mode = mode
        self.head = actor.head
        self.max_action = getattr(actor, 'max_action', 1.0)
        self.dtype = dtype
        self.strides = [conv.stride for conv in convs]
        self.eps = [bn.eps for bn in bns]
        drops = [m for m in actor.modules() if isinstance(m, nn.Dropout)]
        self.p_drop = drops[0].p if drops else 0.0
        cl = torch.channels_last
        dev = convs[0].weight.device
        self.w = nn.ParameterList([nn.Parameter(torch.empty_like(c.weight, dtype=dtype)
                                                .contiguous(memory_format=cl), requires_grad=False)
                                   for c in convs])
        self.b = nn.ParameterList([nn.Parameter(torch.empty_like(c.bias, dtype=dtype),
                                                requires_grad=False) for c in convs])
        self.gamma = nn.ParameterList([nn.Parameter(torch.empty(bn.num_features, device=dev),
                                                    requires_grad=False) for bn in bns])
        self.beta = nn.ParameterList([nn.Parameter(torch.empty(bn.num_features, device=dev),
                                                   requires_grad=False) for bn in bns])
        self.w1 = nn.Parameter(torch.empty_like(lin1.weight, dtype=dtype), requires_grad=False)
        self.b1 = nn.Parameter(torch.empty_like(lin1.bias, dtype=dtype), requires_grad=False)
        self.w2 = nn.Parameter(torch.empty_like(lin2.weight, dtype=dtype), requires_grad=False)
        self.b2 = nn.Parameter(torch.empty_like(lin2.bias, dtype=dtype), requires_grad=False)
        # the convs as MFMA A fragments for dt_conv1 / dt_conv32 (fp16 path,
        # include/dtactor.h), biases in f32
        self.register_buffer('w0frag', torch.zeros(16, 64, 8, dtype=torch.float16, device=dev))
        self.register_buffer('wfrag', torch.zeros(3, 32, 64, 8, dtype=torch.float16, device=dev))
        self.register_buffer('bf', torch.zeros(4, 32, device=dev))
        # the float32-accurate chain (dt_conv1x_split / dt_conv32x_split,
        # reference mode in float32): conv1's fragments as (hi, lo) fp16
        # halves, conv2..4's in float32
        self.x3 = dtype == torch.float32 and mode == 'reference'
        if dtype == torch.float16 and tuple(lin1.weight.shape) == (512, FLAT):
            # the fast mode's head (dt_actor_head_f16_drop): lin1's fp16
            # weights in the head fragment layout
            self.register_buffer('w1f', torch.zeros(16, 252, 64, 8, dtype=torch.float16,
                                                    device=dev))
        if self.x3:
            self.register_buffer('w0x', torch.zeros(2, 16, 64, 8, dtype=torch.float16, device=dev))
            self.register_buffer('wx32', torch.zeros(3, 32, 64, 8, device=dev))
            if tuple(lin1.weight.shape) == (512, FLAT):   # dt_actor_head_x3's lin1 fragments
                self.register_buffer('w1x', torch.zeros(2, 16, 252, 64, 8, dtype=torch.float16,
                                                        device=dev))
        self.refresh(actor, graph=False)

    @torch.no_grad()
    def refresh(self, actor, graph=None):
        """Re-derive the acting weights from `actor`'s current ones, in place.
        On the GPU the ~12 copy / gather kernels of a refresh are captured into
        a HIP graph at the first refresh from a given source (its parameters'
        addresses) and replayed afterwards: the training loop refreshes both
        acting copies after every update, and issued one by one from Python
        the kernels left the GPU idle ~0.4 ms a decision (launch gaps).
        graph=False forces the eager path."""
        dev = self.w0frag.device
        if graph is None:
            graph = dev.type == 'cuda'
        if not graph:
            return self._refresh(actor)
        if self.mode == 'reference' and (self.dtype == torch.float16 or self.x3):
            return self._refresh_gather(actor)
        # the source's tensors are listed once per source module (walking the
        # module tree costs ~80 us of host time a call); their addresses are
        # checked on every call, so a source whose storage moved is recaptured
        srcs = self.__dict__.setdefault('_refresh_srcs', {})
        ts = srcs.get(id(actor))
        if ts is None or ts[0] is not actor:
            ts = srcs[id(actor)] = (actor, list(actor.parameters()) + list(actor.buffers()))
        key = (id(actor),) + tuple(t.data_ptr() for t in ts[1])
        cache = self.__dict__.setdefault('_refresh_graphs', {})
        g = cache.get(key)
        if g is None:
            self._refresh(actor)                 # eager once: lazily built index maps, pools
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._refresh(actor)
            cache[key] = g
        g.replay()

    def _refresh_pairs(self, actor):
        """(destination, source, logical index map or None, kind) of a
        reference-mode refresh: what _refresh copies, with the fragment
        gathers' index maps; kind 2 = the x3 (hi, lo) pair into dst[0], dst[1]
        (dt_refresh_copy), None = by the destination's dtype."""
        convs, bns, lin1, lin2 = actor.layers()
        pairs = [(d, sp, None, None) for d, sp in zip(
            list(self.w) + list(self.b) + list(self.gamma) + list(self.beta) +
            [self.w1, self.b1, self.w2, self.b2],
            [c.weight for c in convs] + [c.bias for c in convs] + [bn.weight for bn in bns] +
            [bn.bias for bn in bns] + [lin1.weight, lin1.bias, lin2.weight, lin2.bias])]
        dev = self.w0frag.device
        if getattr(self, '_fidx', None) is None or self._fidx[0].device != dev:
            self._fidx = (conv1_fragment_index(dev), conv32_fragment_index(dev))
            self._w0pad = torch.zeros(32 * 3 * 64 + 1, device=dev)
        n0 = convs[0].weight.numel()
        f0 = self._fidx[0].reshape(-1)
        f0 = torch.where(f0 < n0, f0, torch.full_like(f0, -1))
        pairs.append((self.w0frag, convs[0].weight, f0, None))
        for i in range(1, 4):
            pairs.append((self.wfrag[i - 1], convs[i].weight, self._fidx[1].reshape(-1), None))
        if self.x3:   # the x3 chain's fragments
            pairs.append((self.w0x, convs[0].weight, f0, 2))
            for i in range(1, 4):
                pairs.append((self.wx32[i - 1], convs[i].weight, self._fidx[1].reshape(-1), None))
            if hasattr(self, 'w1x'):
                if getattr(self, '_h1idx', None) is None or self._h1idx.device != dev:
                    self._h1idx = head_fragment_index(dev)
                pairs.append((self.w1x, lin1.weight, self._h1idx, 2))
        if hasattr(self, 'w1f'):   # the fp16 head's fragments (from float32: fp16 rounding)
            if getattr(self, '_h1idx', None) is None or self._h1idx.device != dev:
                self._h1idx = head_fragment_index(dev)
            pairs.append((self.w1f, lin1.weight, self._h1idx, None))
        for i in range(4):
            pairs.append((self.bf[i], convs[i].bias, None, None))
        return pairs

    @staticmethod
    def _phys_map(dst, src, logical=None):
        """For every element of dst in its physical order, the physical offset
        in src of the element copied there (src's logical element, or
        src.flatten()[logical[...]] with -1 kept); None for a plain copy."""
        n = src.numel()
        dev = src.device
        ar = torch.arange(n, device=dev, dtype=torch.int64)
        src_phys = ar.as_strided(tuple(src.shape), tuple(src.stride())).reshape(-1)
        if logical is None:
            lg = torch.empty_strided(tuple(dst.shape), tuple(dst.stride()), dtype=torch.int64,
                                     device=dev)
            lg.copy_(torch.arange(dst.numel(), device=dev, dtype=torch.int64).view(dst.shape))
            lg = lg.as_strided((dst.numel(),), (1,))
            m = src_phys[lg]
            return None if torch.equal(m, torch.arange(dst.numel(), device=dev)) else m
        if not dst.is_contiguous():
            raise ValueError('refresh: a gathered destination must be contiguous')
        lg = logical.reshape(-1).to(dev)
        return torch.where(lg >= 0, src_phys[lg.clamp(min=0)], lg)

    def _refresh_gather(self, actor):
        """A reference-mode fp16 refresh as ONE dt_refresh_copy launch
        (include/dtactor.h): every acting tensor gathered and converted from
        the source's float32 parameters through index maps built at the first
        refresh from a source (its tensors' addresses are checked every call).
        Issued as ~28 small kernels (or their graph) it cost ~0.19 ms of GPU
        time a decision in the training loop."""
        import ctypes
        from aido1_amd import _lib
        srcs = self.__dict__.setdefault('_refresh_srcs', {})
        ts = srcs.get(id(actor))
        if ts is None or ts[0] is not actor:
            ts = srcs[id(actor)] = (actor, list(actor.parameters()) + list(actor.buffers()))
        key = (id(actor),) + tuple(t.data_ptr() for t in ts[1])
        cache = self.__dict__.setdefault('_refresh_tables', {})
        ent = cache.get(key)
        if ent is None:
            pairs = self._refresh_pairs(actor)
            keep, rows = [], []
            for dst, src, lg, kind in pairs:
                if src.dtype != torch.float32 or dst.dtype not in (torch.float16, torch.float32):
                    raise ValueError('refresh: float32 sources, fp16 / f32 destinations')
                if kind == 2 and not (dst.is_contiguous() and dst.dtype == torch.float16):
                    raise ValueError('refresh: an x3 pair is a contiguous fp16 [2, ...]')
                half = dst[0] if kind == 2 else dst      # an x3 pair: the map of its hi half
                m = self._phys_map(half, src.detach(), lg)
                if m is not None:
                    keep.append(m)
                if kind is None:
                    kind = 1 if dst.dtype == torch.float16 else 0
                rows.append(_lib.DtCopyEntry(src.data_ptr(), dst.data_ptr(),
                                             m.data_ptr() if m is not None else None,
                                             half.numel(), kind, 0))
            arr = (_lib.DtCopyEntry * len(rows))(*rows)
            table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(
                self.w0frag.device)
            ent = cache[key] = (table, keep, len(rows), max(r.count for r in rows))
        table, _keep, n, most = ent
        rc = _lib.lib().dt_refresh_copy(n, table.data_ptr(), most,
                                        torch.cuda.current_stream(table.device).cuda_stream)
        if rc != 0:
            raise _lib.DtError('dt_refresh_copy failed (%d)' % rc)

    def _refresh(self, actor):
        convs, bns, lin1, lin2 = actor.layers()
        if self.mode == 'reference':
            ws = [c.weight for c in convs]
            bs = [c.bias for c in convs]
            copy_grouped(
                list(self.w) + list(self.b) + list(self.gamma) + list(self.beta) +
                [self.w1, self.b1, self.w2, self.b2],
                ws + bs + [bn.weight for bn in bns] + [bn.bias for bn in bns] +
                [lin1.weight, lin1.bias, lin2.weight, lin2.bias])
            if hasattr(self, 'w1x'):
                if getattr(self, '_h1idx', None) is None or self._h1idx.device != self.w1.device:
                    self._h1idx = head_fragment_index(self.w1.device)
                self.w1x.view(2, -1).copy_(split_hl(torch.take(self.w1, self._h1idx)))
        else:
            scale = shift = None
            ws, bs = [], []
            for i, (conv, bn) in enumerate(zip(convs, bns)):
                w = conv.weight.detach().double()
                b = conv.bias.detach().double()
                if scale is not None:   # fold previous BN: conv(s*x + t)
                    b = b + (w * shift.view(1, -1, 1, 1)).sum((1, 2, 3))
                    w = w * scale.view(1, -1, 1, 1)
                self.w[i].copy_(w)
                self.b[i].copy_(b)
                ws.append(w)
                bs.append(b)
                scale = bn.weight.detach().double() / torch.sqrt(
                    bn.running_var.detach().double() + bn.eps)
                shift = bn.bias.detach().double() - bn.running_mean.detach().double() * scale
            w1 = lin1.weight.detach().double()
            b1 = lin1.bias.detach().double()
            s_flat = scale.repeat_interleave(FLAT // scale.numel())
            t_flat = shift.repeat_interleave(FLAT // shift.numel())
            self.w1.copy_(w1 * s_flat.view(1, -1))
            self.b1.copy_(b1 + w1 @ t_flat)
            self.w2.copy_(lin2.weight)
            self.b2.copy_(lin2.bias)
        if hasattr(self, 'w1f'):   # from the acting w1 (folded in eval mode)
            if getattr(self, '_h1idx', None) is None or self._h1idx.device != self.w1.device:
                self._h1idx = head_fragment_index(self.w1.device)
            self.w1f.view(-1).copy_(torch.take(self.w1, self._h1idx))
        self._fragments(ws, bs)

    def _fragments(self, ws, bs):
        """The MFMA A fragments (fp16) and f32 biases of the four convs for
        dt_conv1 / dt_conv32, from weights of any float dtype and memory
        format: one gather a layer through index maps built once (the layouts
        of conv1_fragments / conv32_fragments)."""
        dev = self.w0frag.device
        if getattr(self, '_fidx', None) is None or self._fidx[0].device != dev:
            self._fidx = (conv1_fragment_index(dev), conv32_fragment_index(dev))
            self._w0pad = torch.zeros(32 * 3 * 64 + 1, device=dev)   # + the zero channel's slot
        self._w0pad[:-1].view(32, 3, 8, 8).copy_(ws[0])
        self.w0frag.view(-1).copy_(torch.take(self._w0pad, self._fidx[0]))
        for i in range(1, 4):
            self.wfrag[i - 1].view(-1).copy_(torch.take(ws[i], self._fidx[1]))
        torch._foreach_copy_(list(self.bf.unbind(0)), list(bs))
        if self.x3:
            self.w0x.view(2, -1).copy_(split_hl(torch.take(self._w0pad, self._fidx[0])))
            for i in range(1, 4):
                self.wx32[i - 1].view(-1).copy_(torch.take(ws[i], self._fidx[1]))

    def _lrelu_sample_norm(self, x, i):
        """LeakyReLU then BatchNorm2d in train mode on a batch of one, for every
        sample at once: the dt_sample_norm HIP kernel (include/dtactor.h) on
        the GPU, in place; a two-pass torch restatement on CPU (tests)."""
        if x.is_cuda:
            from aido1_amd import _lib
            n, c, h, w = x.shape
            assert x.is_contiguous(memory_format=torch.channels_last)
            dt = {torch.bfloat16: 0, torch.float32: 1, torch.float16: 2}[x.dtype]
            L = _lib.lib()
            rc = L.dt_sample_norm(x.data_ptr(), x.data_ptr(), n, h * w, c,
                                  self.gamma[i].data_ptr(), self.beta[i].data_ptr(),
                                  self.eps[i], 0.01, dt,
                                  torch.cuda.current_stream(x.device).cuda_stream)
            if rc != 0:
                raise _lib.DtError('dt_sample_norm failed (%d)' % rc)
            return x
        x = F.leaky_relu(x).float()
        mean = x.mean((2, 3), keepdim=True)
        var = (x - mean).square().mean((2, 3), keepdim=True)
        g = self.gamma[i].view(1, -1, 1, 1)
        b = self.beta[i].view(1, -1, 1, 1)
        return ((x - mean) / torch.sqrt(var + self.eps[i]) * g + b).to(self.dtype)

    def _convs_hip(self, ring, order):
        """The four convolutions by the hand-written MFMA kernels (include/dtactor.h):
        dt_conv1 straight from the ring (grey f32, or palette-index u8 through
        dt_conv1_index_split), then dt_conv32 x3; in reference
        mode every per-sample BatchNorm is applied by the next kernel while it
        stages its input (the last one in conv4's epilogue).  Returns the
        flattened [N, 4032] fp16 activation in NCHW order."""
        from aido1_amd import _lib
        L = _lib.lib()
        n, slots = ring.shape[0], ring.shape[1]
        dev = ring.device
        flat = torch.empty(n, FLAT, dtype=torch.float16, device=dev)
        rc = self._convs(L, ring, slots, order, flat, self._conv_buffers(n, dev))
        if rc != 0:
            raise _lib.DtError('dt_conv1 / dt_conv32 failed (%d)' % rc)
        return flat

    def _conv_buffers(self, n, dev):
        """The intermediate activations (fp16 NHWC) and, in reference mode, the
        per-sample BatchNorm statistics [n, 32, 3] of conv1..conv3 (mean of the
        stored centred values, M2, centre: include/dtactor.h)."""
        key = (n, dev, self.mode)
        if getattr(self, '_bufs_key', None) != key:
            f16 = torch.float16
            ref = self.mode == 'reference'
            self._bufs = {
                'y1': torch.empty(n, 57, 77, 32, dtype=f16, device=dev),
                'y2': torch.empty(n, 27, 37, 32, dtype=f16, device=dev),
                'y3': torch.empty(n, 12, 17, 32, dtype=f16, device=dev),
                'p1': torch.empty(n, 32, 3, device=dev) if ref else None,
                'p2': torch.empty(n, 32, 3, device=dev) if ref else None,
                'p3': torch.empty(n, 32, 3, device=dev) if ref else None}
            self._bufs_key = key
        return self._bufs

    def _convs(self, L, ring, slots, order, flat, B):
        import ctypes
        n = ring.shape[0]
        ref = self.mode == 'reference'
        stream = torch.cuda.current_stream(ring.device).cuda_stream
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        o = (ctypes.c_int32 * 3)(*[int(v) for v in order])
        conv1 = L.dt_conv1_index_split if ring.dtype == torch.uint8 else L.dt_conv1_split
        rc = conv1(ring.data_ptr(), n, slots, o, self.w0frag.data_ptr(), self.bf[0].data_ptr(),
                   None, B['y1'].data_ptr(), ptr(B['p1']), 0.01, stream)
        ins = [(B['y1'], B['p1']), (B['y2'], B['p2']), (B['y3'], B['p3'])]
        outs = [(B['y2'], B['p2']), (B['y3'], B['p3']), (flat, None)]
        for layer in range(3):
            if rc != 0:
                break
            x, pp = ins[layer]
            y, po = outs[layer]
            last = layer == 2
            rc = L.dt_conv32(
                layer + 2, n, x.data_ptr(), self.wfrag[layer].data_ptr(),
                self.bf[layer + 1].data_ptr(), ptr(pp),
                self.gamma[layer].data_ptr() if ref else None,
                self.beta[layer].data_ptr() if ref else None, self.eps[layer] if ref else 0.0,
                y.data_ptr(), ptr(po),
                self.gamma[3].data_ptr() if (ref and last) else None,
                self.beta[3].data_ptr() if (ref and last) else None,
                self.eps[3] if ref else 0.0, 0.01, stream)
        return rc

    def _x3_input(self, x):
        """x is a frame ring the float32-accurate HIP chain takes."""
        return (self.x3 and x.is_cuda and x.dtype in (torch.float32, torch.uint8) and
                x.is_contiguous() and tuple(x.shape[2:]) == (120, 160) and x.shape[1] >= 3 and
                self.w[0].shape == (32, 3, 8, 8))

    def _x3_buffers(self, n, dev):
        """The HLB activations ((hi, lo) fp16 pairs, include/dtactor.h) of
        conv1..conv3, their per-sample statistics [n, 32, 3] and the f32
        flattened conv4 output."""
        key = (n, dev)
        if getattr(self, '_xbufs_key', None) != key:
            f16 = torch.float16
            self._xbufs = {   # each in the layout its consumer reads (stride 2, 2, 1)
                'y1': torch.empty(hlb_shape(n, 57, 77, 2), dtype=f16, device=dev),
                'y2': torch.empty(hlb_shape(n, 27, 37, 2), dtype=f16, device=dev),
                'y3': torch.empty(hlb_shape(n, 12, 17, 1), dtype=f16, device=dev),
                'p1': torch.empty(n, 32, 3, device=dev),
                'p2': torch.empty(n, 32, 3, device=dev),
                'p3': torch.empty(n, 32, 3, device=dev),
                'flat': torch.empty(n, FLAT, device=dev)}
            self._xbufs_key = key
        return self._xbufs

    def _convs_x3(self, ring, order, other=None, n0=None):
        """The four convolutions at float32 accuracy (dt_conv1x_split, then
        dt_conv32x_split x3; include/dtactor.h): every per-sample BatchNorm is
        folded into the next layer's weights, the last one applied in conv4's
        epilogue.  With `other`, samples [n0, n) use its weights in the same
        launches.  Returns the flattened [N, 4032] float32 activation (NCHW
        order); it is the buffers' own memory, valid until the next call."""
        import ctypes
        from aido1_amd import _lib
        L = _lib.lib()
        n, slots = ring.shape[0], ring.shape[1]
        B = self._x3_buffers(n, ring.device)
        stream = torch.cuda.current_stream(ring.device).cuda_stream
        o = (ctypes.c_int32 * 3)(*[int(v) for v in order])
        s1 = None if other is None else ctypes.byref(_lib.DtConvSet(
            n0, other.w0x.data_ptr(), other.bf[0].data_ptr()))
        rc = L.dt_conv1x_split(ring.data_ptr(), 1 if ring.dtype == torch.uint8 else 0, n, slots,
                               o, self.w0x.data_ptr(), self.bf[0].data_ptr(), s1,
                               B['y1'].data_ptr(), B['p1'].data_ptr(), 0.01, stream)
        ins = [(B['y1'], B['p1']), (B['y2'], B['p2']), (B['y3'], B['p3'])]
        outs = [(B['y2'], B['p2']), (B['y3'], B['p3']), (B['flat'], None)]
        for layer in range(3):
            if rc != 0:
                break
            x, pp = ins[layer]
            y, po = outs[layer]
            last = layer == 2
            s2 = None
            if other is not None:
                s2 = ctypes.byref(_lib.DtConvSet(
                    n0, other.wx32[layer].data_ptr(), other.bf[layer + 1].data_ptr(),
                    other.gamma[layer].data_ptr(), other.beta[layer].data_ptr(),
                    other.gamma[3].data_ptr() if last else None,
                    other.beta[3].data_ptr() if last else None))
            rc = L.dt_conv32x_split(
                layer + 2, n, x.data_ptr(), self.wx32[layer].data_ptr(),
                self.bf[layer + 1].data_ptr(), pp.data_ptr(), self.gamma[layer].data_ptr(),
                self.beta[layer].data_ptr(), self.eps[layer], y.data_ptr(),
                po.data_ptr() if po is not None else None,
                self.gamma[3].data_ptr() if last else None,
                self.beta[3].data_ptr() if last else None, self.eps[3], 0.01, s2, stream)
        if rc != 0:
            raise _lib.DtError('dt_conv1x_split / dt_conv32x_split failed (%d)' % rc)
        return B['flat']

    def _pairable(self, other, x):
        if other is None or other.mode != self.mode or not x.is_cuda:
            return False
        if self.x3 and other.x3:
            return self._x3_input(x) and other.w[0].shape == (32, 3, 8, 8)
        return (self.dtype == torch.float16 and other.dtype == torch.float16 and
                x.dtype in (torch.float32, torch.uint8) and x.is_contiguous() and
                tuple(x.shape[2:]) == (120, 160) and x.shape[1] >= 3 and
                self.w[0].shape == (32, 3, 8, 8) and other.w[0].shape == (32, 3, 8, 8))

    @torch.no_grad()
    def forward_pair(self, other, x, order, n0, out=None):
        """The samples [0, n0) through this actor and [n0, n) through `other`
        (the exploiting explorers' copy, rollout.ActorRollout) with ONE launch
        per convolution: dt_conv1_split / dt_conv32_split split the persistent
        workgroups between the two weight sets (include/dtactor.h).  Returns
        [n, 2] (into `out` if given); each row equals the forward of its own
        actor."""
        n = x.shape[0]
        if out is None:
            out = torch.empty(n, 2, dtype=torch.float32, device=x.device)
        if not self._pairable(other, x) or not 0 < n0 < n:
            out[:n0] = self(x[:n0], order)
            out[n0:] = other(x[n0:], order)
            return out
        if self.x3:
            flat = self._convs_x3(x, order, other, n0)
            if self._head_x3_ok(flat, other):
                return self._heads_x3(other, flat, n0, out)
            out[:n0] = self._head(flat[:n0])
            out[n0:] = other._head(flat[n0:])
            return out
        flat = self._convs_pair(other, x, order, n0)
        if self._head_fusable(other):
            return self._heads(other, flat, n0, out)
        for a, sl in ((self, slice(0, n0)), (other, slice(n0, n))):
            out[sl] = a._head(flat[sl])
        return out

    def _convs_pair(self, other, x, order, n0):
        """_convs_hip over both weight sets: the flattened [n, 4032] fp16
        activations, rows [0, n0) from this actor's weights, the rest from
        `other`'s."""
        import ctypes
        from aido1_amd import _lib
        L = _lib.lib()
        n = x.shape[0]
        ref = self.mode == 'reference'
        flat = torch.empty(n, FLAT, dtype=torch.float16, device=x.device)
        B = self._conv_buffers(n, x.device)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        o = (ctypes.c_int32 * 3)(*[int(v) for v in order])
        s1 = _lib.DtConvSet(n0, other.w0frag.data_ptr(), other.bf[0].data_ptr())
        conv1 = L.dt_conv1_index_split if x.dtype == torch.uint8 else L.dt_conv1_split
        rc = conv1(x.data_ptr(), n, x.shape[1], o, self.w0frag.data_ptr(), self.bf[0].data_ptr(),
                   ctypes.byref(s1), B['y1'].data_ptr(), ptr(B['p1']), 0.01, stream)
        ins = [(B['y1'], B['p1']), (B['y2'], B['p2']), (B['y3'], B['p3'])]
        outs = [(B['y2'], B['p2']), (B['y3'], B['p3']), (flat, None)]
        for layer in range(3):
            if rc != 0:
                break
            xi, pp = ins[layer]
            y, po = outs[layer]
            last = layer == 2
            s2 = _lib.DtConvSet(n0, other.wfrag[layer].data_ptr(), other.bf[layer + 1].data_ptr(),
                                ptr(other.gamma[layer]) if ref else None,
                                ptr(other.beta[layer]) if ref else None,
                                ptr(other.gamma[3]) if (ref and last) else None,
                                ptr(other.beta[3]) if (ref and last) else None)
            rc = L.dt_conv32_split(
                layer + 2, n, xi.data_ptr(), self.wfrag[layer].data_ptr(),
                self.bf[layer + 1].data_ptr(), ptr(pp),
                self.gamma[layer].data_ptr() if ref else None,
                self.beta[layer].data_ptr() if ref else None, self.eps[layer] if ref else 0.0,
                y.data_ptr(), ptr(po),
                self.gamma[3].data_ptr() if (ref and last) else None,
                self.beta[3].data_ptr() if (ref and last) else None,
                self.eps[3] if ref else 0.0, 0.01, ctypes.byref(s2), stream)
        if rc != 0:
            raise _lib.DtError('dt_conv1_split / dt_conv32_split failed (%d)' % rc)
        return flat

    _HEAD_CODES = {'none': 0, 'tanh': 1, 'sigmoid': 2}

    def _head_fusable(self, other=None):
        nets = [self] if other is None else [self, other]
        return all(a.dtype == torch.float16 and a.w2.is_cuda and a.w2.shape[0] == 2 and
                   a.head == self.head and a.head in self._HEAD_CODES and
                   a.w1.shape == self.w1.shape and a.w1.shape[0] % 8 == 0 for a in nets)

    def _heads(self, other, flat, n0, out):
        """_head over rows [0, n0) with this actor and [n0, n) with `other`:
        dropout + lin1 per weight set (hipBLASLt into one [n, 512] buffer),
        then LeakyReLU -> lin2 -> head for every row in ONE dt_actor_head
        launch (include/dtactor.h), written into out [n, 2] f32."""
        import ctypes
        from aido1_amd import _lib
        o = other if other is not None else self
        if (hasattr(self, 'w1f') and hasattr(o, 'w1f') and flat.dtype == torch.float16
                and flat.is_contiguous() and tuple(flat.shape[1:]) == (FLAT,)
                and o.p_drop == self.p_drop and o.mode == self.mode):
            return self._heads_f16(o, flat, n0, out)
        n, k = flat.shape[0], self.w1.shape[0]
        h = torch.empty(n, k, dtype=torch.float16, device=flat.device)
        for a, sl in ((self, slice(0, n0)), (o, slice(n0, n))):
            if sl.stop > sl.start:
                x = flat[sl]
                if a.mode == 'reference' and a.p_drop > 0:
                    x = F.dropout(x, a.p_drop, training=True)
                torch.addmm(a.b1, x, a.w1.t(), out=h[sl])
        rc = _lib.lib().dt_actor_head(
            n, n0, k, h.data_ptr(), k, self.w2.data_ptr(), self.b2.data_ptr(), o.w2.data_ptr(),
            o.b2.data_ptr(), self._HEAD_CODES[self.head], 0.01, out.data_ptr(),
            ctypes.c_void_p(torch.cuda.current_stream(flat.device).cuda_stream))
        if rc != 0:
            raise _lib.DtError('dt_actor_head failed (%d)' % rc)
        return out

    def _drop_seed(self, p):
        """A fresh key for the head's folded dropout (one a call), from a
        base drawn once from torch's generator."""
        if p <= 0:
            return 0
        if getattr(self, '_drop_key', None) is None:
            self._drop_key = [int(torch.randint(0, 2 ** 31, (1,)).item()), 0]
        self._drop_key[1] += 1
        return (self._drop_key[0] + 0x9E3779B9 * self._drop_key[1]) & 0xFFFFFFFF

    def _heads_f16(self, o, flat, n0, out):
        """The fast mode's head (dropout -> lin1 -> LeakyReLU -> lin2 -> head)
        for both weight sets in one dt_actor_head_f16_drop launch pair: lin1
        on fp16 MFMA with f32 accumulation, the dropout folded into its
        staging (include/dtactor.h)."""
        import ctypes
        from aido1_amd import _lib
        p = self.p_drop if self.mode == 'reference' else 0.0
        L = _lib.lib()
        n = flat.shape[0]
        work = getattr(self, '_hwork', None)
        if work is None or work.numel() < L.dt_actor_head_x3_work_floats(n) or \
                work.device != flat.device:
            work = self._hwork = torch.empty(int(L.dt_actor_head_x3_work_floats(n)),
                                             device=flat.device)
        rc = L.dt_actor_head_f16_drop(
            n, n0, FLAT, flat.data_ptr(), float(p), self._drop_seed(p), self.w1f.data_ptr(),
            self.b1.data_ptr(), self.w2.data_ptr(), self.b2.data_ptr(), o.w1f.data_ptr(),
            o.b1.data_ptr(), o.w2.data_ptr(), o.b2.data_ptr(), self._HEAD_CODES[self.head], 0.01,
            work.data_ptr(), out.data_ptr(),
            ctypes.c_void_p(torch.cuda.current_stream(flat.device).cuda_stream))
        if rc != 0:
            raise _lib.DtError('dt_actor_head_f16_drop failed (%d)' % rc)
        return out

    def _head_x3_ok(self, x, other=None):
        nets = [self] if other is None else [self, other]
        return (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and
                tuple(x.shape[1:]) == (FLAT,) and
                all(hasattr(a, 'w1x') and a.head in self._HEAD_CODES and
                    tuple(a.w2.shape) == (2, 512) for a in nets))

    def _heads_x3(self, other, x, n0, out):
        """dropout (reference mode) -> lin1 -> LeakyReLU -> lin2 -> head at
        float32 accuracy in ONE dt_actor_head_x3_drop launch pair
        (include/dtactor.h; the dropout folded into lin1's staging): rows
        [0, n0) with this actor's weights, [n0, n) with `other`'s."""
        import ctypes
        from aido1_amd import _lib
        o = other if other is not None else self
        p = self.p_drop if self.mode == 'reference' else 0.0
        if p > 0 and o.p_drop != self.p_drop:     # one rate a launch: torch's dropout
            x = F.dropout(x, p, training=True)
            p = 0.0
        # the dropout folded into lin1's staging (dt_actor_head_x3_drop): a
        # fresh counter-based key a call, drawn from torch's generator once
        seed = self._drop_seed(p)
        L = _lib.lib()
        n = x.shape[0]
        work = getattr(self, '_hwork', None)
        if work is None or work.numel() < L.dt_actor_head_x3_work_floats(n) or \
                work.device != x.device:
            work = self._hwork = torch.empty(int(L.dt_actor_head_x3_work_floats(n)),
                                             device=x.device)
        rc = L.dt_actor_head_x3_drop(
            n, n0, FLAT, x.data_ptr(), float(p), seed, self.w1x.data_ptr(), self.b1.data_ptr(),
            self.w2.data_ptr(), self.b2.data_ptr(), o.w1x.data_ptr(), o.b1.data_ptr(),
            o.w2.data_ptr(), o.b2.data_ptr(), self._HEAD_CODES[self.head], 0.01, work.data_ptr(),
            out.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        if rc != 0:
            raise _lib.DtError('dt_actor_head_x3 failed (%d)' % rc)
        return out

    def _head(self, x):
        """dropout (reference mode) -> lin1 -> LeakyReLU -> lin2 -> head."""
        if self._head_x3_ok(x) and x.shape[0] > 0:
            out = torch.empty(x.shape[0], 2, dtype=torch.float32, device=x.device)
            return self._heads_x3(None, x, x.shape[0], out)
        if self.mode == 'reference' and self.p_drop > 0:
            x = F.dropout(x, self.p_drop, training=True)
        x = F.leaky_relu(F.linear(x, self.w1, self.b1))
        x = F.linear(x, self.w2, self.b2).float()
        return apply_head(x, self.head, self.max_action)

    @torch.no_grad()
    def forward(self, x, order=None):
        """x: [N,3,120,160] stack (oldest first), or the frame ring with
        `order` = ring slots oldest->newest (RenderOutput.order()); grey
        float32 or palette-index uint8 frames (render.py)."""
        # MIOpen's heuristic choice for conv2 at these shapes is a 2.5 ms CK
        # kernel; its benchmark-mode search finds a 0.57 ms one (once per shape)
        with torch.backends.cudnn.flags(enabled=True, benchmark=True,
                                        deterministic=False, allow_tf32=False):
            return self._forward(x, order)

    def _forward(self, x, order):
        ref = self.mode == 'reference'
        if self._x3_input(x):
            # the reference-precision product path: the float32-accurate HIP convs
            return self._head(self._convs_x3(x, order if order is not None else [0, 1, 2]))
        if (x.is_cuda and self.dtype == torch.float16 and
                x.dtype in (torch.float32, torch.uint8) and
                x.is_contiguous() and tuple(x.shape[2:]) == (120, 160) and x.shape[1] >= 3 and
                self.w[0].shape == (32, 3, 8, 8)):
            # the fp16 product path: all four convs are the hand-written MFMA kernels
            x = self._convs_hip(x, order if order is not None else [0, 1, 2])
            if self._head_fusable() and x.shape[0] > 0:
                out = torch.empty(x.shape[0], 2, dtype=torch.float32, device=x.device)
                return self._heads(None, x, x.shape[0], out)
        else:
            from aido1_amd.render import as_gray
            x = as_gray(x)
            w0 = self.w[0]
            if order is not None:
                inv = sorted(range(len(order)), key=lambda c: order[c])
                w0 = w0[:, inv].contiguous(memory_format=torch.channels_last)
            x = x.to(self.dtype, memory_format=torch.channels_last)
            for i in range(4):
                x = F.conv2d(x, w0 if i == 0 else self.w[i], self.b[i], stride=self.strides[i])
                x = self._lrelu_sample_norm(x, i) if ref else F.leaky_relu(x)
            # flatten in NCHW order, as the reference's view(x.size(0), -1)
            x = x.contiguous().flatten(1)
        return self._head(x)


def copy_grouped(dsts, srcs):
    """dst.copy_(src) for every pair, one torch._foreach_copy_ per (dst dtype,
    src dtype) group.  A single _foreach_copy_ over destinations of mixed
    dtypes is NOT safe on this ROCm build: its multi-tensor kernel wrote the
    fp16 conversion of the sources into the float32 destinations too (the
    reference-mode actor's BatchNorm gamma / beta held fp16 bit pairs in their
    first half and stale memory in the rest -- NaN after a test that left NaN
    in freed memory; tools/nan_repro.py)."""
    groups = {}
    for d, s in zip(dsts, srcs):
        groups.setdefault((d.dtype, s.dtype, d.device), ([], []))
        groups[(d.dtype, s.dtype, d.device)][0].append(d)
        groups[(d.dtype, s.dtype, d.device)][1].append(s)
    for ds, ss in groups.values():
        torch._foreach_copy_(ds, ss)


def split_hl(t):
    """A float32 tensor as its (hi, lo) fp16 halves stacked in a new first
    dim: hi = fp16(t), lo = fp16((t - hi) * 2^11) (the x3 operands of
    include/dtactor.h's dt_conv1x_split)."""
    hi = t.half()
    return torch.stack([hi, ((t - hi.float()) * 2048.0).half()])


def hlb_geometry(w, stride):
    """The HLB layout of a w-wide image read at `stride` by its consumer
    (include/dtactor.h): the chunks a segment holds, and pixel x's chunk."""
    half = (w + 1) // 2
    if stride == 2:
        return 2 * half, [(half + x // 2) if x % 2 else x // 2 for x in range(w)]
    return w, list(range(w))


def hlb_shape(n, h, w, stride):
    """fp16 shape of n HLB images: [n, h, 4 blocks, {hi, lo}, chunks, 8]."""
    return (n, h, 4, 2, hlb_geometry(w, stride)[0], 8)


def hlb_decode(y, h, w, stride):
    """n HLB images -> float64 [n, h, w, 32]: hi + 2^-11 lo (test helper)."""
    segpx, pos = hlb_geometry(w, stride)
    t = y.reshape(-1, h, 4, 2, segpx, 8)[:, :, :, :, pos, :]
    v = t[:, :, :, 0].double() + t[:, :, :, 1].double() / 2048.0     # [n, h, 4, w, 8]
    return v.permute(0, 1, 3, 2, 4).reshape(-1, h, w, 32)


def hlb_encode(x, stride):
    """float32 [n, h, w, 32] -> its HLB images (test helper)."""
    n, h, w, _ = x.shape
    segpx, pos = hlb_geometry(w, stride)
    out = torch.zeros(hlb_shape(n, h, w, stride), dtype=torch.float16, device=x.device)
    out[:, :, :, :, pos, :] = split_hl(x.float()).reshape(2, n, h, w, 4, 8).permute(
        1, 2, 4, 0, 3, 5)
    return out


def conv1_fragments(w, dtype=torch.float16):
    """conv1 weights [32, 3, 8, 8] -> dt_conv1's MFMA A fragments [16, 64, 8]
    (fp16, or `dtype`): element [s][l][j] = w[l % 32][j % 4][s // 2][4 (s % 2)
    + 2 (l // 32) + j // 4], zero for the padding channel j % 4 == 3."""
    dev = w.device
    s = torch.arange(16, device=dev).view(16, 1, 1)
    ln = torch.arange(64, device=dev).view(1, 64, 1)
    j = torch.arange(8, device=dev).view(1, 1, 8)
    wp = torch.cat([w.float(), torch.zeros(w.shape[0], 1, 8, 8, device=dev)], 1)
    return wp[ln % 32, j % 4, s // 2, 4 * (s % 2) + 2 * (ln // 32) + j // 4].to(dtype)


def conv32_fragments(w, dtype=torch.float16):
    """A 32 -> 32 4x4 conv's weights [32, 32, 4, 4] -> dt_conv32's MFMA A
    fragments [32, 64, 8] (fp16, or `dtype`): element [s][l][j] = w[l % 32][16
    (s % 2) + 8 (l // 32) + j][(s // 2) // 4][(s // 2) % 4]."""
    dev = w.device
    s = torch.arange(32, device=dev).view(32, 1, 1)
    ln = torch.arange(64, device=dev).view(1, 64, 1)
    j = torch.arange(8, device=dev).view(1, 1, 8)
    return w.float()[ln % 32, 16 * (s % 2) + 8 * (ln // 32) + j, (s // 2) // 4,
                     (s // 2) % 4].to(dtype)


def head_fragment_index(dev):
    """dt_actor_head_x3's lin1 fragment layout as flat indices into lin1's
    weights [512, 4032]: element [t][s][l][j] = w1[32 t + l % 32][16 s + 8
    (l // 32) + j]."""
    t = torch.arange(16, device=dev).view(16, 1, 1, 1)
    s = torch.arange(252, device=dev).view(1, 252, 1, 1)
    ln = torch.arange(64, device=dev).view(1, 1, 64, 1)
    j = torch.arange(8, device=dev).view(1, 1, 1, 8)
    return ((32 * t + ln % 32) * FLAT + 16 * s + 8 * (ln // 32) + j).reshape(-1)


def conv1_fragment_index(dev):
    """conv1_fragments' layout as flat indices into the weights [32, 3, 8, 8]
    viewed 1-D, the padding channel pointing past them (at a zero)."""
    s = torch.arange(16, device=dev).view(16, 1, 1)
    ln = torch.arange(64, device=dev).view(1, 64, 1)
    j = torch.arange(8, device=dev).view(1, 1, 8)
    c = j % 4
    flat = ((ln % 32) * 3 + c) * 64 + (s // 2) * 8 + 4 * (s % 2) + 2 * (ln // 32) + j // 4
    return torch.where(c < 3, flat, torch.full_like(flat, 32 * 3 * 64)).reshape(-1)


def conv32_fragment_index(dev):
    """conv32_fragments' layout as flat indices into the weights [32, 32, 4, 4]."""
    s = torch.arange(32, device=dev).view(32, 1, 1)
    ln = torch.arange(64, device=dev).view(1, 64, 1)
    j = torch.arange(8, device=dev).view(1, 1, 8)
    ci = 16 * (s % 2) + 8 * (ln // 32) + j
    return ((((ln % 32) * 32 + ci) * 4 + (s // 2) // 4) * 4 + (s // 2) % 4).reshape(-1)


def flops_per_sample():
    """Multiply-adds x 2 of the actor trunk + head for one 3x120x160 input."""
    shapes = [(3, 32, 8, 57, 77), (32, 32, 4, 27, 37), (32, 32, 4, 12, 17), (32, 32, 4, 9, 14)]
    f = sum(2 * ci * co * k * k * ho * wo for ci, co, k, ho, wo in shapes)
    return f + 2 * FLAT * 512 + 2 * 512 * 2


def x3_bytes_per_sample(frame_bytes=1):
    """HBM bytes one sample moves through the float32-accurate chain
    (dt_conv1x_split, dt_conv32x_split x3, the first linear): the three
    stacked frames read (palette index: 1 B a pixel), each layer's HL
    activations (4 B an element) written once and read once, the f32
    flattened conv4 output written and read by lin1.  Weights and
    statistics are per launch, not per sample, and left out."""
    frames = 3 * 120 * 160 * frame_bytes
    hl = sum(h * w * 32 * 4 for h, w in ((57, 77), (27, 37), (12, 17)))
    return frames + 2 * hl + 2 * FLAT * 4


def clone_eval(actor):
    a = copy.deepcopy(actor)
    a.eval()
    return a
