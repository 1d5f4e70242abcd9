"""DDPG update on the GPU (BASELINE config 5).

``DDPGTrainer.update`` follows training/trainers.py:143-237 step for step:

  1. lr of both optimisers from TrainingDecay at the global update step
     (utils/util.py:77-90, linear decay in config.json);
  2. target actor -> target critic on next_obs (train mode: BatchNorm on batch
     statistics, running stats updated — all reference models are .train());
  3. y = r + notdone * gamma * Q'(s', pi'(s'));
  4. critic MSE (or smooth-L1) backward, Adam step;
  5. actor loss -mean Q(s, pi(s)) backward, Adam step;
  6. soft update of both targets, tau (models/torch_utils.py:5-9);
  7. td_error = y - Q(s, a) under no_grad (trainers.py:223-229), returned for
     the prioritized replay's update_priorities.

Multi-GPU: the reference's periodic barrier + parameter averaging
across trainer processes (trainers.py:206-213) becomes an RCCL all-reduce of
the gradients before each optimiser step (distributed.GradAllReduce), which
keeps every rank's replica identical.

Layout: modules and image batches are channels_last.  Besides being MIOpen's
faster convolution layout, it selects MIOpen's NHWC BatchNorm: its NCHW
train-mode BatchNorm loses precision on large H x W planes (5.8e-3 max error
on a 57x77 N(3, 2) plane vs ~1e-6 for NHWC or torch's native kernel,
tools/bn_probe.py), which the train-mode networks here hit every update.

Metrics stay on the device (no .item() inside update) so the update can run
back to back with the rollout without host synchronisation.

HIP graphs (``graph=True``, GPU only): a batch-64 update is ~400 small
kernels, so it is launch-bound.  The update is split in three stages at the
two gradient all-reduces (critic: targets + critic loss + backward; critic
step + actor loss + backward; actor step + soft updates + TD error).  The
first ``warmup`` updates run eagerly (MIOpen algorithm selection, optimiser
state creation), then each stage is captured once and replayed: one graph
when there is nothing to all-reduce, three with the RCCL all-reduces run
between them otherwise.  Inputs are copied into static buffers; Adam is the
capturable variant with a device-tensor learning rate set by fill_ before
each replay.  Dropout draws stay fresh per replay (graph-safe Philox offsets).
"""
import contextlib
import copy

import torch
import torch.nn.functional as F

from aido1_amd.distributed import GradAllReduce, world
from aido1_amd.explore import create_decay_fn
from aido1_amd.guard import Guard
from aido1_amd.optim import DeviceAdam, SoftUpdate, make_optimizer
from aido1_amd import train_ops


class TrainingDecay:
    """utils/util.py:77-90: per-hyperparameter decay functions applied to an
    optimiser param group."""

    def __init__(self, config):
        self.decays = {name: create_decay_fn(c['type'], **c['args']) for name, c in config.items()}
        self.realization = {}

    def __call__(self, params):
        for name, v in self.realization.items():
            if isinstance(params[name], torch.Tensor):
                params[name].fill_(v)           # capturable optimiser: lr lives on the device
            else:
                params[name] = v

    def update_step(self, step):
        for name, fn in self.decays.items():
            self.realization[name] = fn(step)


_SOFT = SoftUpdate()


def soft_update(target, source, tau):
    """models/torch_utils.py:5-9: t <- t * (1 - tau) + p * tau (two products
    rounded separately, as the reference's expression); one dt_soft_update
    launch on the GPU (optim.SoftUpdate)."""
    _SOFT(target, source, tau)


def hard_update(target, source):
    """models/torch_utils.py:12-14."""
    torch._foreach_copy_([p.data for p in target.parameters()],
                         [p.data for p in source.parameters()])


def _nullctx():
    return contextlib.nullcontext()


class DDPGTrainer:
    def __init__(self, config, actor, critic, target_actor=None, target_critic=None,
                 device=None, sync_grads=None, bucket_mb=16, graph=False, warmup=3,
                 conv_search=True, guard=None):
        t = config['training']
        self.config = config
        self.gamma, self.tau = float(t['gamma']), float(t['tau'])
        self.critic_loss_kind = t.get('critic_loss', 'mse_loss')
        if self.critic_loss_kind not in ('mse_loss', 'smooth_l1_loss'):
            raise NotImplementedError(self.critic_loss_kind)
        self.device = torch.device(device) if device is not None else \
            next(actor.parameters()).device
        self.dtype = next(actor.parameters()).dtype      # float32 (float64 for parity tests)
        self.actor, self.critic = actor.to(self.device), critic.to(self.device)
        self.target_actor = (target_actor if target_actor is not None
                             else copy.deepcopy(actor)).to(self.device)
        self.target_critic = (target_critic if target_critic is not None
                              else copy.deepcopy(critic)).to(self.device)
        for m in (self.actor, self.critic, self.target_actor, self.target_critic):
            m.to(memory_format=torch.channels_last)
            m.train()                           # managers.py:264-268 _prime_model
        self.graph = bool(graph) and self.device.type == 'cuda'
        if self.graph and t['optimizer'] != 'adam':
            raise NotImplementedError('graph capture needs the capturable Adam')
        self.actor_optim = make_optimizer(t['optimizer'], self.actor.parameters(), self.graph,
                                          self.device)
        self.critic_optim = make_optimizer(t['optimizer'], self.critic.parameters(), self.graph,
                                           self.device)
        # non-finite guards (guard.py): every stage reports into one device
        # block, read only by check()
        self.guard = guard if guard is not None else Guard(self.device)
        if self.device.type == 'cuda':
            for m in (self.actor, self.critic, self.target_actor, self.target_critic):
                train_ops.attach_guard(m, self.guard)
        for opt, stages in ((self.actor_optim, ('actor_grad', 'actor_param')),
                            (self.critic_optim, ('critic_grad', 'critic_param'))):
            if isinstance(opt, DeviceAdam):
                opt.set_guard(self.guard, *stages)
        self.warmup = warmup
        # stream layout of the stages (A/B: tools/update_only.py AB_ATTR=...)
        self.multi_stream = True      # independent forwards on a side stream (_fork)
        self.split_target = False     # + the target critic trunk on a third (measured slower)
        self.fold_dropout = True      # dropouts folded into the linears after them (train_ops)
        self._pending_grads = {}      # module id -> its autograd gradients (_grads -> _opt_step)
        self.conv_search = bool(conv_search)
        self._graphs = None
        self._in = None
        self.actor_decay = TrainingDecay(t['actor_train_decay'])
        self.critic_decay = TrainingDecay(t['critic_train_decay'])
        self.global_update_step = 0
        if sync_grads is None:
            sync_grads = world()[1] > 1
        self.sync_actor = GradAllReduce(self.actor.parameters(), bucket_mb) if sync_grads else None
        self.sync_critic = GradAllReduce(self.critic.parameters(), bucket_mb) if sync_grads \
            else None

    def _tensor(self, x, dtype=None):
        return torch.as_tensor(x, device=self.device).to(dtype or self.dtype)

    def _inputs(self, train_data):
        observations, actions, rewards, next_observations, dones = train_data
        cl = torch.channels_last
        x = {'obs': self._tensor(observations).contiguous(memory_format=cl),
             'nxt': self._tensor(next_observations).contiguous(memory_format=cl),
             'act': self._tensor(actions),
             'rew': self._tensor(rewards).reshape(-1, 1),
             'notdone': (~self._tensor(dones, torch.bool).reshape(-1, 1)).to(self.dtype)}
        if not self.graph:
            self._in = x
        elif self._in is None:
            self._in = {k: v.clone(memory_format=torch.preserve_format) for k, v in x.items()}
        else:
            for k, v in x.items():
                if v.shape != self._in[k].shape:
                    raise ValueError('graph mode needs a fixed batch shape')
                self._in[k].copy_(v)

    def static_inputs(self, batch, obs_shape=(3, 120, 160)):
        """The inputs an update reads (graph mode: the captured graphs' static
        tensors), for a producer that writes them in place (TrainLoop: the
        replay's dt_frame_gather); then update_prepared()."""
        if self._in is None:
            cl = torch.channels_last
            z = (lambda *s: torch.zeros(*s, device=self.device, dtype=self.dtype))
            self._in = {'obs': z(batch, *obs_shape).contiguous(memory_format=cl),
                        'nxt': z(batch, *obs_shape).contiguous(memory_format=cl),
                        'act': z(batch, 2), 'rew': z(batch, 1), 'notdone': z(batch, 1)}
        if self._in['obs'].shape[0] != batch:
            raise ValueError('graph mode needs a fixed batch shape')
        return self._in

    def _grads(self, loss, module):
        """zero_grad + loss.backward() for `module`'s parameters
        (trainers.py:178-179, 197-198) as torch.autograd.grad: the same
        gradients, written into .grad, and none computed for the other
        networks on the path.  The reference's actor_loss.backward() also
        runs the critic's whole backward and fills the critic's .grad, which
        its next critic_optim.zero_grad() discards unread; here the critic's
        conv trunk (independent of the actor) is not differentiated at all."""
        params = [p for p in module.parameters() if p.requires_grad]
        # a persistent 1 as the seed: no fill kernel a backward
        one = getattr(self, '_one', None)
        if one is None or one.device != loss.device or one.dtype != loss.dtype:
            one = self._one = torch.ones((), device=loss.device, dtype=loss.dtype)
        grads = torch.autograd.grad(loss, params, grad_outputs=one, allow_unused=True,
                                    materialize_grads=True)
        opt = self.actor_optim if module is self.actor else self.critic_optim
        if (self.graph and isinstance(opt, DeviceAdam) and len(params) == len(list(
                module.parameters())) and (self.sync_actor if module is self.actor
                                            else self.sync_critic) is None):
            # graph mode, one rank: dt_adam reads the autograd outputs
            # themselves (their addresses are fixed in the graph's pool), so
            # no copy into .grad (two multi-tensor kernels an update)
            self._pending_grads[id(module)] = list(grads)
            return
        if all(p.grad is not None for p in params):
            torch._foreach_copy_([p.grad for p in params], list(grads))
        else:   # .grad in the parameter's own memory format (DeviceAdam's layout)
            for p, g in zip(params, grads):
                p.grad = torch.empty_like(p).copy_(g)

    # ---- the three stages (trainers.py:156-229) ------------------------------------
    def _fork(self):
        """A side stream joined to the current one (GPU), or None (CPU)."""
        if self.device.type != 'cuda' or not self.multi_stream:
            return None
        if getattr(self, '_side', None) is None:
            self._side = torch.cuda.Stream(self.device)
        self._side.wait_stream(torch.cuda.current_stream(self.device))
        return self._side

    def _fork2(self):
        """A second side stream joined to the current one (GPU)."""
        if getattr(self, '_side2', None) is None:
            self._side2 = torch.cuda.Stream(self.device)
        self._side2.wait_stream(torch.cuda.current_stream(self.device))
        return self._side2

    @staticmethod
    def _join_on(stream, other, *tensors):
        """`stream` waits for `other`; tensors made on `other` are used on it."""
        stream.wait_stream(other)
        for t in tensors:
            t.record_stream(stream)

    def _join(self, side, *tensors):
        if side is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_stream(side)
            for t in tensors:
                t.record_stream(cur)

    def _opt_step(self, opt, module, grad_stage, param_stage):
        """opt.step() with its gradients and results guarded: DeviceAdam reports
        from inside dt_adam, any other optimiser is scanned around."""
        if isinstance(opt, DeviceAdam):
            opt.step(grads=self._pending_grads.pop(id(module), None))
            return
        params = [p for p in module.parameters() if p.grad is not None]
        self.guard.scan(grad_stage, *[p.grad for p in params])
        opt.step()
        self.guard.scan(param_stage, *[p.data for p in params])

    def save(self, directory, episode, reward, target=True):
        """A checkpoint in the reference's layout (models/ddpg/model.py:130-140,
        aido1_amd/checkpoint.py).  target=True saves the target networks: the
        weights the reference's exploiters act with and save
        (training/explorers.py:104-105, 142-152); False the online ones."""
        from aido1_amd import checkpoint
        actor, critic = ((self.target_actor, self.target_critic) if target
                         else (self.actor, self.critic))
        return checkpoint.save(self.config, directory, episode, reward, actor, critic)

    def load(self, directory):
        """Load a checkpoint directory (the reference's or save()'s) into the
        online and the target networks (DDPG.load, then the hard copy the
        trainer starts from)."""
        from aido1_amd import checkpoint
        checkpoint.load(directory, self.actor, self.critic)
        checkpoint.load(directory, self.target_actor, self.target_critic)

    def check(self):
        """Raise guard.NonFiniteError naming the stages of the updates since the
        last check that produced NaN / Inf (synchronises)."""
        return self.guard.check('DDPG update')

    # folded dropouts an update draws (train_ops.drop_pool): the target actor,
    # the target critic, the critic, the actor and the critic's head twice
    DROP_SITES = 6

    def _drop_width(self):
        """The flatten width every folded dropout of the two networks sees
        (the input of a linear right after a dropout), or None."""
        ks = set()
        for net in (self.actor, self.critic):
            for seq in getattr(getattr(net, 'net', None), 'input_nets', []):
                mods = list(seq.internal_modules)
                for j in range(len(mods) - 1):
                    if (isinstance(mods[j], torch.nn.Dropout) and mods[j].p > 0
                            and hasattr(mods[j + 1], 'linear')):
                        ks.add(mods[j + 1].linear.in_features)
        return ks.pop() if len(ks) == 1 else None

    def _drop_open(self):
        """One launch draws every folded dropout's uniforms of the update
        (instead of one dropout kernel a site); closed by _drop_close."""
        train_ops.FOLD_DROPOUT = self.fold_dropout
        k = self._drop_width() if (self.device.type == 'cuda' and self.dtype == torch.float32
                                   and self.fold_dropout) else None
        if k is None:
            return
        self._drop_ctx = train_ops.drop_pool(self.DROP_SITES, self._in['obs'].shape[0], k,
                                             self.device)
        self._drop_buf = self._drop_ctx.__enter__()

    def _drop_close(self):
        ctx = getattr(self, '_drop_ctx', None)
        if ctx is not None:
            ctx.__exit__(None, None, None)
            self._drop_ctx = None

    def _stage_critic(self):
        x = self._in
        self.guard.tick()
        self._drop_open()
        self.guard.scan('batch', x['obs'], x['act'], x['rew'], x['nxt'])
        # the targets' forward (target actor -> target critic on next_obs) and
        # the critic's forward on obs are independent: two streams, so their
        # batch-64 kernels (a few CUs each) run side by side -- in a HIP graph
        # two branches of the captured DAG
        side = self._fork()
        # the target critic's conv trunk does not depend on the target actor's
        # action: a third stream, so the target branch is one trunk deep
        # instead of two (the trunk draws no dropout, so the RNG order holds)
        side2 = self._fork2() if (side is not None and self.split_target and
                                  hasattr(self.target_critic, 'trunk')) else None
        if side2 is not None:
            with torch.cuda.stream(side2), torch.no_grad():
                t_next = self.target_critic.trunk(x['nxt'])
        with torch.cuda.stream(side) if side is not None else _nullctx():
            with torch.no_grad():
                next_actions = self.target_actor(x['nxt'])
                if side2 is not None:
                    self._join_on(side, side2, t_next)
                    next_v = self.target_critic.head(t_next, next_actions)
                    self._y = x['rew'] + x['notdone'] * self.gamma * next_v
                elif hasattr(self.target_critic, 'td_target'):
                    # the head and the target in one launch on the GPU
                    self._y = self.target_critic.td_target(x['nxt'], next_actions, x['rew'],
                                                           x['notdone'], self.gamma)
                else:
                    next_v = self.target_critic(x['nxt'], next_actions)
                    self._y = x['rew'] + x['notdone'] * self.gamma * next_v
                self.guard.scan('target', self._y)
        y_predicted = self.critic(x['obs'], x['act'])
        self._join(side, self._y)
        if self.critic_loss_kind == 'mse_loss':
            critic_loss = train_ops.mse_loss(y_predicted, self._y)
        else:
            critic_loss = F.smooth_l1_loss(y_predicted, self._y)
        self._grads(critic_loss, self.critic)
        self._critic_loss = critic_loss.detach()
        self.guard.scan('critic_loss', self._critic_loss)

    def _shared_trunk(self):
        """Share the critic's conv trunk between the actor-loss forward and the
        TD-error forward (trainers.py:190-192, 223-226): both run the critic
        after its step and before anything else changes it, on the same
        observations, so the trunk output is the same tensor; only the head
        (dropout, linears, with the action) runs twice.  The BatchNorms move
        their running statistics twice, as the two reference forwards do
        (dt_bn_leaky_fwd updates = 2).  The actor loss needs no gradient
        through the trunk (it does not depend on the actor).  GPU float32 with
        the fused train-mode tail only; elsewhere the two full forwards run."""
        return (self.device.type == 'cuda' and self.dtype == torch.float32
                and hasattr(self.critic, 'trunk'))

    def _stage_actor(self):
        x = self._in
        self._opt_step(self.critic_optim, self.critic, 'critic_grad', 'critic_param')
        if self._shared_trunk():
            # the (stepped) critic's trunk and the actor's forward are
            # independent until the head: two streams, two graph branches
            side = self._fork()
            with torch.cuda.stream(side), torch.no_grad(), \
                    train_ops.running_updates(self.critic, 2):
                self._trunk = self.critic.trunk(x['obs'])
            pred_actions = self.actor(x['obs'])
            self._join(side, self._trunk)
            q = self.critic.head(self._trunk, pred_actions)
        else:
            pred_actions = self.actor(x['obs'])
            q = self.critic(x['obs'], pred_actions)
        actor_loss = train_ops.neg_mean(q)
        self._grads(actor_loss, self.actor)
        self._actor_loss = actor_loss.detach()
        self.guard.scan('actor_loss', self._actor_loss)

    def _stage_targets(self):
        x = self._in
        # the TD-error forward reads only the (already stepped) critic: it runs
        # beside the actor step and the soft updates
        side = self._fork()
        with torch.cuda.stream(side) if side is not None else _nullctx():
            with torch.no_grad():                                    # trainers.py:223-229
                if self._shared_trunk():
                    q = self.critic.head(self._trunk, x['act'])
                else:
                    q = self.critic(x['obs'], x['act'])
                self._td = self._y - q
                self.guard.scan('td', self._td)
        self._opt_step(self.actor_optim, self.actor, 'actor_grad', 'actor_param')
        # trainers.py:215-216, both pairs in one launch
        _SOFT.many([(self.target_actor, self.actor), (self.target_critic, self.critic)], self.tau)
        self._join(side, self._td)
        self._drop_close()
        with torch.no_grad():
            self._metrics = (torch.sqrt(self._critic_loss), self._actor_loss)

    def _capture(self):
        stages = [self._stage_critic, self._stage_actor, self._stage_targets]
        groups = [stages] if self.sync_actor is None else [[st] for st in stages]
        self._graphs = []
        for group in groups:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for st in group:
                    st()
            self._graphs.append(g)
        for opt in (self.actor_optim, self.critic_optim):
            if isinstance(opt, DeviceAdam):
                opt.finish_capture()

    def update(self, train_data):
        """train_data = (obs, actions, rewards, next_obs, dones), leading batch
        dimension (numpy or tensors).  Returns (metrics, info) like the
        reference; metric values are 0-dim device tensors (valid until the
        next update in graph mode)."""
        self._inputs(train_data)
        return self.update_prepared()

    def update_prepared(self):
        """update() on the inputs already in static_inputs() (written in place
        by the caller on the current stream)."""
        self.critic_decay.update_step(self.global_update_step)
        self.actor_decay.update_step(self.global_update_step)
        for group in self.critic_optim.param_groups:
            self.critic_decay(group)
        for group in self.actor_optim.param_groups:
            self.actor_decay(group)
        with self._conv_flags():
            self._run_stages()
        self.global_update_step += 1
        metrics = {'critic_loss': self._metrics[0], 'actor_loss': self._metrics[1]}
        return metrics, {'td_error': self._td}

    def _conv_flags(self):
        """MIOpen Find mode for the update's convolutions (cudnn.benchmark): the
        first update of each shape searches the solvers and later ones (and the
        captured graphs) reuse the fastest.  With the default heuristic every
        convolution call also ran a MIOpen tensor op (SubTensorOpWithScalar1d,
        ~5.8 us, one per call in profiles/r03_train_kernel_stats.csv);
        measured update 2.56 -> 2.25 ms per decision (tools/train_phases.py
        with and without TP_CUDNN_BENCH)."""
        if self.device.type != 'cuda' or not self.conv_search:
            return _nullctx()
        cd = torch.backends.cudnn
        return cd.flags(enabled=cd.enabled, benchmark=True, deterministic=cd.deterministic,
                        allow_tf32=cd.allow_tf32)

    def _run_stages(self):
        syncs = [self.sync_critic, self.sync_actor, None]
        if self.graph and self.global_update_step >= self.warmup:
            if self._graphs is None:
                self._capture()
            if len(self._graphs) == 1:
                self._graphs[0].replay()
            else:
                for g, sync in zip(self._graphs, syncs):
                    g.replay()
                    if sync is not None:
                        sync()
        else:
            for st, sync in zip((self._stage_critic, self._stage_actor, self._stage_targets),
                                syncs):
                st()
                if sync is not None:
                    sync()
