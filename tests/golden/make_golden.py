"""Generate the golden fixtures in tests/golden/ by importing the reference.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py [/root/reference]

The reference is pure Python; the pieces on this path that import without its
absent dependencies are imported directly.  Minimal in-process stand-ins are
installed for the modules the reference imports but that are not installed and
that the captured code paths never exercise in a way that matters:
  - ``gym`` (Wrapper base classes + spaces.Box): the wrappers only call
    ``__init__(env)`` and read ``observation_space``;
  - ``scipy.misc.imresize`` (removed from scipy) and ``skimage.color`` (absent):
    only needed so utils/reward_shaping/env_utils.py imports; the captured
    Transformer stacking never calls them on meaningful data;
  - ``tensorboardX``/``requests`` are not needed by the modules imported here.
The gym-duckietown Simulator is absent, so EnvironmentWrapper fixtures drive the
reference's own EnvironmentWrapper code over the oracle's SimulatorRef: they pin
the wrapper's repeat / break / reward-shaping / in-place action mapping, not the
Simulator.

Outputs are JSON (small) and .npz (arrays); nothing here is reference source.
"""
import json
import math
import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = sys.argv[1] if len(sys.argv) > 1 else '/root/reference'


def install_stubs():
    gym = types.ModuleType('gym')

    class Wrapper:
        def __init__(self, env=None):
            self.env = env
            self.observation_space = getattr(env, 'observation_space', None)
            self.action_space = getattr(env, 'action_space', None)

        def reset(self):
            return self.observation(self.env.reset()) if hasattr(self, 'observation') \
                else self.env.reset()

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.shape = tuple(shape) if shape is not None else np.shape(low)
            self.low = np.full(self.shape, low, dtype) if np.isscalar(low) else low
            self.high = np.full(self.shape, high, dtype) if np.isscalar(high) else high
            self.dtype = dtype

    gym.Wrapper = Wrapper
    gym.ObservationWrapper = type('ObservationWrapper', (Wrapper,), {})
    gym.ActionWrapper = type('ActionWrapper', (Wrapper,), {})
    gym.RewardWrapper = type('RewardWrapper', (Wrapper,), {})
    gym.make = lambda *a, **k: None
    spaces = types.ModuleType('gym.spaces')
    spaces.Box = Box
    gym.spaces = spaces
    sys.modules['gym'] = gym
    sys.modules['gym.spaces'] = spaces

    import scipy.misc
    from PIL import Image

    def imresize(arr, size):
        h, w = size[:2]
        return np.asarray(Image.fromarray(np.asarray(arr, np.uint8)).resize((w, h),
                                                                              Image.BILINEAR))
    scipy.misc.imresize = imresize
    sk = types.ModuleType('skimage')
    color = types.ModuleType('skimage.color')
    color.rgb2gray = lambda rgb: (np.asarray(rgb, np.float64) / 255.0) @ \
        np.array([0.2125, 0.7154, 0.0721])
    sk.color = color
    sys.modules['skimage'] = sk
    sys.modules['skimage.color'] = color
    tb = types.ModuleType('tensorboardX')
    tb.SummaryWriter = object
    sys.modules.setdefault('tensorboardX', tb)


def dump(name, obj):
    with open(os.path.join(HERE, name), 'w') as f:
        json.dump(obj, f, indent=None, separators=(',', ':'))
    print('wrote', name)


def gen_bresenham():
    from utils.bresenham import bresenham
    rng = random.Random(1234)
    cases = [(0, 0, 0, 0), (0, 0, 5, 0), (0, 0, 0, 5), (0, 0, -5, 0), (0, 0, 0, -5),
             (0, 0, 5, 3), (0, 0, 3, 5), (0, 0, -5, 3), (0, 0, -3, 5), (0, 0, 5, -3),
             (0, 0, 3, -5), (0, 0, -5, -3), (0, 0, -3, -5), (0, 0, 4, 4), (0, 0, -4, 4),
             (2, 3, 2, 3), (10, 7, -6, 7), (159, 119, 0, 0), (0, 119, 159, 0)]
    for _ in range(150):
        cases.append(tuple(rng.randint(-40, 170) for _ in range(4)))
    dump('bresenham.json', [{'line': list(c), 'points': [list(p) for p in bresenham(*c)]}
                            for c in cases])


def gen_aggregation():
    from utils.reward_shaping.aggregation_functions import BaselineAggregationFunction
    from duckietown_rl.wrappers import DtRewardWrapper
    f = BaselineAggregationFunction({})
    rng = np.random.default_rng(5)
    xs = [-1000, -1000.0, 0, 0.0, -0.0, 1e-300, -1e-300, 0.5, -0.5, 1.2, -999.999999, -1000.0001,
          5e-324] + [float(v) for v in rng.normal(0, 5, 200)]
    w = DtRewardWrapper(None)
    dump('aggregation.json', [{'r': x, 'baseline': f(None, None, x), 'dt_reward_wrapper':
                               w.reward(x)} for x in xs])


def gen_steering():
    from duckietown_rl.wrappers import ActionWrapper, SteeringToWheelVelWrapper

    class Dummy:
        observation_space = None
        action_space = None
    # wrapper order of train-ddpg-cnn.py:48-50 / solution.py:35-36:
    # env = ActionWrapper(env); env = SteeringToWheelVelWrapper(env)
    # -> the agent's action goes through SteeringToWheelVel.action first, then
    #    ActionWrapper.action (x0.8 on element 0 = the LEFT wheel).
    inner = ActionWrapper(Dummy())
    outer = SteeringToWheelVelWrapper(inner)
    rng = np.random.default_rng(6)
    acts = [(0.5, 0.0), (0.4, 0.3), (1.0, 1.0), (-1.0, -1.0), (0.0, 0.0), (1.0, -8.0), (0.2, 20.0),
            (0.05, -0.5)] + [tuple(float(v) for v in rng.uniform(-1.5, 1.5, 2)) for _ in range(200)]
    out = []
    for a in acts:
        wheels = outer.action(np.array(a))
        final = inner.action(wheels)
        out.append({'action': list(a), 'wheels': [float(v) for v in wheels],
                    'sim_action': [float(v) for v in final]})
    # float32 inputs (the actor emits float32)
    acts32 = rng.uniform(-1, 1, (100, 2)).astype(np.float32)
    for a in acts32:
        wheels = outer.action(a)
        final = inner.action(wheels)
        out.append({'action32': [float(v) for v in a], 'wheels': [float(v) for v in wheels],
                    'sim_action': [float(v) for v in final]})
    dump('steering.json', out)


def gen_stacking():
    from duckietown_rl.wrappers import ImgStacker
    from utils.reward_shaping.env_utils import Transformer

    class Env:
        def __init__(self):
            self.k = 0
            self.observation_space = sys.modules['gym'].spaces.Box(0.0, 1.0, (1, 2, 2))

        def reset(self):
            self.k = 100
            return np.full((1, 2, 2), self.k, np.float64)

    # ImgStacker: newest first, reset pre-fills copies
    env = Env()
    st = ImgStacker(env)
    seq = []
    o = st.observation(env.reset())
    seq.append(o[:, 0, 0].tolist())
    for k in range(1, 6):
        o = st.observation(np.full((1, 2, 2), k, np.float64))
        seq.append(o[:, 0, 0].tolist())
    st.reset()
    o = st.observation(np.full((1, 2, 2), 200, np.float64))
    seq.append(o[:, 0, 0].tolist())
    # Transformer: oldest first; reset fills three copies, then the wrapper's
    # reset() calls transform once more (utils/env_wrappers.py:198-201)
    tr = Transformer()
    tseq = []
    first = np.full((1, 2, 2), 100, np.float64)
    tr.reset(first)
    tseq.append(tr.transform(first)[:, 0, 0].tolist())
    for k in range(1, 6):
        tseq.append(tr.transform(np.full((1, 2, 2), k, np.float64))[:, 0, 0].tolist())
    dump('stacking.json', {'img_stacker': seq, 'transformer': tseq})


def gen_env_wrapper():
    """Drive the reference's EnvironmentWrapper over the oracle SimulatorRef."""
    import utils.env_wrappers as ew
    sys.path.insert(0, REPO)
    from oracle import dtsim_ref as R
    with open(os.path.join(REF, 'config.json')) as f:
        config = json.load(f)
    rows = [['curve_left/W', 'straight/W', 'curve_left/N'],
            ['straight/S', 'grass', 'straight/N'],
            ['curve_left/S', 'straight/E', 'curve_left/E']]
    fixtures = []
    for mode, seed in (('tanh', 11), ('wheels', 12)):
        head = config['model']['actor'][-1]['modules'][-1][-1]
        head['name'] = 'tanh' if mode == 'tanh' else 'sigmoid'
        log = {'raw': []}

        class OracleDT(ew.BaseEnvironment):
            def __init__(self):
                self.sim = R.SimulatorRef(rows, seed=seed, env_id=0,
                                          cfg=R.SimConfig(max_env_steps=40))
                self.obs = [[[0.0, 0.0], [0.0, 0.0]]]  # from_numpy'd, as the reference's env returns

            def step(self, action):
                _, r, d, info = self.sim.step(np.array(action, np.float64))
                log['raw'].append([float(r), bool(d)])
                return [self.obs, r, d, None]

            def reset(self):
                self.sim.reset()
                return self.obs

            def get_observation(self):
                return self.obs

            def change_model(self, seed):
                return 'ok'

            def collect_garbage(self):
                pass

        ew.DuckietownEnvironmentWrapper = lambda **kw: OracleDT()
        cfg = json.loads(json.dumps(config))
        cfg['environment']['wrapper']['max_env_steps'] = 40
        env = ew.EnvironmentWrapper(cfg, {'env_type': 'normal', 'env_init_args': {},
                                          'env_config': {'seed': seed}}, transfer=False)
        rng = np.random.default_rng(seed)
        steps = []
        env.reset()
        for t in range(120):
            if mode == 'tanh':
                a = rng.uniform(-1, 1, 2).astype(np.float32)
            else:
                a = rng.uniform(0, 1, 2).astype(np.float32)
            a_in = a.copy()
            log['raw'] = []
            _, (r, rm), done, _ = env.step(a)
            steps.append({'action_in': [float(v) for v in a_in],
                          'action_after': [float(v) for v in a],
                          'raw': log['raw'], 'reward': float(r), 'reward_mod': float(rm),
                          'done': bool(done), 'env_step': env.env_step})
            if done:
                env.reset()
        fixtures.append({'mode': mode, 'seed': seed, 'max_env_steps': 40, 'steps': steps})
    dump('env_wrapper.json', fixtures)


def gen_segment_tree():
    from utils.segment_tree import MinSegmentTree, SumSegmentTree
    rng = np.random.default_rng(7)
    out = []
    for cap in (1, 2, 16, 64):
        s, m = SumSegmentTree(cap), MinSegmentTree(cap)
        ops = []
        for _ in range(200):
            i = int(rng.integers(0, cap))
            v = float(rng.random() ** 2)
            s[i] = v
            m[i] = v
            a = int(rng.integers(0, cap))
            b = int(rng.integers(a + 1, cap + 1))
            total = s.sum()
            p = float(rng.random()) * total
            ops.append({'set': [i, v], 'range': [a, b], 'sum': s.sum(a, b), 'min': m.min(a, b),
                        'total': total, 'prefix': p, 'idx': s.find_prefixsum_idx(p)})
        out.append({'capacity': cap, 'ops': ops})
    dump('segment_tree.json', out)


def gen_prioritized_replay():
    """Drive utils/buffers.py PrioritizedReplayBuffer through adds (with wrap),
    proportional samples and priority updates (with duplicate indices).  The
    uniforms random.random() returns are scripted and recorded, so a GPU run fed
    the same uniforms must return the same indices."""
    import utils.buffers as buffers
    rng = np.random.default_rng(11)
    out = []
    for size, alpha, beta in ((100, 0.6, 0.4), (37, 0.5, 1.0), (16, 0.6, 0.4)):
        buf = buffers.PrioritizedReplayBuffer(size, alpha)
        cap = buf._it_sum._capacity
        ops = []
        counter = 0
        for step in range(12):
            n_add = int(rng.integers(1, 2 * size // 3 + 2))
            items = list(range(counter, counter + n_add))
            counter += n_add
            for k in items:
                # ndarray items: numpy 2's np.array(x, copy=False) refuses to copy
                buf.add(np.array([k]), np.array([k, -k]), float(k), np.array([k + 1]), k % 5 == 0)
            op = {'add': items}
            if len(buf) >= 2:
                batch = int(rng.integers(1, 33))
                us = [float(u) for u in rng.random(batch)]
                it = iter(us)
                saved = buffers.random.random
                buffers.random.random = lambda: next(it)
                try:
                    obs, act, rew, nxt, done, w, idx = buf.sample(batch, beta=beta)
                finally:
                    buffers.random.random = saved
                op['sample'] = {'batch': batch, 'beta': beta, 'u': us, 'idx': [int(i) for i in idx],
                                'weights': [float(x) for x in w], 'obs': [int(o) for o in obs.reshape(-1)]}
                n_up = int(rng.integers(1, batch + 1))
                up_idx = [int(idx[int(j)]) for j in rng.integers(0, batch, n_up)]
                pr = [float(x) for x in rng.random(n_up) * 3 + 1e-3]
                buf.update_priorities(up_idx, pr)
                op['update'] = {'idx': up_idx, 'priorities': pr}
            op['len'] = len(buf)
            op['next_idx'] = buf._next_idx
            op['max_priority'] = buf._max_priority
            op['sum_tree'] = [float(v) for v in buf._it_sum._value]
            op['min_tree'] = [float(v) if v != float('inf') else None for v in buf._it_min._value]
            ops.append(op)
        out.append({'size': size, 'alpha': alpha, 'capacity': cap, 'ops': ops})
    dump('prioritized_replay.json', out)


def gen_random_process_and_decay():
    from utils.random_process import OrnsteinUhlenbeckProcess
    from utils.util import create_decay_fn
    np.random.seed(42)
    ou = OrnsteinUhlenbeckProcess(size=2, theta=0.15, mu=0.0, sigma=0.3, sigma_min=0.15)
    # record the normals too: the reference draws them from numpy's global RNG
    np.random.seed(42)
    normals = np.random.normal(size=(300, 2)).tolist()
    np.random.seed(42)
    samples = [ou.sample().tolist() for _ in range(300)]
    ou.reset_states()
    decays = {}
    steps = [0, 1, 7, 31, 32, 33, 100, 1000, 23999, 24000]
    decays['cycle'] = [create_decay_fn('cycle', initial_value=0.5, final_value=0.025,
                                       cycle_len=32, num_cycles=24000 // 32)(s) for s in steps]
    decays['linear'] = [create_decay_fn('linear', initial_value=0.002, final_value=1e-5,
                                        max_step=4000000)(s) for s in steps]
    decays['exponential'] = [create_decay_fn('exponential', initial_value=1.0,
                                             final_value=0.01, max_step=1000,
                                             updates=10)(s) for s in steps]
    decays['cyclic_cosine'] = [create_decay_fn('cyclic_cosine', initial_value=1.0,
                                               final_value=0.1, period_base=10,
                                               period_modifier=2)(s) for s in steps]
    dump('random_process.json', {'normals': normals, 'ou': samples, 'decay_steps': steps,
                                 'decay': decays})


def gen_actor():
    import torch
    from duckietown_rl.ddpg import ActorCNN
    from models.ddpg.modules import Actor
    sys.path.insert(0, HERE)
    from formulas import formula_input, formula_state_dict
    with open(os.path.join(REF, 'config.json')) as f:
        config = json.load(f)
    x = formula_input(4)
    out = {}
    a = ActorCNN(2, 1.0)
    a.load_state_dict(formula_state_dict(a.state_dict()))
    a.eval()
    with torch.no_grad():
        out['actor_cnn'] = a(x).numpy()
    c = Actor(config['model']['actor'])
    c.load_state_dict(formula_state_dict(c.state_dict()))
    c.eval()
    with torch.no_grad():
        out['config_actor'] = c(x).numpy()
    out['config_actor_keys'] = np.array(list(c.state_dict().keys()))
    from models.ddpg.modules import Critic
    from formulas import hash_u
    cr = Critic(config['model']['critic'])
    cr.load_state_dict(formula_state_dict(cr.state_dict()))
    cr.eval()
    act = hash_u(8, 77).reshape(4, 2).float()
    with torch.no_grad():
        out['config_critic'] = cr(x, act).numpy()
    out['config_critic_keys'] = np.array(list(cr.state_dict().keys()))
    out['actor_cnn_keys'] = np.array(list(a.state_dict().keys()))
    np.savez_compressed(os.path.join(HERE, 'actor.npz'), **out)
    print('wrote actor.npz')


def no_dropout(net_config):
    for part in net_config:
        for branch in part.get('modules', []):
            for m in branch:
                if m['name'] == 'dropout':
                    m['args']['p'] = 0.0
    return net_config


def gen_ddpg_update(double=False):
    """training/trainers.py DDPGTrainer.update, run as the reference runs it
    (models in train mode: BatchNorm on batch statistics), three updates on a
    formula batch.  Dropout p is set to 0 so the run is deterministic.
    double=True: the same in float64 (models .double(), the module-level
    to_torch_tensor helper producing float64) — float32 runs of this update
    drift apart after the first Adam step (near-zero bias gradients get full
    +-lr steps), float64 pins all three updates tightly."""
    import copy
    import threading
    from types import SimpleNamespace

    import torch
    from models.ddpg.model import create_model
    from training.trainers import DDPGTrainer
    from utils.util import TrainingDecay
    sys.path.insert(0, HERE)
    from formulas import formula_batch, formula_state_dict, param_summary
    with open(os.path.join(REF, 'config.json')) as f:
        cfg = json.load(f)
    no_dropout(cfg['model']['actor'])
    no_dropout(cfg['model']['critic'])
    torch.manual_seed(0)
    target = create_model(cfg['model'])
    target.actor.load_state_dict(formula_state_dict(target.actor.state_dict()))
    target.critic.load_state_dict(formula_state_dict(target.critic.state_dict()))
    target.train()
    if double:
        import training.trainers as trainers_mod
        target.actor.double()
        target.critic.double()
        trainers_mod.to_torch_tensor = lambda a, cpu=False: torch.from_numpy(
            np.asarray(a, np.float64))
    model = copy.deepcopy(target)            # managers.py:82
    tr = DDPGTrainer(cfg, 0, target, copy.deepcopy(target), [model], None, None,
                     threading.Lock(), None, None, SimpleNamespace(value=0),
                     SimpleNamespace(value=0))
    tr.target_actor, tr.target_critic = target.get_actor(), target.get_critic()
    tr.actor, tr.critic = model.get_actor(), model.get_critic()
    tr.actor_optim = torch.optim.Adam(tr.actor.parameters(), lr=0.)
    tr.critic_optim = torch.optim.Adam(tr.critic.parameters(), lr=0.)
    tr.actor_decay = TrainingDecay(cfg['training']['actor_train_decay'])
    tr.critic_decay = TrainingDecay(cfg['training']['critic_train_decay'])
    batch = formula_batch(16)
    out = {'critic_loss': [], 'actor_loss': [], 'td_error': []}
    for _ in range(3):
        metrics, info = tr.update(batch)
        out['critic_loss'].append(float(metrics['critic_loss']))
        out['actor_loss'].append(float(metrics['actor_loss']))
        out['td_error'].append([float(x) for x in info['td_error'].reshape(-1)])
    for name, net in (('actor', tr.actor), ('critic', tr.critic), ('target_actor', tr.target_actor),
                      ('target_critic', tr.target_critic)):
        out[name] = param_summary(net)
    dump('ddpg_update_f64.json' if double else 'ddpg_update.json', out)


def gen_ddpg_single(double=False):
    """duckietown_rl/ddpg.py DDPG.train over duckietown_rl/utils.py ReplayBuffer:
    20 formula transitions added to a max_size-12 buffer (8 random-eviction
    pops), then three train iterations of batch 8, one call each so the
    parameters are summarised after every iteration.  Seeds: random 7, numpy 11.
    Dropout p=0 (deterministic).  double=True: the module's FloatTensor makes
    float64 and the nets are .double() (float32 drifts after the first Adam step,
    as for gen_ddpg_update)."""
    import torch
    import duckietown_rl.ddpg as dd
    from duckietown_rl.utils import ReplayBuffer
    sys.path.insert(0, HERE)
    from formulas import formula_batch, formula_state_dict, param_summary
    if double:
        shim = types.SimpleNamespace(**{k: getattr(torch, k) for k in dir(torch)
                                        if not k.startswith('__')})
        shim.FloatTensor = lambda a: torch.from_numpy(np.asarray(a, np.float64))
        dd.torch = shim
    try:
        torch.manual_seed(0)
        agent = dd.DDPG(None, 2, 1.0, 'cnn')
        for net, tgt in ((agent.actor, agent.actor_target), (agent.critic, agent.critic_target)):
            sd = formula_state_dict(net.state_dict())
            net.load_state_dict(sd)
            tgt.load_state_dict(sd)
        for net in (agent.actor, agent.actor_target):
            net.dropout.p = 0.0
        if double:
            for net in (agent.actor, agent.actor_target, agent.critic, agent.critic_target):
                net.double()
            agent.actor_optimizer = torch.optim.Adam(agent.actor.parameters(), lr=1e-4)
            agent.critic_optimizer = torch.optim.Adam(agent.critic.parameters())
        obs, act, rew, nxt, done = formula_batch(20)
        dt = np.float64 if double else np.float32
        random.seed(7)
        np.random.seed(11)
        rb = ReplayBuffer(12)
        for i in range(20):
            # 0-d arrays: the reference's np.array(x, copy=False) refuses Python
            # floats under numpy 2 (same values as the training script's floats)
            rb.add(obs[i].astype(dt), nxt[i].astype(dt), act[i].astype(dt),
                   np.asarray(float(rew[i]), dt), np.asarray(float(done[i]), dt))
        order = [int(np.argmin(np.abs(rew - s[3]))) for s in rb.storage]
        out = {'storage_order': order, 'iterations': []}
        for _ in range(3):
            agent.train(rb, 1, batch_size=8)
            out['iterations'].append({name: param_summary(net) for name, net in (
                ('actor', agent.actor), ('critic', agent.critic),
                ('actor_target', agent.actor_target), ('critic_target', agent.critic_target))})
        out['numpy_after'] = int(np.random.randint(0, 1 << 30))
        out['random_after'] = random.randrange(1 << 30)
    finally:
        dd.torch = torch
    dump('ddpg_single_f64.json' if double else 'ddpg_single.json', out)


def gen_explorer():
    """SingleThreadExplorer._explore_episode (training/explorers.py:164-213), the
    reference's own loop, over the oracle SimulatorRef (the reference's own
    EnvironmentWrapper around it, as gen_env_wrapper): records every random
    draw in the loop's order -- the OU normals (utils/random_process.py:42-47),
    the every-second-random coin (random.uniform) and random action
    (np.random.random) -- the actor output DDPG.act saw (a stub actor: the
    network itself is pinned by gen_actor), the action handed to env.step and
    the replay tuple's action after the wrapper's in-place map, reward (the
    reward_modified choice) and done.  Explorers: exploring p_id 0 (even: every
    second random) and 1, and the exploiting_virtual explorer (epsilon 0, no
    noise; explorers.py:104-116, 182-184)."""
    import torch

    import training.explorers as tx
    import utils.env_wrappers as ew
    import utils.random_process as rp
    from utils.util import create_decay_fn
    sys.path.insert(0, REPO)
    from oracle import dtsim_ref as R
    with open(os.path.join(REF, 'config.json')) as f:
        config = json.load(f)
    rows = [['curve_left/W', 'straight/W', 'curve_left/N'],
            ['straight/S', 'grass', 'straight/N'],
            ['curve_left/S', 'straight/E', 'curve_left/E']]
    log = {}

    class RandProxy:       # numpy.random / random with the loop's draws recorded
        def __init__(self, real):
            self.real = real

        def normal(self, *a, **k):
            v = self.real.normal(*a, **k)
            log['normals'].append([float(x) for x in np.atleast_1d(v)])
            return v

        def random(self, *a, **k):
            v = self.real.random(*a, **k)
            log['randoms'].append([float(x) for x in np.atleast_1d(v)])
            return v

        def uniform(self, *a, **k):
            v = self.real.uniform(*a, **k)
            log['coins'].append(float(v))
            return v

        def __getattr__(self, k):
            return getattr(self.real, k)

    class NpProxy:
        random = RandProxy(np.random)

        def __getattr__(self, k):
            return getattr(np, k)
    rp.np = NpProxy()
    tx.np = NpProxy()
    tx.random = RandProxy(random)

    class StubActor(torch.nn.Module):
        """A deterministic function of the observation (the stacked frame
        markers below), so consecutive decisions see different outputs."""
        def forward(self, x):
            m = x.double().mean()
            out = torch.stack([torch.tanh(3.0 * torch.sin(7.0 * m) - 0.2),
                               torch.tanh(2.0 * torch.cos(5.0 * m) + 0.1)]).float().view(1, 2)
            log['actor_out'].append([float(v) for v in out.view(-1)])
            return out

    class OracleDT(ew.BaseEnvironment):
        def __init__(self, seed):
            self.sim = R.SimulatorRef(rows, seed=seed, env_id=0, cfg=R.SimConfig(max_env_steps=60))

        def _obs(self):
            # a 1 x 2 x 2 marker of the pose (from_numpy'd, as the reference's env returns)
            x, z = float(self.sim.cur_pos[0]), float(self.sim.cur_pos[2])
            return [[[x, z], [float(self.sim.cur_angle), 0.25]]]

        def step(self, action):
            _, r, d, info = self.sim.step(np.array(action, np.float64))
            return [self._obs(), r, d, None]

        def reset(self):
            self.sim.reset()
            return self._obs()

        def get_observation(self):
            return self._obs()

        def change_model(self, seed):
            return 'ok'

        def collect_garbage(self):
            pass

    out = []
    t = config['training']
    cycle_len = 20
    decay = create_decay_fn('cycle', initial_value=t['initial_epsilon'],
                            final_value=t['final_epsilon'], cycle_len=cycle_len,
                            num_cycles=t['max_episodes'] // cycle_len)
    for kind, p_id in (('exploration_virtual', 0), ('exploration_virtual', 1),
                       ('exploiting_virtual', 7)):
        cfg = json.loads(json.dumps(config))
        cfg['environment']['wrapper']['max_env_steps'] = 60
        seed_box = {}
        ew.DuckietownEnvironmentWrapper = lambda **kw: OracleDT(seed_box['seed'])
        seed_box['seed'] = 31 + p_id
        model = tx.create_model(cfg['model'])
        model.actor = StubActor()
        explorer = tx.SingleThreadExplorer(kind, cfg, p_id, model,
                                           {'env_type': 'normal', 'env_init_args': {},
                                            'env_config': {}}, [], None, None, None)
        if kind.startswith('exploiting'):
            explorer.model.actor = StubActor()
        orig_step = explorer.environment.step

        def step(action, orig_step=orig_step):
            log['action'].append([float(v) for v in action])   # before the in-place map
            return orig_step(action)
        explorer.environment.step = step
        ou = rp.create_action_random_process(cfg)
        episodes = []
        for e in range(3):
            # episode counters that are multiples of the cycle: cos(0) = 1 exactly
            ep = e * cycle_len
            eps = min(t['initial_epsilon'], max(t['final_epsilon'], decay(ep)))
            if kind.startswith('exploiting'):
                eps = 0.0
            for k in ('normals', 'randoms', 'coins', 'actor_out', 'action'):
                log[k] = []
            metrics = {'reward': 0.0, 'reward_modified': 0.0, 'step': 0, 'epsilon': eps}
            ou.reset_states()
            replay, _ = explorer._explore_episode(ou, eps, metrics, t)
            # per decision: which draws happened (the coin only for even
            # exploring ids, the random action only when the coin came up)
            steps, ci, ri, ai = [], 0, 0, 0
            for d, (obs, act, rew, nxt, done) in enumerate(replay):
                rec = {'normals': log['normals'][d], 'action': log['action'][d],
                       'replay_action': [float(v) for v in act], 'reward': float(rew),
                       'done': bool(done)}
                if kind.startswith('exploration') and t['every_second_random'] and p_id % 2 == 0:
                    rec['coin'] = log['coins'][ci]
                    ci += 1
                    if rec['coin'] < t['epsilon_ratio'] * eps:
                        rec['random'] = log['randoms'][ri]
                        ri += 1
                        steps.append(rec)
                        continue
                rec['actor_out'] = log['actor_out'][ai]
                ai += 1
                steps.append(rec)
            assert ci == len(log['coins']) and ri == len(log['randoms'])
            assert ai == len(log['actor_out'])
            episodes.append({'episode_counter': ep, 'epsilon': eps, 'ou_steps_before':
                             float(ou.n_steps) - len(steps), 'steps': steps})
        out.append({'exploration_type': kind, 'p_id': p_id, 'cycle_len': cycle_len,
                    'episodes': episodes})
    dump('explorer.json', {'numpy': np.__version__, 'explorers': out})


def gen_config_keys():
    """The config.json keys the env path reads (wrapper section, actor head, the
    explorer's noise/epsilon keys) — a data extract, not the file."""
    with open(os.path.join(REF, 'config.json')) as f:
        cfg = json.load(f)
    head = cfg['model']['actor'][-1]['modules'][-1][-1]['name']
    keys = ('global_seed', 'rp_theta', 'rp_mu', 'rp_sigma', 'rp_sigma_min', 'epsilon_cycle_len',
            'initial_epsilon', 'final_epsilon', 'epsilon_ratio', 'max_episodes',
            'every_second_random', 'alpha', 'beta', 'batch_size', 'buffer_size', 'gamma', 'tau',
            'optimizer', 'critic_loss', 'actor_train_decay', 'critic_train_decay',
            'num_threads_training', 'update_steps_between_update', 'num_threads_exploring',
            'num_threads_exploring_virtual', 'num_threads_exploiting',
            'num_threads_exploiting_virtual')
    mini = {'environment': {'wrapper': cfg['environment']['wrapper']},
            'model': {'num_action': cfg['model']['num_action'], 'actor': cfg['model']['actor'],
                      'critic': cfg['model']['critic']},
            'training': {k: cfg['training'][k] for k in keys}}
    assert mini['model']['actor'][-1]['modules'][-1][-1]['name'] == head
    for path in (os.path.join(HERE, 'reference_config.json'),
                 os.path.join(REPO, 'aido1_amd', 'configs', 'reference_config.json')):
        if os.path.exists(path):
            os.chmod(path, 0o644)
        with open(path, 'w') as f:
            json.dump(mini, f, indent=1)
        os.chmod(path, 0o444)
    print('wrote reference_config.json')


def main():
    sys.path.insert(0, REF)
    only = os.environ.get('ONLY')   # e.g. ONLY=gen_explorer: regenerate one fixture
    if only:
        install_stubs()
        globals()[only]()
        return
    gen_config_keys()
    install_stubs()
    gen_bresenham()
    gen_aggregation()
    gen_steering()
    gen_stacking()
    gen_env_wrapper()
    gen_segment_tree()
    gen_prioritized_replay()
    gen_random_process_and_decay()
    gen_actor()
    gen_ddpg_update()
    gen_ddpg_update(double=True)
    gen_ddpg_single()
    gen_ddpg_single(double=True)
    gen_explorer()


if __name__ == '__main__':
    main()
