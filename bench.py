#!/usr/bin/env python
"""bench.py — BASELINE.json's metric: env-steps/s (whole node) at 4096 envs/GPU,
with pose/reward max-abs-err vs the CPU oracle in the same line.

Headline workload (default, --config render): BASELINE.json configs[2], the
largest single-GPU configuration: 4096 envs per GPU on loop_empty, i.i.d.
U[0,1)^2 wheel actions (the train.py contract after utils/env_wrappers.py:214-216)
resident in HBM, Philox spawn streams keyed by seed 1234, auto-reset on done or
at the 2000-step wrapper cap, and per decision the full observation path: the
120x160 top-down raster + grey frame into the 3-slot Transformer ring (the
ring refilled for respawned envs) + the features/line_detector1 masks.  One
bench "step" = one decision = one EnvironmentWrapper.step for every env = up to
repeat_actions (3) Simulator steps each, plus the render of the pose it ends
in; the unit counted is the Simulator step (env-step), read back exactly from
the device counters.

Timed region (default --obs-mode many): the actions are i.i.d. and resident,
so the K decisions are stepped in chunks of up to --many (20) decisions, one
dt_step_many launch a chunk writing every decision's end pose, then the
chunk's renders --render-group (3) consecutive decisions a launch (dt_render3,
a trailing pair by dt_render2), each decision rendered from its own pose with
its own done flags, its frame into the ring and its masks into its own buffer;
one stream, every foreign call bound before the region (ObsLoop).  The other
modes ('serial', 'pipe': dt_step + dt_copy_pose + dt_render of the snapshot
on a second stream, the form an actor-in-the-loop consumer uses; 'many2')
compute the same outputs.  After it, outside the timed region:
  * parity: the C oracle (oracle/dtsim_oracle.c, test infrastructure) re-runs
    every env of this rank from the saved start state through the same actions;
    reward/reward_mod/obs/done of every decision and the end pose/counters are
    compared with the timed launches' outputs, and a second GPU pass (dt_step,
    tile index asked for) checks tile indices; 256 envs' masks of EVERY timed
    decision and their final frame stacks (the last three decisions' frames,
    as the ring holds them) are compared bit for bit with
    oracle/render_oracle.c renders of the oracle's poses (a process pool on
    the host);
  * roofline: render_kernel's algorithmic bytes (grey + masks + pose, plus the
    ring refill of respawned envs) / its mean duration from HIP events on the
    render stream;
  * config2: BASELINE configs[1] (lane-pose obs only, dt_step_many launches) as
    a sub-record with its own parity and roofline.

Other configs: --config lane (configs[1] as the headline), actor = configs[3]
(actor in the loop), train = configs[4] (full DDPG: rollout + GPU prioritized
replay + update + RCCL gradient all-reduce).

N > 1: `python bench.py --gpus N` starts torch.distributed.run with N ranks as
a child process BEFORE anything touches the GPU (the driver may also launch
torch.distributed.run itself; WORLD_SIZE must then equal --gpus).  One rank per
GPU over RCCL; envs shard by env_id_base = rank * envs (disjoint spawn
streams), no data-path collective; timing = barrier + synchronize on both
sides, max over ranks; value = all ranks' env-steps / that time.  Rank 0 prints
one JSON line with every rank's counts.  `--dry-run` runs the same launcher and
reduction on CPU over gloo with no kernels (tests/test_bench_launcher.py).
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = 'env-steps/sec (whole node) at 4096 envs/GPU; pose/reward max-abs-err vs CPU ref'
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec
FP64_VECTOR_PEAK_TFLOPS = 78.6   # MI355X spec: fp64 vector = 1/2 of fp32 vector 157.3 TF
BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16/fp16 MFMA (spec)
F32_MFMA_PEAK_TFLOPS = 157.3     # MI355X spec: f32 matrix (MFMA) dense
# the float32-accurate actor (include/dtactor.h dt_conv1x_split): three fp16
# MFMA products per f32 product, so its arithmetic ceiling is the fp16 peak / 3
X3_PEAK_TFLOPS = BF16_DENSE_PEAK_TFLOPS / 3.0

# algorithmic HBM bytes per env-step of config 2 = action 8 +
# state read 28 + state write 28 + reward 4 + done 1 + dist/angle 8 + tile 4.
SURVEY_BYTES_PER_ENV_STEP = 81
# What one dt_step_many launch of k decisions really has to move (DESIGN.md
# §3.1; state stays in registers across the k decisions):
# per env, once: reads pose 24 + step_count,env_step 8 + episode,tick 8 + seed 8
#                + the 8 slot words 64 = 112; writes pose 24 + counters 8 + tick 4 = 36
#   refill scan: want 4 + tick 4 + slot words 64 + seed 8 = 80
# per env and decision: action 8 + reward 8 + reward_mod 8 + done 1 + obs 8 = 33
# per reset: the slot's 56-B record read, episode + want 8, refilled record 56 + word 8 = 128
MANY_BYTES_PER_ENV = 112 + 36 + 80
MANY_BYTES_PER_ENV_DECISION = 33
MANY_BYTES_PER_RESET = 128


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=100)
    p.add_argument('--warmup', type=int, default=30)
    p.add_argument('--envs', type=int, default=4096)
    p.add_argument('--map', default='loop_empty')
    p.add_argument('--config', default='render', choices=['render', 'lane', 'actor', 'train'])
    p.add_argument('--actor-mode', default='reference', choices=['reference', 'eval'],
                   help="actor/train: 'reference' = train-mode batch-of-one BatchNorm + live "
                        "dropout as the reference's explorers act; 'eval' = BN folded")
    p.add_argument('--actor-dtype', default='float32', choices=['float16', 'float32'],
                   help='actor/train: the acting actor\'s arithmetic (float32 = the '
                        'reference\'s precision, the x3 chain; float16 = the fast mode)')
    p.add_argument('--frames', default='index', choices=['index', 'gray'],
                   help="actor/train: the frame ring's format: 'index' = palette-index u8 frames "
                        "(lossless, a quarter of the bytes; render.py), 'gray' = float32 grey")
    p.add_argument('--batch-size', type=int, default=0, help='train: 0 = config.json (64)')
    p.add_argument('--buffer-size', type=int, default=131072)
    p.add_argument('--updates-per-step', type=int, default=1)
    p.add_argument('--overlap', action='store_true',
                   help='train: run each update beside the next rollout (side stream); a '
                        'different schedule (acting one update behind), DESIGN 3.8')
    p.add_argument('--render-group', type=int, default=3,
                   help='config 3 many modes: consecutive decisions a render launch '
                        '(1 dt_render, 2 dt_render2, 3 dt_render3: the ring\'s slots)')
    p.add_argument('--no-pair', action='store_true', help='= --render-group 1')
    p.add_argument('--many', type=int, default=20,
                   help='most decisions per dt_step_many launch (lane config, and the render '
                        'config\'s many mode); K decisions are split into ceil(K / many) '
                        'equal launches')
    p.add_argument('--graph', action='store_true',
                   help='lane config: replay the timed launches as one captured HIP graph '
                        '(default: prebound eager dt_step_many calls)')
    p.add_argument('--no-parity', action='store_true', help='skip the oracle parity pass')
    p.add_argument('--obs-mode', default='many', choices=['many', 'many2', 'serial', 'pipe'],
                   help='render: how the steps are launched (ObsLoop)')
    p.add_argument('--no-lane', action='store_true', help='render: skip the config-2 sub-record')
    p.add_argument('--no-sub', action='store_true',
                   help='render: skip the config-4 / config-5 sub-records')
    p.add_argument('--f64-envs', type=int, default=1024,
                   help='configs 4 / 5: envs whose actions are checked against the float64 '
                        'actor (actor_f64 on the GPU)')
    p.add_argument('--sub-steps', type=int, default=20,
                   help='timed decisions of the config-4 / config-5 sub-records')
    p.add_argument('--sub-warmup', type=int, default=5)
    p.add_argument('--event-stride', type=int, default=4,
                   help='render: HIP events around every S-th dt_render of the timed region '
                        '(the roofline\'s average kernel duration is over those launches); '
                        'an event pair around every launch adds ~6 us a decision of stream '
                        'packets to the wall time (measured: 0.1805 vs 0.1745 ms per step)')
    p.add_argument('--roofline-launches', type=int, default=60,
                   help='render: dt_render launches of the event-only pass after the timed '
                        'region that the roofline averages (at least --steps)')
    p.add_argument('--lane-steps', type=int, default=320,
                   help='render: decisions timed by the config-2 sub-record')
    p.add_argument('--lane-warmup', type=int, default=20)
    p.add_argument('--seed', type=int, default=1234)
    p.add_argument('--cpu-steps', type=int, default=30000,
                   help='config-2 CPU baseline: timed env-steps per process after 1000 warm-up '
                        'steps (BASELINE.md §3); 0 = skip every CPU baseline')
    p.add_argument('--cpu-decisions', type=int, default=1000,
                   help='config-3 CPU baseline: timed decisions (step + render) per process')
    p.add_argument('--cpu-actor-decisions', type=int, default=3000,
                   help='configs 4 / 5 CPU baselines: timed decisions per explorer process')
    p.add_argument('--cpu-updates', type=int, default=10,
                   help='config-5 CPU baseline: timed updates of the trainer process')
    p.add_argument('--cpu-procs', type=int, default=0,
                   help='CPU baseline processes (0 = the box CPU share: min(16, affinity))')
    p.add_argument('--dry-run', action='store_true',
                   help='launcher/reduction check on CPU over gloo, no kernels')
    return p.parse_args(argv)


# ---- N-rank launcher ---------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args, argv):
    """Start N ranks with torch.distributed.run as a child process and return its
    exit code.  Runs before torch is imported here, so no GPU is touched by the
    parent (it must never exec after HIP initialisation)."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(args.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return subprocess.call(cmd, env=env)


# ---- CPU baselines, one env per process ------------------------
def _map_rows(map_name):
    import yaml
    with open(os.path.join(REPO, 'aido1_amd', 'maps', map_name + '.yaml')) as f:
        return yaml.safe_load(f)['tiles']


def _cpu_worker(args):
    """configs[1]: the numpy restatement of Simulator.step + EnvironmentWrapper.step."""
    idx, warm, steps_wanted, map_name = args
    from oracle import dtsim_ref as R
    env = R.EnvironmentWrapperRef(R.SimulatorRef(_map_rows(map_name), seed=1234, env_id=idx))
    env.reset()
    rng = np.random.default_rng(1234 + idx)

    def run(target):
        steps = 0
        while steps < target:
            a = rng.random(2, dtype=np.float32)
            before = env.sim.step_count
            _, _, d = env.step(a)
            steps += env.sim.step_count - before
            if d:
                env.reset()
        return steps
    run(warm)
    t0 = time.perf_counter()
    steps = run(steps_wanted)
    return steps, time.perf_counter() - t0


def _cpu_obs_worker(args):
    """configs[2]: per decision the numpy step restatement, then the C restatement
    of the raster + grey + LineDetectorHSV filter (oracle/render_oracle.c) of
    the pose it ends in, pushed into a 3-frame stack (Transformer; a respawn
    refills the stack, utils/reward_shaping/env_utils.py:54-70)."""
    idx, warm, decisions, map_name = args
    from oracle import dtsim_ref as R
    from oracle import oracle_c as OC
    rows = _map_rows(map_name)
    env = R.EnvironmentWrapperRef(R.SimulatorRef(rows, seed=1234, env_id=idx))
    rend = OC.OracleRender(rows)
    env.reset()
    rng = np.random.default_rng(1234 + idx)
    stack = np.zeros((3, 120, 160), np.float32)

    def run(k):
        steps = 0
        for _ in range(k):
            a = rng.random(2, dtype=np.float32)
            before = env.sim.step_count
            _, _, d = env.step(a)
            steps += env.sim.step_count - before
            if d:
                env.reset()
            p = env.sim.cur_pos
            g, m, _ = rend.render((p[0],), (p[2],), (env.sim.cur_angle,))
            if d:
                stack[:] = g[0]
            else:
                stack[:2] = stack[1:]
                stack[2] = g[0]
        return steps
    run(warm)
    t0 = time.perf_counter()
    steps = run(decisions)
    return steps, time.perf_counter() - t0


def _reference_config():
    with open(os.path.join(REPO, 'aido1_amd', 'configs', 'reference_config.json')) as f:
        return json.load(f)


def _cpu_actor_worker(args):
    """configs[3] / [4] on the host, the reference's way: one explorer per
    process acting on ONE observation at a time (training/explorers.py:164-211,
    models/ddpg/model.py:74-102: a batch-of-one float32 forward of the
    train-mode ConfigActor on torch's CPU, one thread), OU noise, the numpy
    step restatement x repeat 3 with the tanh head's mapping, the C render +
    line filter and the 3-frame stack.  role 'train': a DDPG trainer process
    instead (training/trainers.py:143-237 on torch's CPU, batch 64, one
    thread), `decisions` updates on synthetic batches."""
    idx, warm, decisions, map_name, role = args
    import torch
    torch.set_num_threads(1)
    from aido1_amd.actor import ConfigActor, ConfigCritic
    cfg = _reference_config()
    torch.manual_seed(idx)
    if role == 'train':
        from aido1_amd.trainer import DDPGTrainer
        tr = DDPGTrainer(cfg, ConfigActor(cfg['model']['actor']),
                         ConfigCritic(cfg['model']['critic']), device='cpu')
        b = int(cfg['training']['batch_size'])
        g = torch.Generator().manual_seed(idx)
        batch = (torch.rand(b, 3, 120, 160, generator=g), torch.rand(b, 2, generator=g),
                 torch.randn(b, generator=g).double(), torch.rand(b, 3, 120, 160, generator=g),
                 (torch.rand(b, generator=g) < 0.05))
        tr.update(batch)
        t0 = time.perf_counter()
        for _ in range(decisions):
            tr.update(batch)
        return 0, time.perf_counter() - t0, decisions
    from oracle import dtsim_ref as R
    from oracle import oracle_c as OC
    rows = _map_rows(map_name)
    env = R.EnvironmentWrapperRef(R.SimulatorRef(rows, seed=1234, env_id=idx,
                                                 cfg=R.SimConfig(action_mode='tanh')))
    rend = OC.OracleRender(rows)
    actor = ConfigActor(cfg['model']['actor'])
    actor.train()                           # the explorers' models are in train mode
    t = cfg['training']
    rng = np.random.default_rng(1234 + idx)
    ou = np.zeros(2)
    stack = np.zeros((3, 120, 160), np.float32)

    def frame(fresh):
        p = env.sim.cur_pos
        g, _, _ = rend.render((p[0],), (p[2],), (env.sim.cur_angle,))
        if fresh:
            stack[:] = g[0]
        else:
            stack[:2] = stack[1:]
            stack[2] = g[0]

    env.reset()
    frame(True)

    def run(k):
        nonlocal ou
        steps = 0
        for _ in range(k):
            with torch.no_grad():
                a = actor(torch.from_numpy(stack[None])).numpy()[0]
            ou = ou + t['rp_theta'] * (t['rp_mu'] - ou) * 1e-2 + \
                t['rp_sigma'] * np.sqrt(1e-2) * rng.standard_normal(2)
            a = np.clip(a + 2 * 0.5 * ou, -1.0, 1.0).astype(np.float32)   # tanh head, eps 0.5
            before = env.sim.step_count
            _, _, d = env.step(a)
            steps += env.sim.step_count - before
            if d:
                env.reset()
                ou = np.zeros(2)
            frame(d)
        return steps
    run(warm)
    t0 = time.perf_counter()
    steps = run(decisions)
    return steps, time.perf_counter() - t0, decisions


def cpu_actor_baseline(decisions, procs, train=False, updates=3):
    """configs[3] (train=False) / configs[4] (train=True) on the host cores: P
    explorer processes of the reference's per-observation act path on the
    config-4 maps (alternating small_loop / zigzag); with train, one of the P
    processes is a DDPG trainer instead (the reference's TrainManager runs
    explorers and trainers as separate processes side by side), timed
    concurrently.  value = the explorers' env-steps / the slowest explorer."""
    procs, avail, model = _cpu_info(procs)
    items = [(i, 3, decisions, ('small_loop', 'zigzag')[i % 2], 'explore')
             for i in range(procs - (1 if train else 0))]
    if train:
        items.append((procs, 0, updates, None, 'train'))
    res = _cpu_pool(_cpu_actor_worker, items, procs)
    ex = [r for r, it in zip(res, items) if it[4] == 'explore']
    total = sum(r[0] for r in ex)
    wall = max(r[1] for r in ex)
    out = {'value': total / wall, 'unit': 'env-steps/s', 'cores': procs, 'kind': 'port',
           'procs': procs, 'host_cores': os.cpu_count(), 'affinity_cores': avail,
           'deviation': DEVIATION % (procs, os.cpu_count()),
           'sample': '%d explorer processes x (3 warm-up + %d timed decisions), one env each: '
                     'per decision a batch-of-one float32 forward of the train-mode ConfigActor '
                     '(torch CPU, 1 thread; models/ddpg/model.py:74-102), OU noise, '
                     'oracle/dtsim_ref.py numpy-float64 step x repeat 3 (tanh head mapping), '
                     'oracle/render_oracle.c render + line filter, 3-frame stack; small_loop / '
                     'zigzag alternating; %d timed env-steps in %.1f s; host CPU: %s'
                     % (len(ex), decisions, total, wall, model)}
    if train:
        tr = [r for r, it in zip(res, items) if it[4] == 'train'][0]
        out['trainer'] = {'updates': tr[2], 'seconds': tr[1], 'updates_per_s': tr[2] / tr[1],
                          'what': 'one process: DDPGTrainer.update (critic + actor + soft '
                                  'targets) on torch CPU, batch %d, 1 thread, beside the '
                                  'explorers' % int(_reference_config()['training']['batch_size'])}
    return out


def _cpu_pool(worker, items, procs):
    import multiprocessing as mp
    pool = mp.get_context('spawn').Pool(procs)
    try:
        res = pool.map(worker, items)
    finally:
        pool.close()   # workers exit on their own (no terminate(): no SIGTERM under a profiler)
        pool.join()
    return res


def _cpu_info(procs):
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    if procs <= 0:
        # the GPU box's CPU share is 16 per GPU (harness rule; os.cpu_count() shows
        # the whole host there), so the pool is capped at 16 processes
        procs = max(1, min(16, avail))
    model = ''
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    return procs, avail, model


DEVIATION = ('BASELINE.md §3 asks for P = nproc processes; the pool is capped at the GPU box\'s '
             'CPU share of 16 per GPU (harness rule), so cores = processes = %d of %s logical '
             'cores on the host')


def cpu_baseline(steps, procs, map_name):
    """configs[1]: one env per process, 1,000 warm-up env-steps,
    then `steps` timed env-steps per process; aggregate = sum / slowest process."""
    procs, avail, model = _cpu_info(procs)
    res = _cpu_pool(_cpu_worker, [(i, 1000, steps, map_name) for i in range(procs)], procs)
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {'value': total / wall, 'unit': 'env-steps/s', 'cores': procs, 'kind': 'port',
            'procs': procs, 'host_cores': os.cpu_count(), 'affinity_cores': avail,
            'per_process': total / wall / procs, 'deviation': DEVIATION % (procs, os.cpu_count()),
            'sample': '%d processes x (1000 warm-up + %d timed env-steps), one env each: '
                      'oracle/dtsim_ref.py numpy-float64 restatement of Simulator.step + '
                      'EnvironmentWrapper.step (no render), %s, U[0,1)^2 wheel actions, '
                      'auto-reset; %d timed env-steps in %.1f s; host CPU: %s'
                      % (procs, steps, map_name, total, wall, model)}


def cpu_obs_baseline(decisions, procs, map_name):
    """configs[2] (BASELINE.md §3 obs path): one env per process, 20 warm-up
    decisions, then `decisions` timed decisions of step + render + line filter."""
    procs, avail, model = _cpu_info(procs)
    res = _cpu_pool(_cpu_obs_worker, [(i, 20, decisions, map_name) for i in range(procs)], procs)
    total = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {'value': total / wall, 'unit': 'env-steps/s', 'cores': procs, 'kind': 'port',
            'procs': procs, 'host_cores': os.cpu_count(), 'affinity_cores': avail,
            'per_process': total / wall / procs, 'deviation': DEVIATION % (procs, os.cpu_count()),
            'sample': '%d processes x (20 warm-up + %d timed decisions), one env each: per '
                      'decision oracle/dtsim_ref.py (numpy float64 Simulator.step x repeat 3 + '
                      'EnvironmentWrapper) then oracle/render_oracle.c (C, -O2, scalar: '
                      '120x160 raster + grey + HSV/inRange/dilate/Canny masks) and the 3-frame '
                      'stack, %s, U[0,1)^2 wheel actions, auto-reset; %d timed env-steps in '
                      '%.1f s; host CPU: %s' % (procs, decisions, map_name, total, wall, model)}


def load_pmc(kernel):
    """Per-launch PMC record of a kernel from profiles/pmc_traffic.json (or None)."""
    path = os.path.join(REPO, 'profiles', 'pmc_traffic.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    v = d.get(kernel)
    return v if isinstance(v, dict) else None


def split_even(total, most):
    """`total` decisions as ceil(total/most) launches whose sizes differ by <= 1."""
    if total <= 0:
        return []
    nl = -(-total // max(1, most))
    return [total // nl + (1 if i < total % nl else 0) for i in range(nl)]


class _Slice:
    """A StepOutput-shaped view of decisions [a, b) of a k*n-entry StepOutput."""

    def __init__(self, out, a, b, n):
        for name in ('reward', 'reward_mod', 'done', 'obs', 'lanepos', 'tile'):
            t = getattr(out, name)
            setattr(self, name, t[a * n:b * n] if t is not None else None)


# ---- process group ---------------------------------------------------------------------
class Ctx:
    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        self.local = int(os.environ.get('LOCAL_RANK', '0'))
        if self.world != args.gpus:
            raise SystemExit('bench.py: WORLD_SIZE=%d but --gpus %d' % (self.world, args.gpus))
        self.dry = args.dry_run
        if self.dry:
            self.dev = torch.device('cpu')
            self.backend = 'gloo'
        else:
            torch.cuda.set_device(self.local)
            self.dev = torch.device('cuda', self.local)
            self.backend = 'nccl'
        self.pg = False
        if self.world > 1:
            if self.dry:
                dist.init_process_group('gloo')
            else:
                dist.init_process_group('nccl', device_id=self.dev)
            self.pg = True

    def barrier(self):
        if self.pg:
            self.dist.barrier()

    def sync(self):
        if not self.dry:
            self.torch.cuda.synchronize(self.dev)

    def gather(self, values):
        """Every rank's float64 vector -> [world, len] list (rank order)."""
        t = self.torch.tensor(values, dtype=self.torch.float64, device=self.dev)
        if not self.pg:
            return [t.tolist()]
        parts = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return [p.tolist() for p in parts]

    def close(self):
        if self.pg:
            self.dist.destroy_process_group()


def rank_report(ctx, counts, elapsed):
    """All ranks' (env_steps, decisions, resets, elapsed) -> totals + per-rank list."""
    rows = ctx.gather(list(counts) + [elapsed])
    tot = [sum(r[i] for r in rows) for i in range(len(counts))]
    tmax = max(r[-1] for r in rows)
    per = [{'rank': i, 'env_steps': r[0], 'decisions': r[1], 'resets': r[2], 'elapsed_s': r[-1]}
           for i, r in enumerate(rows)]
    return tot, tmax, per


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(launch(args, argv))
    ctx = Ctx(args)
    if args.dry_run:
        return bench_dry(args, ctx)
    if args.config == 'actor':
        return bench_actor(args, ctx)
    if args.config == 'train':
        return bench_train(args, ctx)
    if args.config == 'lane':
        line = lane_record(args, ctx, args.steps, args.warmup, cpu=True)
        if ctx.rank == 0:
            print(json.dumps(line), flush=True)
        ctx.close()
        return
    return bench_obs(args, ctx)


def bench_dry(args, ctx):
    """No kernels: each rank 'steps' its shard synthetically, then the same
    barrier/max/sum/gather as the GPU path."""
    ctx.barrier()
    t0 = time.perf_counter()
    steps = args.envs * args.steps * 3
    elapsed = time.perf_counter() - t0 + 1e-6
    ctx.barrier()
    tot, tmax, per = rank_report(ctx, [steps, args.envs * args.steps, 0], elapsed)
    if ctx.rank == 0:
        print(json.dumps({'metric': METRIC, 'value': tot[0] / tmax, 'unit': 'env-steps/s',
                          'n_gpus': ctx.world, 'steps': args.steps, 'warmup': args.warmup,
                          'dry_run': True, 'backend': ctx.backend,
                          'process_group_world': ctx.world if ctx.pg else 1,
                          'per_rank': per,
                          'config': {'envs_per_gpu': args.envs,
                                     'global_envs': args.envs * ctx.world}}), flush=True)
    ctx.close()


def _bounds(sizes):
    a = 0
    for s in sizes:
        yield a, a + s
        a += s


def worst_over_ranks(ctx, parity, keys):
    """Parity fields: mismatch counts summed, errors maxed over ranks."""
    if parity is None or not ctx.pg:
        return parity
    rows = ctx.gather([parity[k] for k in keys])
    for i, k in enumerate(keys):
        vals = [r[i] for r in rows]
        parity[k] = sum(vals) if k.endswith('mismatches') else max(vals)
    parity['envs_checked'] *= ctx.world
    parity['ok'] = all(r[0] > 0 for r in ctx.gather([1.0 if parity['ok'] else 0.0]))
    return parity


STEP_PARITY_KEYS = ['pose_max_abs_err', 'reward_max_abs_err', 'reward_mod_max_abs_err',
                    'obs_max_abs_err', 'tile_mismatches', 'done_mismatches', 'counter_mismatches',
                    'check_pass_max_abs_diff']


# ---- config 3: the headline line --------------------------------------------------------
class ObsLoop:
    """The decisions of BASELINE configs[2], each a step of every env and the
    render of the pose it ends in (fresh = the step's done flags).  Modes:
      'many'   (default) the actions are known ahead (random), so dt_step_many
               steps a chunk of decisions in one launch (the fan kernel, 4.5 us
               a decision) and writes each decision's end pose; then the
               chunk's renders, each of its decision's pose and done flags.
      'serial' dt_step then dt_render of each decision on one stream.
      'pipe'   dt_step + dt_copy_pose on a high-priority stream, dt_render of
               the snapshot on another: step d + 1 beside render d.
    Every mode computes the same frames, masks and step outputs."""

    def __init__(self, env, ro, torch, mode='many', chunk=20, event_stride=1, group=3,
                 keep_masks=0):
        self.env, self.ro, self.torch, self.mode = env, ro, torch, mode
        # keep_masks = K: a bind of <= K decisions writes decision d's masks
        # into dmasks[d] (its own buffer, kept for the post-run check of every
        # decision) instead of the buffers a render group reuses
        self.dmasks = torch.empty((keep_masks,) + tuple(ro.masks.shape), dtype=torch.uint8,
                                  device=env.device) if keep_masks and ro.masks is not None \
            else None
        # 'many' / 'many2': up to `group` (<= 3, the ring's slots) consecutive
        # decisions' renders a launch (dt_render2 / dt_render3, one drain for
        # the group), each decision's masks in its own buffer
        self.group = max(1, min(3, int(group))) if mode in ('many', 'many2') and \
            ro.masks is not None else 1
        self.extra = [torch.zeros_like(ro.masks) for _ in range(self.group - 1)]
        self.last_masks = ro.masks
        self.launches = []    # per render launch: the decisions it renders
        # pipe mode orders the step stream on the render end events: all recorded
        self.event_stride = 1 if mode == 'pipe' else max(1, int(event_stride))
        lo, hi = torch.cuda.Stream.priority_range()
        self.s_step = torch.cuda.Stream(env.device, priority=hi if mode == 'pipe' else lo)
        two = mode in ('pipe', 'many2')
        self.s_rend = torch.cuda.Stream(env.device) if two else self.s_step
        self.chunk = max(1, min(int(chunk), 64))
        np_ = {'many': self.chunk, 'many2': 2 * self.chunk}.get(mode, 2)
        self.pose = torch.empty(np_, 3, env.n, dtype=torch.float64, device=env.device)

    def events(self, k):
        E = self.torch.cuda.Event
        return ([E() for _ in range(k)],
                [(E(enable_timing=True), E(enable_timing=True)) for _ in range(k)],
                [(E(enable_timing=True), E(enable_timing=True)) for _ in range(k)],
                [E() for _ in range(k)])

    def bind(self, actions, out):
        """The foreign calls of len(actions) decisions writing `out` (a
        StepOutput of k * n entries), built and checked before the timed region
        (the ring slots are taken here, in decision order)."""
        env, n, k = self.env, self.env.n, int(actions.shape[0])
        groups = []
        self.launches = []
        keep = self.dmasks is not None and k <= self.dmasks.shape[0]
        self.kept = keep
        own = self.ro.masks
        try:
            return self._bind(actions, out, env, n, k, groups, keep)
        finally:
            self.ro.masks = own

    def _bind(self, actions, out, env, n, k, groups, keep):
        from aido1_amd.render import bind_render, bind_render_group
        if self.mode in ('many', 'many2'):
            for c, (a, b) in enumerate(_bounds(split_even(k, self.chunk))):
                # many2: chunk c's poses in half c % 2 (its renders overlap step c + 1)
                h = self.chunk * (c % 2) if self.mode == 'many2' else 0
                pose = self.pose[h:h + b - a]
                step = env.bind_step_many(actions[a:b], _Slice(out, a, b, n), pose=pose,
                                          stream=self.s_step)
                rend = []
                d = a
                while d < b:
                    gk = min(self.group, b - d)
                    fr = [out.done[e * n:(e + 1) * n] for e in range(d, d + gk)]
                    extra = self.extra[:gk - 1]
                    if keep:   # the io structs take the buffers' addresses at bind time
                        self.ro.masks = self.dmasks[d]
                        extra = [self.dmasks[e] for e in range(d + 1, d + gk)]
                    if gk > 1:
                        rend.append(bind_render_group(env, self.ro, self.s_rend, extra, fr,
                                                      [pose[e - a] for e in range(d, d + gk)]))
                        self.last_masks = extra[gk - 2]
                    else:
                        rend.append(bind_render(env, self.ro, self.s_rend, fresh=fr[0],
                                                pose=pose[d - a]))
                        self.last_masks = self.ro.masks
                    self.launches.append(tuple(range(d, d + gk)))
                    d += gk
                groups.append((a, step, None, rend))
            return groups
        serial = self.mode == 'serial'
        for d in range(k):
            self.launches.append((d,))
            o = _Slice(out, d, d + 1, n)
            pose = None if serial else self.pose[d % 2]
            if keep:
                self.ro.masks = self.last_masks = self.dmasks[d]
            groups.append((d, env.bind_step(actions[d], o, self.s_step),
                           None if serial else env.bind_copy_pose(pose, self.s_step),
                           [bind_render(env, self.ro, self.s_rend, fresh=o.done, pose=pose)]))
        return groups

    def run(self, groups, ev):
        """Launch the bound decisions; returns the OR of the calls' status codes."""
        torch, env = self.torch, self.env
        ev_step, t_rend, t_step, ev_done = ev
        ss, sr = self.s_step, self.s_rend
        ss.wait_stream(torch.cuda.current_stream(env.device))
        rcs = 0
        li = 0    # render launch index (events are per launch)
        for c, (d0, step, copy, rends) in enumerate(groups):
            if self.mode == 'pipe' and d0 >= 2:
                ss.wait_event(t_rend[d0 - 2][1])
            if self.mode == 'many2' and c >= 2:     # its pose half is free again
                ss.wait_event(ev_done[groups[c - 2][0]])
            t_step[d0][0].record(ss)
            rcs |= step()
            t_step[d0][1].record(ss)
            if copy is not None:
                rcs |= copy()
            if sr is not ss:
                ev_step[d0].record(ss)
                sr.wait_event(ev_step[d0])
            for rend in rends:
                timed = li % self.event_stride == 0
                if timed:
                    t_rend[li][0].record(sr)
                rcs |= rend()
                if timed:
                    t_rend[li][1].record(sr)
                li += 1
            if self.mode == 'many2':
                ev_done[d0].record(sr)
        torch.cuda.current_stream(env.device).wait_stream(sr)
        return rcs


def bench_obs(args, ctx):
    torch = ctx.torch
    from aido1_amd.config import EnvConfig
    from aido1_amd.render import RENDER_BYTES_PER_ENV, RENDER_BYTES_PER_FRESH, RenderOutput
    from aido1_amd.vec_env import StepOutput, VecEnv
    dev, rank, n = ctx.dev, ctx.rank, args.envs
    W, K = args.warmup, args.steps
    env = VecEnv(n, seed=args.seed, device=dev.index, config=EnvConfig(map_name=args.map),
                 env_id_base=rank * n)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + 7919 * rank)
    actions = torch.rand(W + K, n, 2, generator=g, device=dev, dtype=torch.float32)
    ro = RenderOutput(n, dev)          # 3-slot grey ring (Transformer stack) + 4 masks
    loop = ObsLoop(env, ro, torch, args.obs_mode, args.many, args.event_stride,
                   group=1 if args.no_pair else args.render_group,
                   keep_masks=0 if args.no_parity else K)
    env.reset()
    wout = StepOutput(max(W, 1) * n, dev, lanepos=False, tile=False)
    if W and loop.run(loop.bind(actions[:W], wout), loop.events(W)):
        raise RuntimeError('a warm-up decision failed')
    ctx.sync()
    start = env.get_state()
    env.stats(reset=True)
    out = StepOutput(K * n, dev, lanepos=False, tile=False)
    ev = loop.events(K)
    calls = loop.bind(actions[W:], out)
    ctx.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    rcs = loop.run(calls, ev)
    t_host = time.perf_counter() - t0
    ctx.sync()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    if rcs:
        raise RuntimeError('a dt_step / dt_copy_pose / dt_render call failed in the timed region')
    st = env.stats()
    env.check()
    tot, tmax, per = rank_report(ctx, [st['sim_steps'], st['decisions'], st['resets']], elapsed)
    rend_ms = [ev[1][li][0].elapsed_time(ev[1][li][1]) for li in range(len(loop.launches))
               if li % loop.event_stride == 0]
    starts = [g[0] for g in calls]
    step_ms = [ev[2][d][0].elapsed_time(ev[2][d][1]) for d in starts]

    parity = None
    if not args.no_parity:
        # every timed decision's masks (each its own buffer), or the last one's
        import types
        frames = types.SimpleNamespace(slots=ro.slots, stack_view=ro.stack_view,
                                       masks=loop.last_masks,
                                       dmasks=loop.dmasks if loop.kept else None)
        parity = step_parity(env, start, actions[W:], out, rank, args, frames=frames)
    parity = worst_over_ranks(ctx, parity, STEP_PARITY_KEYS + ['gray_mismatches',
                                                               'mask_mismatches'])
    # the roofline's kernel time: an event-only pass after the timed region
    # with HIP events around EVERY dt_render (in the timed region they wrap
    # every --event-stride-th launch only: an event pair per launch adds ~6 us
    # a decision of stream packets to the wall time)
    KE = max(K, args.roofline_launches)
    ev_loop = ObsLoop(env, ro, torch, args.obs_mode, args.many, 1,
                      group=1 if args.no_pair else args.render_group)
    ev_act = torch.rand(KE, n, 2, generator=g, device=dev, dtype=torch.float32)
    ev_out = StepOutput(KE * n, dev, lanepos=False, tile=False)
    env.stats(reset=True)
    ev_all = ev_loop.events(KE)
    if ev_loop.run(ev_loop.bind(ev_act, ev_out), ev_all):
        raise RuntimeError('a call of the roofline pass failed')
    ctx.sync()
    ev_st = env.stats()
    nl = len(ev_loop.launches)
    rend_all = [ev_all[1][li][0].elapsed_time(ev_all[1][li][1]) for li in range(nl)]
    # the pass's algorithmic bytes, exactly: every decision's grey frame +
    # masks + pose, the refill of respawned envs' other slots, less the stores
    # a render pair does not make (dt_render2: the earlier decision's frame
    # store into the later one's slot, and its whole frame for envs the later
    # decision refills)
    dn = ev_out.done.view(KE, n).to(torch.int64)
    frame_b = RENDER_BYTES_PER_FRESH // 2
    pass_bytes = KE * RENDER_BYTES_PER_ENV * n + RENDER_BYTES_PER_FRESH * int(dn.sum())
    for la in ev_loop.launches:
        # decision i of a group against its sequential frame stores (3 slots
        # on a refill, else 1): none if a later decision refills the env,
        # else all but the later decisions' slots on a refill, else its slot
        g = len(la)
        for i in range(g - 1):
            fi = dn[la[i]]
            later = dn[list(la[i + 1:])].amax(0)
            written = (1 - later) * (fi * (3 - (g - 1 - i)) + (1 - fi))
            pass_bytes -= frame_b * int(((1 + 2 * fi) - written).sum())
    env.close()
    lane = None if args.no_lane else lane_record(args, ctx, args.lane_steps, args.lane_warmup,
                                                 cpu=True)
    # configs 4 and 5 as sub-records of the same line (not the headline)
    # (at the reference's float32 acting precision; the fp16 fast mode beside)
    c4 = c4h = c5 = c5h = None
    if not args.no_sub:
        c4 = actor_record(args, ctx, args.sub_steps, args.sub_warmup, parity=not args.no_parity,
                          cpu=True, dtype=torch.float32)
        c4h = actor_record(args, ctx, args.sub_steps, args.sub_warmup,
                           parity=not args.no_parity, dtype=torch.float16)
        c5 = train_record(args, ctx, args.sub_steps, args.sub_warmup, parity=not args.no_parity,
                          cpu=True, dtype=torch.float32)
        c5h = train_record(args, ctx, args.sub_steps, args.sub_warmup,
                           parity=not args.no_parity, dtype=torch.float16)
    if rank == 0:
        kms = float(np.mean(rend_all))
        fresh_per_launch = ev_st['resets'] / KE
        bpl = pass_bytes / nl
        per_launch_dec = KE / nl
        achieved = bpl / (kms * 1e-3) / 1e9
        pmc = load_pmc('render_kernel') or {}
        line = {
            'metric': METRIC, 'value': tot[0] / tmax, 'unit': 'env-steps/s',
            'n_gpus': ctx.world, 'steps': K, 'warmup': W,
            'ms_per_step': tmax / K * 1e3, 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'f64 step / f32 raster + grey / u8 masks',
            'data': 'synthetic',
            'config': {'workload': 'config3: %d envs/GPU, lane pose + 120x160 top-down render + '
                                   'grey frame ring + line_detector1 HSV/edge masks' % n,
                       'map': args.map, 'envs_per_gpu': n, 'global_envs': n * ctx.world,
                       'repeat_actions': 3, 'auto_reset': True,
                       'actions': 'U[0,1)^2 wheel velocities, resident in HBM',
                       'launch': {
                           'many': 'dt_step_many over chunks of <= %d decisions (each '
                                   'decision\'s end pose written), then the chunk\'s renders, '
                                   'each of its decision\'s pose with its done flags as fresh, '
                                   '%s; one stream, prebound calls'
                                   % (args.many, '%d consecutive decisions a launch '
                                      '(dt_render%d, each decision its own masks buffer)'
                                      % (loop.group, loop.group) if loop.group > 1
                                      else 'one decision a launch (dt_render)'),
                           'many2': 'dt_step_many over chunks of <= %d decisions on a step '
                                    'stream (each decision\'s end pose written, two pose '
                                    'buffers), each decision\'s dt_render of that pose on a '
                                    'render stream: chunk c + 1\'s steps beside chunk c\'s '
                                    'renders; prebound calls' % args.many,
                           'serial': 'per decision: dt_step then dt_render, one stream, prebound',
                           'pipe': 'per decision: dt_step + dt_copy_pose (high-priority stream), '
                                   'dt_render of the snapshot (render stream), prebound'
                       }[args.obs_mode],
                       'parallelism': 'env shards (%d x %d), no collective' % (ctx.world, n)},
            'counts': {'env_steps': tot[0], 'decisions': tot[1], 'resets': tot[2],
                       'elapsed_s': tmax},
            'per_rank': per,
            'process_group': {'backend': 'nccl (RCCL)' if ctx.pg else None,
                              'world': ctx.dist.get_world_size() if ctx.pg else 1},
            'parity': parity,
            'roofline': {'bound': 'hbm', 'kernel': 'render_kernel', 'achieved': achieved,
                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                         'traffic': pmc.get('hbm_bytes_per_launch'),
                         'traffic_round': pmc.get('round'),
                         'avg_kernel_ms': kms, 'min_kernel_ms': float(np.min(rend_all)),
                         'max_kernel_ms': float(np.max(rend_all)),
                         'timed_region_sampled_ms': float(np.mean(rend_ms)),
                         'algorithmic_bytes_per_launch': bpl,
                         'decisions_per_launch': per_launch_dec,
                         'algorithmic_basis': 'per env: grey f32 76,800 + 4 u8 masks 76,800 '
                                              'written + pose 24 read (SURVEY §8d config 3 '
                                              'without the step\'s 81 B); plus 153,600 B of '
                                              'ring refill per respawned env (%.1f per '
                                              'decision), per decision; a dt_render2/3 launch '
                                              'holds two or three decisions, less the stores it '
                                              'does not make (an earlier decision\'s frame where '
                                              'a later one writes or refills), counted from the '
                                              'done flags' % fresh_per_launch,
                         'timing': 'HIP events on the render stream around every dt_render of '
                                   'a %d-decision pass right after the timed region (same '
                                   'envs, launches and streams; %d launches averaged); '
                                   'timed_region_sampled_ms: events around every %d-th '
                                   'dt_render inside the timed region (%d launches)'
                                   % (KE, len(rend_all), loop.event_stride, len(rend_ms))},
            'step_launch_ms': float(np.mean(step_ms)),
            'step_launches': len(starts),
            'host_enqueue_ms_per_step': t_host / K * 1e3,
            'config2': lane,
            'config4': c4,
            'config4_fp16': c4h,
            'config5': c5,
            'config5_fp16': c5h,
        }
        line['cpu_baseline'] = (cpu_obs_baseline(args.cpu_decisions, args.cpu_procs, args.map)
                                if ctx.world == 1 and args.cpu_steps > 0 else None)
        print(json.dumps(line), flush=True)
    ctx.close()


# ---- config 2 ------------------------------------------------------------------------------
def lane_record(args, ctx, K, W, cpu):
    """BASELINE configs[1]: lane-pose obs only; the K timed decisions split into
    equal dt_step_many launches of at most --many decisions, each one prebound
    foreign call (--graph: one captured HIP graph)."""
    torch = ctx.torch
    from aido1_amd.config import EnvConfig
    from aido1_amd.vec_env import StepOutput, VecEnv
    dev, rank, n = ctx.dev, ctx.rank, args.envs
    env = VecEnv(n, seed=args.seed, device=dev.index, config=EnvConfig(map_name=args.map),
                 env_id_base=rank * n)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + 7919 * rank)
    actions = torch.rand(W + K, n, 2, generator=g, device=dev, dtype=torch.float32)
    env.reset()
    ctx.sync()

    # warm-up: the same launch shape as the timed region
    for a, b in _bounds(split_even(W, args.many)):
        wout = StepOutput((b - a) * n, dev, lanepos=False, tile=False)
        env.step_many_into(actions[a:b], wout)
    ctx.sync()
    start = env.get_state()

    sizes = split_even(K, args.many)
    out = StepOutput(K * n, dev, lanepos=False, tile=False)
    plan = [(W + a, W + b, _Slice(out, a, b, n)) for a, b in _bounds(sizes)]

    graph = None
    if args.graph:
        # the launches as one captured HIP graph (capture only: nothing runs here)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for a, b, o in plan:
                env.step_many_into(actions[a:b], o)
        ctx.sync()
        calls = [graph.replay]
    else:
        # prebound dt_step_many calls: one foreign call per launch, arguments
        # built and checked before the timed region
        calls = [env.bind_step_many(actions[a:b], o) for a, b, o in plan]
    env.stats(reset=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ctx.barrier()
    ctx.sync()
    e0.record()          # enqueued ahead of the launches; brackets them on the stream
    t0 = time.perf_counter()
    rcs = [f() for f in calls]
    e1.record()
    ctx.sync()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    if any(rcs):
        raise RuntimeError('dt_step_many failed in the timed region: %s' % rcs)
    st = env.stats()
    env.check()
    launches_ms = e0.elapsed_time(e1)
    tot, tmax, per = rank_report(ctx, [st['sim_steps'], st['decisions'], st['resets']], elapsed)
    sim_steps, decisions, resets = tot
    parity = None if args.no_parity else step_parity(env, start, actions[W:], out, rank, args)
    parity = worst_over_ranks(ctx, parity, STEP_PARITY_KEYS)
    env.close()
    if rank != 0:
        return None
    nl = len(sizes)
    kms = launches_ms / nl
    steps_per_launch = st['sim_steps'] / nl      # this rank's launches
    resets_per_launch = st['resets'] / nl
    survey_bytes = SURVEY_BYTES_PER_ENV_STEP * steps_per_launch
    fused_bytes = (MANY_BYTES_PER_ENV + MANY_BYTES_PER_ENV_DECISION * K / nl) * n + \
        MANY_BYTES_PER_RESET * resets_per_launch
    achieved = survey_bytes / (kms * 1e-3) / 1e9
    kname = 'step_fan_kernel'
    pmc = load_pmc(kname) or {}
    line = {
        'metric': METRIC,
        'value': sim_steps / tmax,
        'unit': 'env-steps/s',
        'n_gpus': ctx.world,
        'steps': K,
        'warmup': W,
        'ms_per_step': tmax / K * 1e3,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f64',
        'data': 'synthetic',
        'config': {
            'workload': 'config2: %d envs/GPU, lane-pose (dist, angle) obs' % n,
            'map': args.map, 'envs_per_gpu': n, 'repeat_actions': 3,
            'actions': 'U[0,1)^2 wheel velocities, resident in HBM',
            'auto_reset': True, 'global_envs': n * ctx.world,
            'launch': 'dt_step_many: %d launches of %s decisions%s' % (
                nl, '/'.join(str(s) for s in sorted(set(sizes), reverse=True)),
                ', one HIP graph' if graph is not None else ', prebound eager calls'),
            'parallelism': 'env shards (%d x %d), no collective' % (ctx.world, n)},
        'counts': {'env_steps': sim_steps, 'decisions': decisions, 'resets': resets,
                   'elapsed_s': tmax},
        'per_rank': per,
        'process_group': {'backend': 'nccl (RCCL)' if ctx.pg else None,
                          'world': ctx.dist.get_world_size() if ctx.pg else 1},
        'parity': parity,
        'roofline': {'bound': 'hbm', 'kernel': kname, 'achieved': achieved,
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                     'traffic': pmc.get('hbm_bytes_per_launch'),
                     'traffic_per': 'launch of %d decisions' % pmc['decisions_per_launch']
                     if 'decisions_per_launch' in pmc else None,
                     'avg_kernel_ms': kms,
                     'algorithmic_bytes_per_launch': survey_bytes,
                     'algorithmic_basis': 'SURVEY §8d 81 B/env-step x %.0f env-steps '
                                          'per launch' % steps_per_launch,
                     'fused_bytes_per_launch': fused_bytes,
                     'decisions_per_launch': K / nl,
                     'note': 'not HBM-bound (BASELINE.md §4): the bound is one env\'s '
                             'float64 dependency chain; see step_bound'},
        'step_ms_per_decision': launches_ms / K,
        'step_bound': step_bound_record(kms, K / nl, n, pmc),
    }
    line['cpu_baseline'] = (cpu_baseline(args.cpu_steps, args.cpu_procs, args.map)
                            if cpu and ctx.world == 1 and args.cpu_steps > 0 else None)
    return line


def step_bound_record(kms, dec_per_launch, n, pmc):
    """The config-2 kernel's real bound: per-decision time of one env's float64
    chain, and the fp64 issue rate it reaches vs the chip's (PMC counts from
    profiles/pmc_traffic.json when present)."""
    rec = {'us_per_decision': kms * 1e3 / dec_per_launch,
           'waves': 16 * n // 64,   # step_fan_kernel: each env on a quad of 4 waves
           'simds_on_chip': 1024}
    f = pmc.get('fp64_flops_per_launch')
    if f:
        tf = f / (kms * 1e-3) / 1e12
        rec.update({'fp64_tflops': tf, 'fp64_peak_tflops': FP64_VECTOR_PEAK_TFLOPS,
                    'fp64_frac': tf / FP64_VECTOR_PEAK_TFLOPS})
    return rec


def _render_items(item):
    """Pool worker of oracle_frames: oracle/render_oracle.c renders of a chunk
    of poses; returns each render's masks digest and the grey frames of the
    rows flagged in `keep`."""
    import hashlib
    rows, x, z, a, keep = item
    from oracle import oracle_c as OC
    gr, masks, _ = OC.OracleRender(rows).render(x, z, a)
    return [hashlib.blake2b(masks[i].tobytes(), digest_size=16).digest()
            for i in range(len(x))], gr[keep]


def oracle_frames(rows, x, z, a, keep, procs):
    """The oracle renders of poses (x, z, a) over `procs` processes: the 4
    masks of each as a digest, the grey frames of the rows with keep set."""
    parts = [p for p in np.array_split(np.arange(len(x)), max(1, procs)) if len(p)]
    items = [(rows, x[p], z[p], a[p], keep[p]) for p in parts]
    res = _cpu_pool(_render_items, items, len(items)) if len(items) > 1 else \
        [_render_items(items[0])]
    return [d for r in res for d in r[0]], np.concatenate([r[1] for r in res])


def mask_digests(masks):
    """Digests of [m, 4, H, W] u8 masks (as _render_items computes them)."""
    import hashlib
    a = masks.cpu().numpy()
    return [hashlib.blake2b(a[i].tobytes(), digest_size=16).digest() for i in range(len(a))]


def step_parity(env, start, actions, out, rank, args, frames=None, m=256):
    """Every env of this rank re-run by the C oracle (test infrastructure, used
    here as the checker only) from `start` through the timed decisions'
    actions, compared with the timed launches' outputs; then a dt_step check
    pass from the same start state with tile indices asked for.  With `frames`
    (the RenderOutput of the timed decisions), m envs' frame stacks (oldest
    first, as the Transformer concatenates them) are compared with
    oracle/render_oracle.c renders of the oracle's poses, and their masks: of
    EVERY timed decision when frames.dmasks holds each decision's masks (the
    launch form of the timed region, render groups included), else of the
    last one.  The oracle renders run on the host's CPU share (a process
    pool)."""
    import torch
    from aido1_amd.vec_env import StepOutput
    from oracle import oracle_c as OC
    n, K = env.n, out.reward.numel() // env.n
    rows = _map_rows(args.map)
    t0 = time.perf_counter()
    end = env.get_state()
    acts = actions[:K].cpu().numpy()
    g = {k: getattr(out, k).view(K, n, -1).squeeze(-1).cpu().numpy()
         for k in ('reward', 'reward_mod', 'done')}
    g['obs'] = out.obs.view(K, n, 2).cpu().numpy()
    idx = np.linspace(0, n - 1, m).astype(np.int64)
    ob = OC.OracleBatch(rows, n, seed=args.seed, env_base=rank * n)
    ob.set_state(**start)
    refs, track = [], []
    err = {'reward': 0.0, 'reward_mod': 0.0, 'obs': 0.0}
    done_mm = 0
    for d in range(K):
        r = ob.step(acts[d])
        refs.append(r)
        for k in err:
            err[k] = max(err[k], float(np.max(np.abs(g[k][d] - r[k]))))
        done_mm += int(np.count_nonzero(g['done'][d] != r['done']))
        every = frames is not None and getattr(frames, 'dmasks', None) is not None
        if frames is not None and (every or d >= K - frames.slots):
            o = ob.state()
            track.append((d, o['x'][idx].copy(), o['z'][idx].copy(), o['angle'][idx].copy(),
                          r['done'][idx].copy()))
    o = ob.state()
    pose_err = max(float(np.max(np.abs(end[k] - o[k]))) for k in ('x', 'z', 'angle'))
    cnt_mm = sum(int(np.count_nonzero(end[k] != o[k]))
                 for k in ('step_count', 'env_step', 'episode'))
    rec = {'envs_checked': n, 'decisions': K, 'oracle': 'oracle/dtsim_oracle.c (C restatement)'}
    if frames is not None:
        # the oracle renders of the tracked decisions' poses: every decision's
        # masks (digests), the grey frames of the last `slots` decisions
        tail = [t for t in track if t[0] >= K - frames.slots]
        cat = lambda i: np.concatenate([t[i] for t in track])   # noqa: E731
        keep_rows = np.concatenate([np.full(m, t[0] >= K - frames.slots) for t in track])
        procs = _cpu_info(getattr(args, 'cpu_procs', 0))[0]
        dig, grey = oracle_frames(rows, cat(1), cat(2), cat(3), keep_rows, procs)
        grey = grey.reshape(len(tail), m, *grey.shape[1:])
        # the ring as the Transformer holds it after the last decisions: a
        # respawn refills every slot with its frame, otherwise append + drop
        stack = None
        for t, gr in zip(tail, grey):
            dn = t[4]
            if stack is None:
                stack = np.repeat(gr[:, None], frames.slots, 1)
            else:
                stack = np.where(dn[:, None, None, None] != 0, gr[:, None],
                                 np.concatenate([stack[:, 1:], gr[:, None]], 1))
        got = frames.stack_view()[idx.tolist()].cpu().numpy()
        keep = frames.slots - len(tail) if len(tail) < frames.slots else 0
        sel = torch.as_tensor(idx, device=env.device)
        if every:
            mine = [h for d in range(K) for h in mask_digests(frames.dmasks[d].index_select(0, sel))]
        else:
            mine = mask_digests(frames.masks.index_select(0, sel))
            dig = dig[-m:]
        rec.update({'frame_envs_checked': m, 'frame_oracle': 'oracle/render_oracle.c',
                    'frames_per_env': frames.slots - keep,
                    'mask_decisions_checked': K if every else 1,
                    'gray_mismatches': int(np.count_nonzero(got[:, keep:] != stack[:, keep:])),
                    'mask_mismatches': int(sum(a != b for a, b in zip(mine, dig))),
                    'mask_mismatches_unit': '(decision, env) pairs whose 4 masks differ'})
    # check pass: dt_step from the same start, tile + lane pose produced
    env.set_state(**start)
    full = StepOutput(n, env.device)
    tile_mm = 0
    chk = 0.0
    for d in range(K):
        env.step_into(actions[d], full)
        torch.cuda.synchronize(env.device)
        tile_mm += int(np.count_nonzero(full.tile.cpu().numpy() != refs[d]['tile']))
        done_mm += int(np.count_nonzero(full.done.cpu().numpy() != refs[d]['done']))
        chk = max(chk, float(np.max(np.abs(full.reward.cpu().numpy() - g['reward'][d]))))
    end2 = env.get_state()
    chk = max(chk, max(float(np.max(np.abs(end2[k] - end[k]))) for k in ('x', 'z', 'angle')))
    env.check()
    frames_ok = frames is None or (rec['gray_mismatches'] == 0 and rec['mask_mismatches'] == 0)
    rec.update({'pose_max_abs_err': pose_err, 'reward_max_abs_err': err['reward'],
                'reward_mod_max_abs_err': err['reward_mod'], 'obs_max_abs_err': err['obs'],
                'done_mismatches': done_mm, 'tile_mismatches': tile_mm,
                'counter_mismatches': cnt_mm, 'check_pass_max_abs_diff': chk,
                'tolerance': {'pose': 1e-5, 'reward': 1e-5, 'tile_done': 'exact',
                              'frames_masks': 'exact'},
                'ok': bool(pose_err <= 1e-5 and err['reward'] <= 1e-5 and
                           err['reward_mod'] <= 1e-5 and done_mm == 0 and tile_mm == 0 and
                           cnt_mm == 0 and frames_ok),
                'seconds': time.perf_counter() - t0})
    return rec


# ---- configs 4 and 5 -----------------------------------------------------------------------
def actor_f64(actor, x, mode='reference', device='cpu'):
    """The actor in float64 (torch on `device`: the host by default, or the
    GPU's f64 units for large samples), dropout off: mode 'reference' =
    train-mode batch-of-one BatchNorm (per-sample statistics, the explorers'
    forward), 'eval' = the running statistics (the folded-BN policy); the
    precision yardstick of configs 4 / 5 (tools/actor_precision.py).
    Returns a CPU tensor."""
    import torch
    import torch.nn.functional as F
    from aido1_amd.actor import apply_head
    from aido1_amd.render import as_gray
    convs, bns, l1, l2 = actor.layers()
    d = lambda t: t.detach().double().to(device)   # noqa: E731
    h = as_gray(x.to(device)).double()
    for c, b in zip(convs, bns):
        h = F.leaky_relu(F.conv2d(h, d(c.weight), d(c.bias), stride=c.stride))
        if mode == 'eval':
            m = d(b.running_mean).view(1, -1, 1, 1)
            v = d(b.running_var).view(1, -1, 1, 1)
        else:
            m = h.mean((2, 3), keepdim=True)
            v = (h - m).square().mean((2, 3), keepdim=True)
        h = (h - m) / torch.sqrt(v + b.eps) * d(b.weight).view(1, -1, 1, 1) + \
            d(b.bias).view(1, -1, 1, 1)
    h = F.leaky_relu(F.linear(h.flatten(1), d(l1.weight), d(l1.bias)))
    return apply_head(F.linear(h, d(l2.weight), d(l2.bias)), actor.head).cpu()


# fp16 fast mode: the action bound against the float64 forward (DESIGN §3.6:
# measured max 6e-3 .. 1.0e-2 over 8192 actions, p99 3.4e-3 .. 3.9e-3; the
# per-sample BatchNorm of nearly flat channels amplifies fp16 rounding)
FP16_ACTION_TOL = 1.5e-2
F32_ACTION_TOL = 1e-4


def actor_record(args, ctx, K, W, parity=True, dtype=None, cpu=False):
    """BASELINE configs[3]: 4096 envs/GPU, mixed small_loop/zigzag, actor in the
    loop (the explorers' loop body, training/explorers.py:164-213).  Returns
    the line (rank 0) or None.  dtype: the actor's arithmetic (float32, the
    default: the reference's precision, the x3 chain; float16: the fast
    mode).  parity: every env's actions against the other-precision GPU path,
    and --f64-envs envs' against a float64 forward (actor_f64 on the GPU),
    dropout off."""
    torch = ctx.torch
    from aido1_amd.actor import FusedActor
    from aido1_amd.rollout import ActorRollout
    cfg = _reference_config()
    dtype = dtype or torch.float32
    dev, rank, n = ctx.dev, ctx.rank, args.envs
    torch.manual_seed(args.seed)
    roll = ActorRollout(cfg, n, maps=('small_loop', 'zigzag'), device=dev.index, seed=args.seed,
                        env_id_base=rank * n, actor_mode=args.actor_mode, dtype=dtype,
                        frames=args.frames)
    roll.reset()
    for _ in range(W):
        roll.step()
    ctx.sync()
    roll.stats(reset=True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K)]
    ctx.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for k in range(K):
        roll.step(timing=ev[k])
    ctx.sync()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    st = roll.stats()
    actor_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    tot, tmax, per = rank_report(ctx, [st['sim_steps'], st['decisions'], st['resets']], elapsed)
    par = None
    if parity:
        other = torch.float32 if dtype == torch.float16 else torch.float16
        drop = roll.actor.p_drop
        roll.actor.p_drop = 0.0
        with torch.no_grad():
            alt = FusedActor(roll.actor_src, dtype=other, mode=roll.actor.mode)
            alt.p_drop = 0.0
            got = roll.actor(roll.ring, roll.order()).float()
            want = alt(roll.ring, roll.order()).float()
            m = min(n, args.f64_envs)
            ref64 = actor_f64(roll.actor_src, roll.stack()[:m], roll.actor.mode, device=dev)
        roll.actor.p_drop = drop
        d = torch.abs(got - want)
        e64 = (got[:m].double().cpu() - ref64).abs()
        a64 = (want[:m].double().cpu() - ref64).abs()
        tol = FP16_ACTION_TOL if dtype == torch.float16 else F32_ACTION_TOL
        par = {'vs': 'float64 forward (actor_f64 on the GPU\'s f64 units, same weights, live '
                     'frames, dropout off) on %d envs; and the %s GPU path on every env'
                     % (m, other),
               'tolerance_vs_f64': tol, 'envs_checked': n, 'envs_checked_f64': m,
               'max_abs_err_vs_f64': e64.max().item(),
               'other_path_max_abs_err_vs_f64': a64.max().item(),
               'max_abs_err_vs_other': d.max().item(),
               'p99_abs_err_vs_other': torch.quantile(d.flatten(), 0.99).item()}
        par['ok'] = bool(torch.isfinite(got).all()) and par['max_abs_err_vs_f64'] <= tol
        par = worst_over_ranks(ctx, par, ['max_abs_err_vs_f64', 'max_abs_err_vs_other',
                                          'p99_abs_err_vs_other'])
    roll.close()
    base = None
    if cpu and ctx.world == 1 and args.cpu_steps > 0 and rank == 0:
        base = cpu_actor_baseline(args.cpu_actor_decisions, args.cpu_procs)
    if rank != 0:
        return None
    name = str(dtype).replace('torch.', '')
    frame_b = 1 if args.frames == 'index' else 4
    return {
        'metric': METRIC, 'value': tot[0] / tmax, 'unit': 'env-steps/s',
        'n_gpus': ctx.world, 'steps': K, 'warmup': W,
        'ms_per_step': tmax / K * 1e3,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'f64 env / %s actor' % name,
        'precision': ('fast mode: fp16 MFMA operands, f32 accumulation (narrower than the '
                      'reference\'s float32)' if dtype == torch.float16 else
                      'the reference\'s float32 (models/ddpg/model.py:74-88)'),
        'data': 'synthetic',
        'config': {'workload': 'config4: %d envs/GPU, actor in the loop (ConfigActor, '
                               'config.json), mixed small_loop/zigzag' % n,
                   'actor_mode': args.actor_mode, 'frames': args.frames, 'envs_per_gpu': n,
                   'global_envs': n * ctx.world, 'repeat_actions': 3,
                   'weights': 'random init (no checkpoint offline)',
                   'parallelism': 'env shards (%d x %d), no collective' % (ctx.world, n)},
        'counts': {'env_steps': tot[0], 'decisions': tot[1], 'resets': tot[2],
                   'elapsed_s': tmax},
        'per_rank': per,
        'parity': par,
        'roofline': actor_roofline(torch, dtype, n, actor_ms, frame_b),
        'cpu_baseline': base}


def actor_roofline(torch, dtype, n, actor_ms, frame_b):
    """The roofline object of the actor forward (configs 4 / 5).  fp16 fast
    mode: MFMA-bound against the fp16 dense peak.  float32 (the x3 chain,
    include/dtactor.h): its HBM bytes (actor.x3_bytes_per_sample: the HL
    activations written and read) bound it before its arithmetic (three fp16
    MFMA products per f32 product: a ceiling of the fp16 peak / 3), so the
    bound is HBM, the MFMA figures beside it."""
    from aido1_amd.actor import flops_per_sample, x3_bytes_per_sample
    flops = n * flops_per_sample()
    tflops = flops / (actor_ms * 1e-3) / 1e12
    common = {'avg_kernel_ms': actor_ms, 'traffic': None,
              'timing': 'HIP events around the actor forward of every timed decision',
              'algorithmic_flops_per_launch': flops}
    if dtype == torch.float16:
        return dict(common, bound='mfma', kernel='actor forward (fp16 MFMA convs + linears)',
                    achieved=tflops, peak=BF16_DENSE_PEAK_TFLOPS, unit='TFLOP/s',
                    frac=tflops / BF16_DENSE_PEAK_TFLOPS)
    nbytes = n * x3_bytes_per_sample(frame_b)
    gbs = nbytes / (actor_ms * 1e-3) / 1e9
    return dict(common, bound='hbm',
                kernel='actor forward at float32 accuracy (dt_conv1x_split + dt_conv32x_split '
                       'x3 on fp16 MFMA, float32 linears)',
                achieved=gbs, peak=HBM_PEAK_GBS, unit='GB/s', frac=gbs / HBM_PEAK_GBS,
                algorithmic_bytes_per_launch=nbytes,
                algorithmic_basis='per sample: the 3 stacked frames read, each HL activation '
                                  '(conv1..conv3 outputs, 4 B an element) written and read, '
                                  'the f32 flattened conv4 output written and read',
                mfma={'achieved': tflops, 'unit': 'TFLOP/s', 'peak_x3': X3_PEAK_TFLOPS,
                      'frac_x3': tflops / X3_PEAK_TFLOPS,
                      'f32_mfma_peak': F32_MFMA_PEAK_TFLOPS,
                      'note': 'algorithmic f32 FLOP; x3 runs three fp16 MFMA products per '
                              'f32 product'})


def bench_actor(args, ctx):
    torch = ctx.torch
    line = actor_record(args, ctx, args.steps, args.warmup, parity=not args.no_parity,
                        dtype=torch.float32 if args.actor_dtype == 'float32' else torch.float16,
                        cpu=True)
    if line is not None:
        print(json.dumps(line), flush=True)
    ctx.close()


def train_record(args, ctx, K, W, parity=True, cpu=False, dtype=None):
    """BASELINE configs[4]: full DDPG on every GPU -- actor-in-loop rollout of
    4096 envs, GPU prioritized replay, one update per decision
    (training/trainers.py:143-237), gradients all-reduced over RCCL (world >
    1).  value = env-steps/s; updates/s beside.  parity: the non-finite guards
    of every stage (TrainLoop.check), the replay's rejected priorities and the
    sum tree's invariants after the timed run."""
    torch = ctx.torch
    from aido1_amd.train_loop import TrainLoop
    cfg = _reference_config()
    dev, rank, n = ctx.dev, ctx.rank, args.envs
    if dtype is None:
        dtype = torch.float32 if args.actor_dtype == 'float32' else torch.float16
    loop = TrainLoop(cfg, n, device=dev.index, seed=args.seed, env_id_base=rank * n,
                     buffer_size=args.buffer_size, batch_size=args.batch_size or None,
                     updates_per_step=args.updates_per_step, actor_mode=args.actor_mode,
                     overlap=args.overlap, frames=args.frames, actor_dtype=dtype)
    loop.reset()
    for _ in range(max(W, 2)):
        loop.step()
    ctx.sync()
    loop.rollout.stats(reset=True)
    u0 = loop.updates
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(K)]
    uev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(K)]
    ctx.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for k in range(K):
        loop.step(timing=ev[k], update_timing=uev[k])
    loop.flush()
    ctx.sync()
    ctx.barrier()
    elapsed = time.perf_counter() - t0
    st = loop.rollout.stats()
    actor_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    try:   # a decision without an update (buffer below a batch) records no events
        update_ms = float(np.mean([a.elapsed_time(b) for a, b in uev]))
    except RuntimeError:
        update_ms = None
    tot, tmax, per = rank_report(ctx, [st['sim_steps'], st['decisions'], st['resets'],
                                       loop.updates - u0], elapsed)
    sim_steps, decisions, resets, updates = tot
    par = None
    if parity:
        par = {'losses_finite': bool(torch.isfinite(loop.metrics['critic_loss']).item()
                                     and torch.isfinite(loop.metrics['actor_loss']).item())}
        guard_ok = False
        try:
            rec = loop.check()
            par['guard'] = 'clean: no stage reported NaN / Inf over %d updates' % rec['tick']
            guard_ok = True
        except Exception as e:  # noqa: BLE001 -- reported in the line
            par['guard'] = str(e)
        if loop.prioritized:
            s_, mn, mp = loop.replay.trees()
            cap = loop.replay.capacity
            leaves = s_[cap:].double()
            par['tree_root_vs_leaf_sum_rel'] = abs(leaves.sum().item() - s_[1].item()) / max(
                s_[1].item(), 1e-300)
            par['max_priority'] = mp.item()
            par['stored'] = len(loop.replay)
        par['critic_loss'] = loop.metrics['critic_loss'].item()
        par['actor_loss'] = loop.metrics['actor_loss'].item()
        # the finished episodes of the run, gathered over the ranks (explorers.py:134-140)
        eps = loop.poll_episodes()
        par['episodes'] = {'finished': int(len(eps['reward'])),
                           'mean_reward': float(eps['reward'].mean()) if len(eps['reward'])
                           else None,
                           'mean_step': float(eps['step'].mean()) if len(eps['step']) else None,
                           'exploiter_best_reward': loop.book.exploiter.best}
        par['ok'] = bool(guard_ok and par['losses_finite'] and
                         par.get('tree_root_vs_leaf_sum_rel', 0.0) <= 1e-9)
    nparams = sum(p.numel() for p in loop.trainer.actor.parameters()) + \
        sum(p.numel() for p in loop.trainer.critic.parameters())
    dtype_name = str(loop.rollout.actor.dtype).replace('torch.', '')
    batch = loop.batch_size
    loop.rollout.close()
    base = None
    if cpu and ctx.world == 1 and args.cpu_steps > 0 and rank == 0:
        base = cpu_actor_baseline(args.cpu_actor_decisions, args.cpu_procs, train=True,
                                  updates=args.cpu_updates)
    if rank != 0:
        return None
    return {
        'metric': METRIC, 'value': sim_steps / tmax, 'unit': 'env-steps/s',
        'n_gpus': ctx.world, 'steps': K, 'warmup': W,
        'ms_per_step': tmax / K * 1e3,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': 'f64 env / %s actor / f32 update' % dtype_name,
        'precision': ('fast mode: fp16 MFMA actor operands (narrower than the reference\'s '
                      'float32)' if dtype == torch.float16 else
                      'the reference\'s float32 acting (models/ddpg/model.py:74-88)'),
        'data': 'synthetic',
        'config': {'workload': 'config5: %d envs/GPU full DDPG (rollout + GPU prioritized '
                               'replay + update + grad all-reduce)' % n,
                   'actor_mode': args.actor_mode, 'frames': args.frames, 'envs_per_gpu': n,
                   'global_envs': n * ctx.world, 'batch_size_per_gpu': batch,
                   'buffer_size_per_gpu': args.buffer_size,
                   'updates_per_step': args.updates_per_step,
                   'update_overlap': None if not args.overlap else
                   'update t on a side stream beside rollout t+1; acting weights one '
                   'update behind (the reference explorers act asynchronously): a '
                   'different schedule from the sequential loop, not the same run done '
                   'faster',
                   'weights': 'random init (config.json xavier_normal)',
                   'parallelism': 'env shards (%d x %d) + data-parallel update, RCCL '
                                  'all-reduce of %d gradients' % (ctx.world, n, nparams)},
        'counts': {'env_steps': sim_steps, 'decisions': decisions, 'resets': resets,
                   'updates_all_ranks': updates, 'elapsed_s': tmax,
                   'synchronous_updates_per_s': K / tmax,
                   'samples_per_s': batch * updates / tmax},
        'phases_ms': {'actor': actor_ms, 'update': update_ms,
                      'timing': 'HIP events around the actor forward and around the '
                                'update(s) of every timed decision (rank 0)'},
        'per_rank': per,
        'parity': par,
        'roofline': actor_roofline(torch, dtype, n, actor_ms,
                                   1 if args.frames == 'index' else 4),
        'cpu_baseline': base}


def bench_train(args, ctx):
    line = train_record(args, ctx, args.steps, args.warmup, parity=not args.no_parity)
    if line is not None:
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == '__main__':
    main()
