#!/usr/bin/env python
"""bench.py — BASELINE.json's metric: env-steps/s (whole node) at 4096 envs/GPU.

Workload (BASELINE.json configs[1]): 4096 envs per GPU
on loop_empty, lane-pose (dist, angle) observation, i.i.d. U[0,1)^2 wheel
actions (the train.py contract after utils/env_wrappers.py:214-216), Philox
spawn streams keyed by seed 1234, auto-reset on done or at the 2000-step wrapper
cap.  One bench "step" = one VecEnv.step = one EnvironmentWrapper.step for every
env = up to repeat_actions (3) Simulator steps each; the unit counted is the
Simulator step (env-step), read back exactly from the device counters (envs
that finish mid-repeat run fewer).  Actions for every step are generated and
resident in HBM before the timed region.

  python bench.py [--gpus N --steps K --warmup W] [--config lane|render|actor|train]

Other configs (not the headline line): render = configs[2] (obs pipeline),
actor = configs[3] (actor in the loop), train = configs[4] (full DDPG: rollout +
GPU prioritized replay + update + RCCL gradient all-reduce).

N > 1: launched by torch.distributed.run, one rank per GPU; envs shard by
env_id_base = rank * envs (disjoint spawn streams), no data-path collective;
timing = barrier + synchronize on both sides, max over ranks; value = all
ranks' env-steps / that time.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = 'env-steps/sec (whole node) at 4096 envs/GPU; pose/reward max-abs-err vs CPU ref'
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec

# Algorithmic HBM bytes of one dt_step launch (step_kernel, k = 1: step lanes +
# the spawn-ahead refill blocks), DESIGN.md §3.1-3.2:
# step, per env:  reads pose 24 + step_count,env_step 8 + action 8 + episode,tick 8
#                 + seed 8 + the 8 slot words 64                                 = 120
#                 writes pose 24 + counters 8 + tick 4 + reward 8 + reward_mod 8
#                 + done 1 + obs 8                                               = 61
# refill scan, per env: want 4 + tick 4 + slot words 64 + seed 8                 = 80
# per reset:  the slot's record 56 read; episode + want 8 written; the refill of
#             the consumed key writes its slot record 56 + word 8                = 128
STEP_BYTES_PER_ENV = 120 + 61 + 80
SPAWN_BYTES_PER_RESET = 128
# One dt_step_many launch of k decisions (step_pair_kernel over k):
# per env, once: reads pose 24 + step_count,env_step 8 + episode,tick 8 + seed 8
#                + the 8 slot words 64 = 112; writes pose 24 + counters 8 + tick 4 = 36
#   refill scan: 80 (as above)
# per env and decision: action 8 + reward 8 + reward_mod 8 + done 1 + obs 8 = 33
# per reset: 128 (as above)
MANY_BYTES_PER_ENV = 112 + 36 + 80
MANY_BYTES_PER_ENV_DECISION = 33
MANY_BYTES_PER_RESET = 128


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=320)
    p.add_argument('--warmup', type=int, default=30)
    p.add_argument('--envs', type=int, default=4096)
    p.add_argument('--map', default='loop_empty')
    p.add_argument('--config', default='lane', choices=['lane', 'render', 'actor', 'train'])
    p.add_argument('--actor-mode', default='reference', choices=['reference', 'eval'],
                   help="actor/train: 'reference' = train-mode batch-of-one BatchNorm + live "
                        "dropout as the reference's explorers act; 'eval' = BN folded")
    p.add_argument('--batch-size', type=int, default=0, help='train: 0 = config.json (64)')
    p.add_argument('--buffer-size', type=int, default=131072)
    p.add_argument('--updates-per-step', type=int, default=1)
    p.add_argument('--many', type=int, default=16,
                   help='lane config: decisions per dt_step_many launch (0 = dt_step per '
                        'decision, in HIP graphs of --graph-steps)')
    p.add_argument('--graph-steps', type=int, default=30,
                   help='lane config with --many 0: decisions per HIP-graph replay '
                        '(VecEnv.capture); 0 = one eager launch per decision')
    p.add_argument('--seed', type=int, default=1234)
    p.add_argument('--cpu-seconds', type=float, default=1.5,
                   help='per-process seconds of the CPU baseline sample (0 = skip)')
    p.add_argument('--cpu-procs', type=int, default=0)
    return p.parse_args()


# ---- CPU baseline: the oracle's numpy restatement of step(), one env/process ----
def _cpu_worker(args):
    idx, seconds, map_name = args
    import yaml
    from oracle import dtsim_ref as R
    with open(os.path.join(REPO, 'aido1_amd', 'maps', map_name + '.yaml')) as f:
        rows = yaml.safe_load(f)['tiles']
    env = R.EnvironmentWrapperRef(R.SimulatorRef(rows, seed=1234, env_id=idx))
    env.reset()
    rng = np.random.default_rng(1234 + idx)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            a = rng.random(2, dtype=np.float32)
            before = env.sim.step_count
            _, _, d = env.step(a)
            steps += env.sim.step_count - before
            if d:
                env.reset()
    return steps, time.perf_counter() - t0


def cpu_baseline(seconds, procs, map_name):
    import multiprocessing as mp
    if procs <= 0:
        try:
            avail = len(os.sched_getaffinity(0))
        except AttributeError:
            avail = os.cpu_count() or 1
        procs = max(1, min(16, avail))
    ctx = mp.get_context('spawn')
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(i, seconds, map_name) for i in range(procs)])
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    model = ''
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    return {'value': steps / wall, 'unit': 'env-steps/s', 'cores': procs, 'kind': 'port',
            'sample': '%d processes x %.1f s, one env each: oracle/dtsim_ref.py numpy-float64 '
                      'restatement of Simulator.step + EnvironmentWrapper.step (no render), '
                      '%s, U[0,1)^2 wheel actions, auto-reset; %d env-steps; host CPU: %s'
                      % (procs, seconds, map_name, steps, model)}


def load_traffic(kernel):
    """Per-launch HBM bytes from a committed rocprofv3 PMC summary (or None)."""
    path = os.path.join(REPO, 'profiles', 'pmc_traffic.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    v = d.get(kernel)
    return v.get('hbm_bytes_per_launch') if isinstance(v, dict) else None


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device('cuda', local if world > 1 else 0)

    from aido1_amd.config import EnvConfig
    from aido1_amd.vec_env import StepOutput, VecEnv

    n = args.envs
    if args.config == 'actor':
        return bench_actor(args, dev, rank, world, dist)
    if args.config == 'train':
        return bench_train(args, dev, rank, world, dist)
    env = VecEnv(n, seed=args.seed, device=dev.index,
                 config=EnvConfig(map_name=args.map), env_id_base=rank * n)
    out = StepOutput(n, dev, lanepos=False, tile=False)
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + 7919 * rank)
    total = args.warmup + args.steps
    actions = torch.rand(total, n, 2, generator=g, device=dev, dtype=torch.float32)
    render = None
    if args.config == 'render':
        from aido1_amd.render import RenderOutput
        render = RenderOutput(n, dev)
    env.reset()
    torch.cuda.synchronize(dev)

    def one(i):
        env.step_into(actions[i], out)
        if render is not None:
            env.render_into(render, fresh=out.done)

    M = max(0, args.many) if render is None else 0
    G = max(0, args.graph_steps) if render is None and not M else 0
    if M:
        # k = M decisions per launch (dt_step_many), outputs of every decision kept
        mb = list(range(0, args.steps, M)) + [args.steps]   # the last takes the rest
        chunks = list(zip(mb[:-1], mb[1:]))
        outs = {}
        for a, b in chunks + [(0, M)]:
            if b - a not in outs:
                outs[b - a] = StepOutput((b - a) * n, dev, lanepos=False, tile=False)
        mev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in chunks]
        for i in range(0, args.warmup, M):   # warmup launches of M decisions too
            env.step_many_into(actions[:M], outs[M])
    else:
        for i in range(args.warmup):
            one(i)
    torch.cuda.synchronize(dev)
    if G:
        # the timed decisions as HIP graphs of G launches each, captured up
        # front over their own action slices (StepGraph)
        bounds = list(range(0, args.steps, G)) + [args.steps]   # the last takes the rest
        graphs = [env.capture(actions[args.warmup + a:args.warmup + b], out)
                  for a, b in zip(bounds[:-1], bounds[1:])]
        gev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in graphs]
    env.stats(reset=True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)] if not (G or M) else []
    rev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)] if render is not None else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if M:
        for c, (a, b) in enumerate(chunks):
            mev[c][0].record()
            env.step_many_into(actions[args.warmup + a:args.warmup + b], outs[b - a])
            mev[c][1].record()
    elif G:
        for c, gr in enumerate(graphs):
            gev[c][0].record()
            gr.replay()
            gev[c][1].record()
    else:
        for k in range(args.steps):
            i = args.warmup + k
            ev[k][0].record()
            env.step_into(actions[i], out)
            ev[k][1].record()
            if render is not None:
                rev[k][0].record()
                env.render_into(render, fresh=out.done)
                rev[k][1].record()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = env.stats()
    env.check()
    if M:  # per decision: launch times / decisions (a launch runs M of them)
        step_ms = float(np.sum([a.elapsed_time(b) for a, b in mev])) / args.steps
        launch_ms = float(np.mean([a.elapsed_time(b) for a, b in mev]))
    elif G:  # per launch inside the graphs: replay time / launches (gaps included)
        step_ms = float(np.sum([a.elapsed_time(b) for a, b in gev])) / args.steps
    else:
        step_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    render_ms = float(np.mean([a.elapsed_time(b) for a, b in rev])) if rev else None

    sims = torch.tensor([st['sim_steps'], st['decisions'], st['resets']], dtype=torch.float64,
                        device=dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(sims, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    sim_steps, decisions, resets = (float(v) for v in sims.tolist())
    tmax = float(tmax.item())

    if rank == 0:
        if render is None and M:
            # one launch = len(chunks) of them over args.steps decisions;
            # step_pair_kernel unless DTSIM_STEP_PAIR=0
            kname = ('step_kernel' if os.environ.get('DTSIM_STEP_PAIR', '1').startswith('0')
                     else 'step_pair_kernel')
            kms = launch_ms
            per = args.steps / len(chunks)
            bytes_per_launch = ((MANY_BYTES_PER_ENV + MANY_BYTES_PER_ENV_DECISION * per) * n +
                                MANY_BYTES_PER_RESET * resets / len(chunks))
        elif render is None:
            kname, kms = 'step_kernel', step_ms
            bytes_per_launch = STEP_BYTES_PER_ENV * n + SPAWN_BYTES_PER_RESET * resets / max(
                1.0, decisions / n)
        else:
            from aido1_amd.render import RENDER_BYTES_PER_ENV, RENDER_BYTES_PER_FRESH
            kname, kms = 'render_kernel', render_ms
            # resets per launch = the envs the render refills (fresh = done)
            bytes_per_launch = (RENDER_BYTES_PER_ENV * n + RENDER_BYTES_PER_FRESH * resets /
                                max(1.0, decisions / n))
        achieved = bytes_per_launch / (kms * 1e-3) / 1e9
        line = {
            'metric': METRIC,
            'value': sim_steps / tmax,
            'unit': 'env-steps/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': tmax / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic',
            'config': {
                'workload': ('config2: %d envs/GPU, lane-pose (dist, angle) obs' % n
                             if render is None else
                             'config3: %d envs/GPU, lane-pose + 120x160 top-down render + '
                             'line_detector1 HSV/edge obs' % n),
                'map': args.map, 'envs_per_gpu': n, 'repeat_actions': 3,
                'actions': 'U[0,1)^2 wheel velocities, resident in HBM',
                'auto_reset': True, 'global_envs': n * world,
                'launch': ('dt_step_many: %d decisions per launch' % M if M else
                           'HIP graphs of %d decisions (VecEnv.capture)' % G if G else
                           'one eager launch per decision'),
                'parallelism': 'env shards (%d x %d), no collective' % (world, n)},
            'counts': {'env_steps': sim_steps, 'decisions': decisions, 'resets': resets,
                       'elapsed_s': tmax},
            'roofline': {'bound': 'hbm', 'kernel': kname, 'achieved': achieved,
                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                         'traffic': load_traffic(kname), 'avg_kernel_ms': kms,
                         'algorithmic_bytes_per_launch': bytes_per_launch},
        }
        if render_ms is not None:
            line['step_kernel_ms'] = step_ms
        if M:
            line['roofline']['decisions_per_launch'] = args.steps / len(chunks)
            line['step_ms_per_decision'] = step_ms
        if world == 1 and args.cpu_seconds > 0:
            line['cpu_baseline'] = cpu_baseline(args.cpu_seconds, args.cpu_procs, args.map)
        else:
            line['cpu_baseline'] = None
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


BF16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA (spec)


def bench_actor(args, dev, rank, world, dist):
    """BASELINE configs[3]: 4096 envs/GPU, mixed small_loop/zigzag, actor in the loop."""
    import torch
    from aido1_amd.actor import flops_per_sample
    from aido1_amd.rollout import ActorRollout
    with open(os.path.join(REPO, 'aido1_amd', 'configs', 'reference_config.json')) as f:
        cfg = json.load(f)
    n = args.envs
    torch.manual_seed(args.seed)
    roll = ActorRollout(cfg, n, maps=('small_loop', 'zigzag'), device=dev.index, seed=args.seed,
                        env_id_base=rank * n, actor_mode=args.actor_mode)
    roll.reset()
    for _ in range(args.warmup):
        roll.step()
    torch.cuda.synchronize(dev)
    roll.stats(reset=True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        roll.step(timing=ev[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = roll.stats()
    actor_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    sims = torch.tensor([st['sim_steps'], st['decisions'], st['resets']], dtype=torch.float64,
                        device=dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(sims, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    sim_steps, decisions, resets = (float(v) for v in sims.tolist())
    tmax = float(tmax.item())
    if rank == 0:
        tflops = n * flops_per_sample() / (actor_ms * 1e-3) / 1e12
        print(json.dumps({
            'metric': METRIC, 'value': sim_steps / tmax, 'unit': 'env-steps/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': tmax / args.steps * 1e3,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'f64 env / %s actor' % str(roll.actor.dtype).replace('torch.', ''),
            'data': 'synthetic',
            'config': {'workload': 'config4: %d envs/GPU, actor in the loop (ConfigActor, '
                                   'config.json), mixed small_loop/zigzag' % n,
                       'actor_mode': args.actor_mode, 'envs_per_gpu': n, 'global_envs': n * world, 'repeat_actions': 3,
                       'weights': 'random init (no checkpoint offline)',
                       'parallelism': 'env shards (%d x %d), no collective' % (world, n)},
            'counts': {'env_steps': sim_steps, 'decisions': decisions, 'resets': resets,
                       'elapsed_s': tmax},
            'roofline': {'bound': 'mfma', 'kernel': 'actor forward (fp16 MFMA convs + linears)',
                         'achieved': tflops, 'peak': BF16_DENSE_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': tflops / BF16_DENSE_PEAK_TFLOPS, 'traffic': None,
                         'avg_kernel_ms': actor_ms,
                         'algorithmic_flops_per_launch': n * flops_per_sample()},
            'cpu_baseline': None}), flush=True)
    roll.close()
    if world > 1:
        dist.destroy_process_group()


def bench_train(args, dev, rank, world, dist):
    """BASELINE configs[4]: full DDPG on every GPU — actor-in-loop rollout of
    4096 envs, GPU prioritized replay, one update per decision, gradients
    all-reduced over RCCL (world > 1).  value = env-steps/s; updates/s beside."""
    import torch
    from aido1_amd.actor import flops_per_sample
    from aido1_amd.train_loop import TrainLoop
    with open(os.path.join(REPO, 'aido1_amd', 'configs', 'reference_config.json')) as f:
        cfg = json.load(f)
    n = args.envs
    loop = TrainLoop(cfg, n, device=dev.index, seed=args.seed, env_id_base=rank * n,
                     buffer_size=args.buffer_size, batch_size=args.batch_size or None,
                     updates_per_step=args.updates_per_step, actor_mode=args.actor_mode)
    loop.reset()
    for _ in range(max(args.warmup, 2)):
        loop.step()
    torch.cuda.synchronize(dev)
    loop.rollout.stats(reset=True)
    u0 = loop.updates
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        loop.step(timing=ev[k])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = loop.rollout.stats()
    actor_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    sims = torch.tensor([st['sim_steps'], st['decisions'], st['resets'], loop.updates - u0],
                        dtype=torch.float64, device=dev)
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(sims, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    sim_steps, decisions, resets, updates = (float(v) for v in sims.tolist())
    tmax = float(tmax.item())
    if rank == 0:
        tflops = n * flops_per_sample() / (actor_ms * 1e-3) / 1e12
        print(json.dumps({
            'metric': METRIC, 'value': sim_steps / tmax, 'unit': 'env-steps/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': tmax / args.steps * 1e3,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'f64 env / %s actor / f32 update' % str(
                loop.rollout.actor.dtype).replace('torch.', ''), 'data': 'synthetic',
            'config': {'workload': 'config5: %d envs/GPU full DDPG (rollout + GPU prioritized '
                                   'replay + update + grad all-reduce)' % n,
                       'actor_mode': args.actor_mode, 'envs_per_gpu': n,
                       'global_envs': n * world, 'batch_size_per_gpu': loop.batch_size,
                       'buffer_size_per_gpu': args.buffer_size,
                       'updates_per_step': args.updates_per_step,
                       'weights': 'random init (config.json xavier_normal)',
                       'parallelism': 'env shards (%d x %d) + data-parallel update, RCCL '
                                      'all-reduce of %d gradients' % (
                                          world, n, sum(p.numel() for p in
                                                        loop.trainer.actor.parameters()) +
                                          sum(p.numel() for p in
                                              loop.trainer.critic.parameters()))},
            'counts': {'env_steps': sim_steps, 'decisions': decisions, 'resets': resets,
                       'updates_all_ranks': updates, 'elapsed_s': tmax,
                       'synchronous_updates_per_s': args.steps / tmax,
                       'samples_per_s': loop.batch_size * updates / tmax},
            'roofline': {'bound': 'mfma', 'kernel': 'actor forward (fp16 MFMA convs + linears)',
                         'achieved': tflops, 'peak': BF16_DENSE_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': tflops / BF16_DENSE_PEAK_TFLOPS, 'traffic': None,
                         'avg_kernel_ms': actor_ms,
                         'algorithmic_flops_per_launch': n * flops_per_sample()},
            'cpu_baseline': None}), flush=True)
    loop.rollout.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
