"""VecEnv — N Duckietown environments resident on one MI355X.

Replaces N copies of the reference's per-process stack

    Simulator (gym-duckietown, built by duckietown_rl/env.py:4-20)
      -> DuckietownEnvironmentWrapper (utils/env_wrappers.py:103-134)
      -> EnvironmentWrapper.step/reset (utils/env_wrappers.py:182-253)

with one handle of libdtsim.so: pose state lives in HBM, ``step`` is one kernel
launch that runs ``repeat_actions`` Simulator steps + reward shaping for every
env (and, with ``auto_reset``, the rejection-sampled respawn of finished envs,
gym VectorEnv semantics).  I/O are torch tensors on the env's GPU; the kernels
run on torch's current stream, so VecEnv.step can be captured in a
torch.cuda.CUDAGraph (HIP graph).
"""
import ctypes

import numpy as np
import torch

from aido1_amd import _lib
from aido1_amd.config import EnvConfig
from aido1_amd.maps import load_map

_NULL = ctypes.c_void_p(0)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else _NULL


class StepOutput:
    """Preallocated device outputs of one VecEnv.step (reused every call)."""

    def __init__(self, n, device, lanepos=True, tile=True, obs=True):
        kw = dict(device=device)
        self.reward = torch.zeros(n, dtype=torch.float64, **kw)
        self.reward_mod = torch.zeros(n, dtype=torch.float64, **kw)
        self.done = torch.zeros(n, dtype=torch.uint8, **kw)
        self.obs = torch.zeros(n, 2, dtype=torch.float32, **kw) if obs else None
        self.lanepos = torch.zeros(n, 4, dtype=torch.float64, **kw) if lanepos else None
        self.tile = torch.zeros(n, dtype=torch.int32, **kw) if tile else None


class VecEnv:
    """Batched Simulator + EnvironmentWrapper on one GPU.

    Args:
      n_envs: environments in this handle (4096 in the BASELINE configs).
      map_name: a map in aido1_amd/maps (loop_empty = duckietown_rl/env.py:9).
      seed: Philox key of every env's spawn stream (Simulator(seed=123), env.py:8).
      device: GPU index (torch numbering).
      config: EnvConfig; defaults reproduce launch_env() + config.json's wrapper.
      env_id_base: global id of env 0 (multi-GPU sharding: rank * n_envs), so
        shards draw disjoint spawn streams.
    """

    def __init__(self, n_envs, map_name=None, seed=123, device=None, config=None,
                 env_id_base=0):
        self.config = config or EnvConfig()
        if map_name is not None:
            self.config = self.config.replace(map_name=map_name)
        if device is None:
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        self.device = torch.device('cuda', device)
        self.n = int(n_envs)
        self.map = load_map(self.config.map_name, self.config.road_tile_size)
        self.env_id_base = int(env_id_base)
        self._L = _lib.lib()
        cfg = self.config.to_c()
        self._kind = np.ascontiguousarray(self.map.kind, np.int8)
        self._curves = np.ascontiguousarray(self.map.curves, np.float64)
        self._headings = np.ascontiguousarray(self.map.headings, np.float64)
        self._curve_start = np.ascontiguousarray(self.map.curve_start, np.int32)
        self._objects = np.ascontiguousarray(self.map.object_table, np.float64)
        self._spawn_objects = np.ascontiguousarray(self.map.spawn_table, np.float64)
        m = _lib.DtMap(self.map.width, self.map.height,
                       self._kind.ctypes.data_as(ctypes.c_void_p),
                       self._curve_start.ctypes.data_as(ctypes.c_void_p),
                       self._curves.ctypes.data_as(ctypes.c_void_p),
                       self._headings.ctypes.data_as(ctypes.c_void_p),
                       len(self._objects), self._objects.ctypes.data_as(ctypes.c_void_p),
                       len(self._spawn_objects),
                       self._spawn_objects.ctypes.data_as(ctypes.c_void_p))
        h = ctypes.c_void_p()
        rc = self._L.dt_create(ctypes.byref(cfg), ctypes.byref(m), ctypes.c_uint64(seed),
                               self.n, device, ctypes.byref(h))
        _lib.check(self._L, None, rc, 'dt_create')
        self._h = h
        self.seed(seed)
        self.out = StepOutput(self.n, self.device)
        self._reset_obs = torch.zeros(self.n, 2, dtype=torch.float32, device=self.device)

    # ---- helpers --------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check(self, rc, what):
        _lib.check(self._L, self._h, rc, what)

    def close(self):
        if getattr(self, '_h', None):
            torch.cuda.synchronize(self.device)
            self._L.dt_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- seeding (Simulator.seed / change_model) ----------------------------------
    def seed(self, seed=None, seeds=None):
        """All envs keyed by `seed`, or per-env `seeds` (len n); episode counters
        restart at 0 (utils/env_wrappers.py:126-130)."""
        arr = None
        if seeds is not None:
            arr = np.ascontiguousarray(np.asarray(seeds, np.uint64))
            assert arr.shape == (self.n,)
        rc = self._L.dt_seed(self._h, arr.ctypes.data_as(ctypes.c_void_p) if arr is not None
                             else _NULL, ctypes.c_uint64(int(seed or 0)),
                             ctypes.c_uint32(self.env_id_base))
        self._check(rc, 'dt_seed')

    # ---- hot path ----------------------------------------------------------------------
    def seed_env(self, env, seed):
        """Re-seed one env (its episode counter restarts); the others are untouched."""
        self._check(self._L.dt_seed_env(self._h, int(env), int(seed) & 0xFFFFFFFFFFFFFFFF),
                    'dt_seed_env')

    def reset(self, mask=None):
        """Simulator.reset for every env (or the envs where mask != 0); returns the
        (dist, angle_rad) lane observation [n,2] f32."""
        if mask is not None:
            mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        self._check(self._L.dt_reset(self._h, _ptr(mask), self._stream()), 'dt_reset')
        lp = self.lane_pos()[0]
        self._reset_obs.copy_(torch.stack([lp[:, 0], lp[:, 3]], 1).nan_to_num(0.0).float())
        return self._reset_obs

    def step_into(self, actions, out=None, mask=None):
        """Launch one EnvironmentWrapper.step for all envs into `out` (no sync);
        with `mask` (device [n] u8), only the envs where it is nonzero step — the
        others keep their state and their entries of `out`."""
        out = out or self.out
        if actions.dtype != torch.float32 or not actions.is_contiguous() or \
                actions.device != self.device or tuple(actions.shape) != (self.n, 2):
            raise ValueError('actions must be a contiguous float32 [%d,2] tensor on %s'
                             % (self.n, self.device))
        if mask is None:
            rc = self._L.dt_step(self._h, _ptr(actions), _ptr(out.reward), _ptr(out.reward_mod),
                                 _ptr(out.done), _ptr(out.obs), _ptr(out.lanepos),
                                 _ptr(out.tile), self._stream())
        else:
            if mask.dtype != torch.uint8 or mask.device != self.device or \
                    tuple(mask.shape) != (self.n,) or not mask.is_contiguous():
                raise ValueError('mask must be a contiguous uint8 [%d] tensor on %s'
                                 % (self.n, self.device))
            rc = self._L.dt_step_masked(self._h, _ptr(mask), _ptr(actions), _ptr(out.reward),
                                        _ptr(out.reward_mod), _ptr(out.done), _ptr(out.obs),
                                        _ptr(out.lanepos), _ptr(out.tile), self._stream())
        self._check(rc, 'dt_step')
        return out

    def _check_many(self, actions, out, pose):
        k = int(actions.shape[0]) if actions.dim() == 3 else 0
        if actions.dtype != torch.float32 or not actions.is_contiguous() or \
                actions.device != self.device or k < 1 or tuple(actions.shape[1:]) != (self.n, 2):
            raise ValueError('actions must be a contiguous float32 [k,%d,2] tensor on %s'
                             % (self.n, self.device))
        if out.reward.numel() != k * self.n or (out.obs is not None and
                                                out.obs.shape[0] != k * self.n):
            raise ValueError('out must be a StepOutput of k * n = %d entries' % (k * self.n))
        if pose is not None and (pose.dtype != torch.float64 or not pose.is_contiguous() or
                                 tuple(pose.shape) != (k, 3, self.n) or
                                 pose.device != self.device):
            raise ValueError('pose must be a contiguous float64 [k, 3, %d] tensor on %s'
                             % (self.n, self.device))
        return k

    def step_many_into(self, actions, out, pose=None):
        """k decisions in one launch (dt_step_many): actions [k, n, 2] f32 on the
        device, out a StepOutput(k * n, ...) whose entries of decision d are at
        [d * n:(d + 1) * n] (view them as [k, n]); lanepos/tile are not
        produced.  pose: optional [k, 3, n] f64, each decision's end pose (what
        a render of that decision draws: render_into(..., pose=pose[d])).
        Same results as k step_into calls."""
        k = self._check_many(actions, out, pose)
        self._check(self._L.dt_step_many(self._h, k, _ptr(actions), _ptr(out.reward),
                                         _ptr(out.reward_mod), _ptr(out.done), _ptr(out.obs),
                                         _ptr(pose), self._stream()), 'dt_step_many')
        return out

    def bind_step_many(self, actions, out, pose=None, stream=None):
        """A zero-argument callable that launches step_many_into(actions, out,
        pose) on `stream` (default: the current stream) with its ctypes
        arguments built once (checked here): the launch then costs one foreign
        call, for timed loops.  The callable returns dt_step_many's status
        (0 = DT_OK)."""
        k = self._check_many(actions, out, pose)
        fn = self._L.dt_step_many
        st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else self._stream()
        args = (self._h, k, _ptr(actions), _ptr(out.reward), _ptr(out.reward_mod),
                _ptr(out.done), _ptr(out.obs), _ptr(pose), st)
        keep = (actions, out, pose, stream)

        def launch():
            keep  # noqa: B018 (the tensors stay alive with the callable)
            return fn(*args)
        return launch

    def bind_step(self, actions, out, stream):
        """A zero-argument callable that launches step_into(actions, out) on
        `stream` (a torch.cuda.Stream) with its ctypes arguments built and
        checked once, for timed loops (one foreign call per launch).  Returns
        dt_step's status."""
        if actions.dtype != torch.float32 or not actions.is_contiguous() or \
                actions.device != self.device or tuple(actions.shape) != (self.n, 2):
            raise ValueError('actions must be a contiguous float32 [%d,2] tensor on %s'
                             % (self.n, self.device))
        fn = self._L.dt_step
        args = (self._h, _ptr(actions), _ptr(out.reward), _ptr(out.reward_mod), _ptr(out.done),
                _ptr(out.obs), _ptr(out.lanepos), _ptr(out.tile),
                ctypes.c_void_p(stream.cuda_stream))
        keep = (actions, out, stream)

        def launch():
            keep  # noqa: B018 (the tensors stay alive with the callable)
            return fn(*args)
        return launch

    def bind_copy_pose(self, pose, stream):
        """A zero-argument callable for copy_pose(pose) on `stream`."""
        if pose.dtype != torch.float64 or not pose.is_contiguous() or \
                tuple(pose.shape) != (3, self.n) or pose.device != self.device:
            raise ValueError('pose must be a contiguous float64 [3, %d] tensor on %s'
                             % (self.n, self.device))
        fn = self._L.dt_copy_pose
        args = (self._h, _ptr(pose), ctypes.c_void_p(stream.cuda_stream))
        keep = (pose, stream)

        def launch():
            keep  # noqa: B018
            return fn(*args)
        return launch

    def capture(self, actions, out=None, render=None):
        """StepGraph of len(actions) consecutive decisions (see StepGraph)."""
        return StepGraph(self, actions, out or self.out, render)

    def step(self, actions):
        """Returns (obs [n,2] f32, (reward [n] f64, reward_mod [n] f64), done [n] bool,
        info) — the EnvironmentWrapper.step tuple, batched."""
        if not torch.is_tensor(actions):
            actions = torch.as_tensor(np.asarray(actions, np.float32))
        actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        out = self.step_into(actions)
        info = {'lanepos': out.lanepos, 'tile': out.tile}
        return out.obs, (out.reward, out.reward_mod), out.done.bool(), info

    def lane_pos(self):
        lp = torch.empty(self.n, 4, dtype=torch.float64, device=self.device)
        tile = torch.empty(self.n, dtype=torch.int32, device=self.device)
        self._check(self._L.dt_lane_pos(self._h, _ptr(lp), _ptr(tile), self._stream()),
                    'dt_lane_pos')
        return lp, tile

    # ---- observation path (config 3) ----------------------------------------------------
    def render_into(self, out, fresh=None, pose=None, list_cap=0):
        """Top-down raster + grey + line masks of every env's current pose (or of a
        copy_pose snapshot) into a RenderOutput (see aido1_amd/render.py)."""
        from aido1_amd.render import render_into
        return render_into(self, out, fresh, pose, list_cap)

    def copy_pose(self, pose):
        """Enqueue a copy of every env's (x, z, angle) into pose, a contiguous
        float64 [3, n] device tensor (dt_copy_pose): the render of this decision
        reads the snapshot while the next step runs on another stream."""
        if pose.dtype != torch.float64 or not pose.is_contiguous() or \
                tuple(pose.shape) != (3, self.n) or pose.device != self.device:
            raise ValueError('pose must be a contiguous float64 [3, %d] tensor on %s'
                             % (self.n, self.device))
        self._check(self._L.dt_copy_pose(self._h, _ptr(pose), self._stream()), 'dt_copy_pose')
        return pose

    def render_order(self):
        """(launches, cost [n] u32 shader cycles, order [n] i32): dt_render's
        dispatch order state (diagnostics; synchronises)."""
        launches = ctypes.c_uint32(0)
        cost = np.zeros(self.n, np.uint32)
        order = np.zeros(self.n, np.int32)
        self._check(self._L.dt_render_order(self._h, ctypes.byref(launches),
                                            cost.ctypes.data_as(ctypes.c_void_p),
                                            order.ctypes.data_as(ctypes.c_void_p)),
                    'dt_render_order')
        return launches.value, cost, order

    def set_line_params(self, params):
        self._check(self._L.dt_set_line_params(self._h, ctypes.byref(params)),
                    'dt_set_line_params')

    def stats(self, reset=False):
        """{'sim_steps', 'decisions', 'resets', 'episodes'} counted on the device."""
        o = (ctypes.c_uint64 * 4)()
        self._check(self._L.dt_stats(self._h, o, int(reset)), 'dt_stats')
        return dict(zip(('sim_steps', 'decisions', 'resets', 'episodes'), list(o)))

    def check(self):
        """Synchronise and raise if a kernel flagged an error (e.g. spawn exhausted)."""
        f = ctypes.c_uint32(0)
        self._check(self._L.dt_check(self._h, ctypes.byref(f)), 'dt_check')
        return f.value

    # ---- state access (parity tests) --------------------------------------------------
    def get_state(self):
        n = self.n
        s = {k: np.zeros(n, np.float64) for k in ('x', 'z', 'angle')}
        s.update({k: np.zeros(n, np.uint32) for k in ('step_count', 'env_step', 'episode')})
        p = [s[k].ctypes.data_as(ctypes.c_void_p) for k in
             ('x', 'z', 'angle', 'step_count', 'env_step', 'episode')]
        self._check(self._L.dt_get_state(self._h, *p), 'dt_get_state')
        return s

    def set_state(self, **kw):
        keys = ('x', 'z', 'angle', 'step_count', 'env_step', 'episode')
        arrs = []
        for k in keys:
            if k in kw and kw[k] is not None:
                dt = np.float64 if k in ('x', 'z', 'angle') else np.uint32
                a = np.ascontiguousarray(np.asarray(kw[k], dt))
                assert a.shape == (self.n,), (k, a.shape)
                arrs.append(a)
            else:
                arrs.append(None)
        p = [a.ctypes.data_as(ctypes.c_void_p) if a is not None else _NULL for a in arrs]
        self._check(self._L.dt_set_state(self._h, *p), 'dt_set_state')


class StepGraph:
    """k consecutive VecEnv.step launches (plus, optionally, the render of each
    decision) captured once into a HIP graph and replayed as one launch.

    The reference steps one Simulator per Python call; here a decision of all
    envs is one kernel of ~25 us, so an eager loop is bound by the host's
    per-call cost.  A graph issues the k kernels back to back with no host in
    between.  Each launch reads its own slice actions[i] ([k, n, 2] f32 on the
    env's device; the caller refills it between replays), writes `out`, and the
    env state advances exactly as k eager step_into calls would (the auto-reset
    spawn-ahead path is graph-safe: tests/test_gpu_step.py).  With `render`, k
    must be a multiple of the ring's slot count so that the slots baked into the
    graph continue the ring's order on every replay.
    """

    def __init__(self, env, actions, out, render=None):
        if actions.dim() != 3 or tuple(actions.shape[1:]) != (env.n, 2):
            raise ValueError('actions must be [k, %d, 2]' % env.n)
        self.k = int(actions.shape[0])
        if render is not None and self.k % render.slots:
            raise ValueError('k (%d) must be a multiple of the ring slots (%d)'
                             % (self.k, render.slots))
        self.env, self.actions, self.out, self.render = env, actions, out, render
        torch.cuda.synchronize(env.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for i in range(self.k):
                env.step_into(actions[i], out)
                if render is not None:
                    env.render_into(render, fresh=out.done)

    def replay(self):
        self.graph.replay()
