"""HTTP env-server compatibility: the reference's per-port env
worker protocol served by ONE process holding a batch of envs on the GPU.

The reference runs one ``pyramid_worker.py`` process per env, each wrapping a
``DuckietownEnvironmentWrapper`` (utils/env_wrappers.py:103-134) on its own
port, and its ``VirtualEnvironment`` client (utils/env_wrappers.py:51-100)
POSTs to ``http://host:port/<route>/``:

  /post_step_request/            body: json.dumps({'action': [...]}) sent with
                                 requests' json= (so double-encoded; the worker
                                 json.loads(request.json_body))
                                 -> {'observation', 'reward', 'done', 'info'}
  /post_reset_request/           -> {'observation'}
  /post_change_model_request/    body: json.dumps({'seed': s}) -> {'success': True}
  /post_collect_garbage_request/ -> json.dumps({'success': True}) (a JSON string)

``EnvServer`` listens on ``port_start + i`` for env i of one VecEnv and keeps
those routes, bodies and replies, so the reference's TrainManager "virtual"
mode (config.json ``client.port_tcp_start``) runs against it unchanged.
Requests that arrive together are served together: a dispatcher gathers the
pending ones and runs ONE masked dt_step / dt_reset for all of them, then one
render.  The observation is PreliminaryTransformer's output
(env_utils.py:41-51): rgb2gray of the 120x160 raster in float64, shape
(1, 120, 160), as nested lists (utils/util.py:124-131 from_numpy).

Env semantics are the Simulator's as DuckietownEnvironmentWrapper sees it:
one Simulator step per request (the client-side EnvironmentWrapper owns
repeat_actions, the env-step cap and reward shaping), no auto-reset.
``collect_garbage`` re-creates the env in the reference (launch_env + seed);
here that is re-seeding it, which restarts its spawn stream the same way.
"""
import argparse
import json
import queue
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np

ROUTES = ('post_step_request', 'post_reset_request', 'post_change_model_request',
          'post_collect_garbage_request')
GRAY = np.array([0.2125, 0.7154, 0.0721])   # skimage rgb2gray (env_utils.py:50)


def _numpy_default(o):
    """utils/util.py:124-131 from_numpy for whatever a batch hands back."""
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, np.generic):
        return o.item()
    raise TypeError('not JSON serializable: %r' % type(o))


def _decode(body):
    """The worker's json.loads(request.json_body): accept the client's
    double-encoded body, or a plain JSON object."""
    if not body:
        return {}
    data = json.loads(body)
    if isinstance(data, str):
        data = json.loads(data) if data else {}
    return data if isinstance(data, dict) else {}


class GpuBatch:
    """The batched env behind the server: a VecEnv with Simulator semantics
    plus a 1-slot render (RGB raster) for the observations."""

    def __init__(self, n_envs, map_name='loop_empty', seed=0, device=None, env_id_base=0,
                 max_steps=500001, accept_start_angle_deg=4, frame_skip=1, frame_rate=30):
        import torch
        from aido1_amd.config import EnvConfig
        from aido1_amd.render import RenderOutput
        from aido1_amd.simulator import U32_MAX
        from aido1_amd.vec_env import StepOutput, VecEnv
        cfg = EnvConfig(map_name=map_name, max_steps=max_steps,
                        accept_start_angle_deg=accept_start_angle_deg, frame_skip=frame_skip,
                        frame_rate=frame_rate, repeat_actions=1, max_env_steps=U32_MAX,
                        action_mode='wheels', auto_reset=False)
        self.torch = torch
        self.n = n_envs
        self.env = VecEnv(n_envs, seed=seed, device=device, config=cfg, env_id_base=env_id_base)
        self.dev = self.env.device
        self.out = StepOutput(n_envs, self.dev)
        self.render = RenderOutput(n_envs, self.dev, slots=1, rgb=True, masks=False)
        self.actions = torch.zeros(n_envs, 2, dtype=torch.float32, device=self.dev)
        self.config = cfg

    def seed(self, env, seed):
        self.env.seed_env(env, seed)

    def reset(self, envs):
        m = self.torch.zeros(self.n, dtype=self.torch.uint8)
        m[envs] = 1
        self.env.reset(m.to(self.dev))

    def step(self, envs, actions):
        """actions: [len(envs), 2] float; returns (reward, done, info) per env."""
        t = self.torch
        a = t.zeros(self.n, 2, dtype=t.float32)
        a[envs] = t.as_tensor(np.asarray(actions, np.float64).astype(np.float32))
        m = t.zeros(self.n, dtype=t.uint8)
        m[envs] = 1
        self.actions.copy_(a)
        self.env.step_into(self.actions, self.out, mask=m.to(self.dev))
        rew = self.out.reward.cpu().numpy()
        done = self.out.done.cpu().numpy()
        lp = self.out.lanepos.cpu().numpy()
        tile = self.out.tile.cpu().numpy()
        st = self.env.get_state()
        res = []
        for e in envs:
            info = {'Simulator': {
                'cur_pos': [float(st['x'][e]), 0.0, float(st['z'][e])],
                'cur_angle': float(st['angle'][e]), 'step_count': int(st['step_count'][e]),
                'tile': int(tile[e]),
                'lane_position': None if np.isnan(lp[e]).any() else dict(zip(
                    ('dist', 'dot_dir', 'angle_deg', 'angle_rad'), (float(v) for v in lp[e])))}}
            res.append((float(rew[e]), bool(done[e]), info))
        return res

    def observations(self, envs):
        """PreliminaryTransformer (env_utils.py:48-51) of each env's raster:
        img_as_float(rgb) @ [0.2125, 0.7154, 0.0721], shape (1, 120, 160)."""
        self.render.restart()
        self.env.render_into(self.render)
        rgb = self.render.rgb[envs].cpu().numpy()
        gray = (rgb.astype(np.float64) / 255.0) @ GRAY
        return [g[None].tolist() for g in gray]


class _Request:
    def __init__(self, env, route, data):
        self.env, self.route, self.data = env, route, data
        self.done = threading.Event()
        self.reply = None
        self.error = None


class EnvServer:
    """pyramid_worker.py's routes for env i on port port_start + i."""

    def __init__(self, batch, host='127.0.0.1', port_start=18000, window_s=0.002):
        self.batch = batch
        self.host = host
        self.port_start = port_start
        self.window_s = window_s
        self.q = queue.Queue()
        self.seeds = [None] * batch.n
        self.servers = []
        self.threads = []
        self._stop = threading.Event()

    # ---- HTTP side -----------------------------------------------------------------
    def _handler(self, env):
        server = self

        class Handler(BaseHTTPRequestHandler):
            protocol_version = 'HTTP/1.1'

            def log_message(self, *args):
                pass

            def do_POST(self):
                route = self.path.strip('/')
                n = int(self.headers.get('Content-Length') or 0)
                body = self.rfile.read(n).decode() if n else ''
                if route not in ROUTES:
                    self._send(404, {'error': 'unknown route %s' % self.path})
                    return
                try:
                    data = _decode(body)
                except ValueError as ex:
                    self._send(400, {'error': str(ex)})
                    return
                req = _Request(env, route, data)
                server.q.put(req)
                req.done.wait()
                if req.error is not None:
                    self._send(500, {'error': req.error})
                else:
                    self._send(200, req.reply)

            def _send(self, code, obj):
                payload = json.dumps(obj, default=_numpy_default).encode()
                self.send_response(code)
                self.send_header('Content-Type', 'application/json')
                self.send_header('Content-Length', str(len(payload)))
                self.end_headers()
                self.wfile.write(payload)

        return Handler

    def start(self):
        for i in range(self.batch.n):
            srv = ThreadingHTTPServer((self.host, self.port_start + i), self._handler(i))
            srv.daemon_threads = True
            t = threading.Thread(target=srv.serve_forever, daemon=True)
            t.start()
            self.servers.append(srv)
            self.threads.append(t)
        d = threading.Thread(target=self._dispatch, daemon=True)
        d.start()
        self.threads.append(d)
        return self

    def stop(self):
        self._stop.set()
        self.q.put(None)
        for srv in self.servers:
            srv.shutdown()
            srv.server_close()

    # ---- batching dispatcher ------------------------------------------------------------
    def _dispatch(self):
        while not self._stop.is_set():
            first = self.q.get()
            if first is None:
                return
            reqs = [first]
            try:   # gather what arrives within the window (one request per env at a time)
                while len(reqs) < self.batch.n:
                    r = self.q.get(timeout=self.window_s)
                    if r is None:
                        self._stop.set()
                        break
                    reqs.append(r)
            except queue.Empty:
                pass
            try:
                self._serve(reqs)
            except Exception as ex:       # reply, never leave a client hanging
                for r in reqs:
                    if not r.done.is_set():
                        r.error = '%s: %s' % (type(ex).__name__, ex)
                        r.done.set()

    def _serve(self, reqs):
        # a client waits for each reply, so an env has at most one request here
        by_route = {rt: [r for r in reqs if r.route == rt] for rt in ROUTES}
        for r in by_route['post_change_model_request']:
            seed = int(r.data.get('seed', 0))
            self.seeds[r.env] = seed
            self.batch.seed(r.env, seed)
            r.reply = {'success': True}
        for r in by_route['post_collect_garbage_request']:
            if self.seeds[r.env] is not None:
                self.batch.seed(r.env, self.seeds[r.env])
            r.reply = json.dumps({'success': True})
        resets = by_route['post_reset_request']
        steps = by_route['post_step_request']
        if resets:
            self.batch.reset([r.env for r in resets])
        results = []
        if steps:
            results = self.batch.step([r.env for r in steps],
                                      [np.asarray(r.data['action'], np.float64).reshape(2)
                                       for r in steps])
        if resets or steps:
            obs = self.batch.observations([r.env for r in resets + steps])
            for r, o in zip(resets, obs[:len(resets)]):
                r.reply = {'observation': o}
            for r, o, (rew, done, info) in zip(steps, obs[len(resets):], results):
                r.reply = {'observation': o, 'reward': rew, 'done': done, 'info': info}
        for r in reqs:
            r.done.set()


def main(argv=None):
    p = argparse.ArgumentParser(description='Batched GPU env server (pyramid_worker.py routes)')
    p.add_argument('--n-envs', type=int, default=8)
    p.add_argument('--host', default='127.0.0.1')
    p.add_argument('--port', type=int, default=18000, help='port of env 0; env i on port + i')
    p.add_argument('--map', default='loop_empty')
    p.add_argument('--device', type=int, default=0)
    p.add_argument('--seed', type=int, default=0)
    a = p.parse_args(argv)
    srv = EnvServer(GpuBatch(a.n_envs, map_name=a.map, seed=a.seed, device=a.device),
                    host=a.host, port_start=a.port).start()
    print('serving %d envs on %s:%d-%d' % (a.n_envs, a.host, a.port, a.port + a.n_envs - 1),
          flush=True)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        srv.stop()


if __name__ == '__main__':
    main()
