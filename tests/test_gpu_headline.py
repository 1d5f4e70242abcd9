"""The headline's launch form against the oracle at full size: bench.ObsLoop
in its default 'many' mode (dt_step_many over a chunk of 20 decisions, then
the chunk's renders three decisions a launch, dt_render3 / dt_render2) at
4096 envs on loop_empty, every decision's masks written to its own buffer,
then bench.step_parity: every env's rewards, done flags, lane poses and end
state against oracle/dtsim_oracle.c, and on 1024 envs EVERY decision's four
masks plus the final 3-frame ring against oracle/render_oracle.c renders of
the oracle's poses (features/line_detector1.py:36-61,134-141;
utils/env_wrappers.py:224-248)."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('group', [3, 2])
def test_obsloop_every_decision_matches_oracle(gpu, group):
    import bench
    from aido1_amd.config import EnvConfig
    from aido1_amd.render import RenderOutput
    from aido1_amd.vec_env import StepOutput, VecEnv
    n, K = 4096, 20
    env = VecEnv(n, seed=1234, device=0, config=EnvConfig(map_name='loop_empty'))
    ro = RenderOutput(n, gpu)
    loop = bench.ObsLoop(env, ro, torch, 'many', 20, 1, group=group, keep_masks=K)
    g = torch.Generator(device=gpu).manual_seed(5)
    env.reset()
    warm = torch.rand(5, n, 2, generator=g, device=gpu)
    wout = StepOutput(5 * n, gpu, lanepos=False, tile=False)
    assert loop.run(loop.bind(warm, wout), loop.events(5)) == 0
    torch.cuda.synchronize()
    start = env.get_state()
    actions = torch.rand(K, n, 2, generator=g, device=gpu)
    out = StepOutput(K * n, gpu, lanepos=False, tile=False)
    calls = loop.bind(actions, out)
    assert loop.kept
    assert max(len(la) for la in loop.launches) == group
    assert loop.run(calls, loop.events(K)) == 0
    torch.cuda.synchronize()
    frames = types.SimpleNamespace(slots=ro.slots, stack_view=ro.stack_view,
                                   masks=loop.last_masks, dmasks=loop.dmasks)
    args = types.SimpleNamespace(map='loop_empty', seed=1234, cpu_procs=0)
    rec = bench.step_parity(env, start, actions, out, 0, args, frames=frames, m=1024)
    env.close()
    assert rec['mask_decisions_checked'] == K and rec['frame_envs_checked'] == 1024
    assert rec['mask_mismatches'] == 0 and rec['gray_mismatches'] == 0, rec
    assert rec['done_mismatches'] == 0 and rec['tile_mismatches'] == 0, rec
    assert rec['ok'], rec
