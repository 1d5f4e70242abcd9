"""Actor in the loop on the GPU: the bf16 BN-folded FusedActor against the fp32
eval-mode actor, ring-order equivalence, and the batched rollout."""
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

sys.path.insert(0, GOLDEN)
from formulas import formula_input, formula_state_dict  # noqa: E402

pytestmark = pytest.mark.gpu


def test_fused_bf16_close_to_fp32(gpu):
    from aido1_amd.actor import ConfigActor, FusedActor
    a = ConfigActor(golden('reference_config.json')['model']['actor'])
    a.load_state_dict(formula_state_dict(a.state_dict()))
    a.eval()
    x = formula_input(4)
    with torch.no_grad():
        ref = a(x)
    f = FusedActor(a, dtype=torch.bfloat16).to(gpu)
    y = f(x.to(gpu)).cpu()
    assert torch.max(torch.abs(y - ref)) < 3e-2, (y, ref)
    assert np.max(np.abs(y.numpy() - golden('actor.npz')['config_actor'])) < 3e-2


def test_rollout_runs_and_counts(gpu):
    from aido1_amd.rollout import ActorRollout
    cfg = golden('reference_config.json')
    roll = ActorRollout(cfg, 512, device=0, seed=3)
    roll.reset()
    for _ in range(10):
        r, rm, d = roll.step()
    torch.cuda.synchronize()
    st = roll.stats()
    assert st['decisions'] == 512 * 10
    assert 512 * 10 <= st['sim_steps'] <= 512 * 30
    assert torch.isfinite(r).all() and torch.isfinite(roll.ring).all()
    a = roll.actions
    assert (a.abs() <= 1.0).all()
    roll.close()
