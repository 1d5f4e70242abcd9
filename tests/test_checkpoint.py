"""Checkpoints in the reference's layout (models/ddpg/model.py:130-152,
aido1_amd/checkpoint.py): the episode directory name, config.json, the two
state_dict files with the reference's keys, a round trip through the safe
loader, and DDPGTrainer.save / load (the exploiters' target networks,
training/explorers.py:104-105, 142-152)."""
import json
import os

import torch

from conftest import golden
from test_trainer import make_trainer

from aido1_amd import checkpoint
from aido1_amd.actor import ConfigActor, ConfigCritic


def _nets(seed):
    cfg = golden('reference_config.json')
    torch.manual_seed(seed)
    return cfg, ConfigActor(cfg['model']['actor']), ConfigCritic(cfg['model']['critic'])


def _same(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    return sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sa)


def test_layout_and_round_trip(tmp_path):
    cfg, actor, critic = _nets(1)
    d = checkpoint.save(cfg, str(tmp_path), 150, 12.3456, actor, critic)
    assert d == '{}/episode_150_reward_12.35'.format(tmp_path)          # model.py:131
    assert sorted(os.listdir(d)) == ['actor_state_dict.pth', 'config.json',
                                     'critic_state_dict.pth']
    assert json.load(open(os.path.join(d, 'config.json'))) == cfg
    # the reference's keys (MetaNet paths), plain CPU tensors
    state = torch.load(os.path.join(d, 'actor_state_dict.pth'), weights_only=True)
    assert 'net.input_nets.0.internal_modules.0.kernel.weight' in state
    assert all(v.device.type == 'cpu' and v.is_contiguous() for v in state.values())
    _, actor2, critic2 = _nets(2)
    assert not _same(actor, actor2)
    checkpoint.load(d, actor2, critic2)
    assert _same(actor, actor2) and _same(critic, critic2)


def test_trainer_saves_target_networks(tmp_path):
    tr = make_trainer('cpu')
    with torch.no_grad():                      # targets differ from the online nets
        for p in tr.target_actor.parameters():
            p.add_(0.5)
    d = tr.save(str(tmp_path), 3, -1.0)
    _, actor, critic = _nets(3)
    checkpoint.load(d, actor, critic)
    assert _same(actor, tr.target_actor) and _same(critic, tr.target_critic)
    assert not _same(actor, tr.actor)
    tr2 = make_trainer('cpu')
    tr2.load(d)
    for a, b in ((tr2.actor, tr.target_actor), (tr2.target_actor, tr.target_actor),
                 (tr2.critic, tr.target_critic)):
        assert _same(a, b)
