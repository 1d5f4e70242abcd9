"""Checkpoints in the reference's layout (models/ddpg/model.py:130-152):
<directory>/episode_<n>_reward_<r:.2f>/ holding config.json,
actor_state_dict.pth and critic_state_dict.pth, the networks' state_dicts
with the reference's key names (actor.ConfigActor / ConfigCritic), saved as
contiguous CPU tensors so the reference's DDPG.load reads them unchanged and
these load into the reference's modules.  Loading uses torch.load with
weights_only=True (nothing in the file is executed)."""
import json
import os

import torch

ACTOR_FILE = 'actor_state_dict.pth'
CRITIC_FILE = 'critic_state_dict.pth'


def episode_dir(directory, episode, reward):
    """The reference's '{}/episode_{}_reward_{:.2f}' (model.py:131)."""
    return '{}/episode_{}_reward_{:.2f}'.format(directory, episode, reward)


def _cpu_state(module):
    return {k: v.detach().to('cpu').contiguous() for k, v in module.state_dict().items()}


def save_weights(target_dir, actor, critic):
    """model.py:142-144."""
    os.makedirs(target_dir, exist_ok=True)
    torch.save(_cpu_state(actor), os.path.join(target_dir, ACTOR_FILE))
    torch.save(_cpu_state(critic), os.path.join(target_dir, CRITIC_FILE))


def save(config, directory, episode, reward, actor, critic):
    """DDPG.save (model.py:130-140): the episode directory, config.json and
    both state_dicts.  Returns the episode directory."""
    d = episode_dir(directory, episode, reward)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, 'config.json'), 'w') as f:
        json.dump(config, f)
    save_weights(d, actor, critic)
    return d


def load(directory, actor, critic):
    """DDPG.load (model.py:150-152), with the safe loader."""
    for module, name in ((actor, ACTOR_FILE), (critic, CRITIC_FILE)):
        state = torch.load(os.path.join(directory, name), map_location='cpu', weights_only=True)
        module.load_state_dict(state)
