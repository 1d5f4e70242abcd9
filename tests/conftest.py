import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, 'tests', 'golden')
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU; run with -m gpu')
    config.addinivalue_line('markers', 'slow: long-running')


def golden(name):
    path = os.path.join(GOLDEN, name)
    if name.endswith('.json'):
        with open(path) as f:
            return json.load(f)
    return np.load(path, allow_pickle=False)


def map_rows(name):
    import yaml
    with open(os.path.join(REPO, 'aido1_amd', 'maps', name + '.yaml')) as f:
        return yaml.safe_load(f)['tiles']


def map_objects(name):
    """The map file's `objects` list (static objects)."""
    import yaml
    with open(os.path.join(REPO, 'aido1_amd', 'maps', name + '.yaml')) as f:
        return yaml.safe_load(f).get('objects') or []


@pytest.fixture(scope='session')
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU test selected but no GPU is visible (run -m "not gpu" on CPU boxes)')
    return torch.device('cuda', 0)
