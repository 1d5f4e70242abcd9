"""bench.py's N-rank launcher and cross-rank reduction, on CPU over gloo.

`python bench.py --gpus N` must start N ranks itself (torch.distributed.run as
a child, before anything touches a GPU) and rank 0 must report every rank;
`--dry-run` runs that launcher and the same barrier / max / sum / all_gather
as the GPU path with no kernels.  Replaces the reference's process farm
(training/managers.py:113-124) for the bench's purposes."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, env_extra=None, timeout=240):
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py')] + list(args),
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=REPO)
    return r


def last_json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.parametrize('n', [1, 2])
def test_launcher_reports_every_rank(n):
    r = run_bench('--gpus', str(n), '--dry-run', '--envs', '64', '--steps', '3', '--warmup', '1')
    assert r.returncode == 0, r.stderr[-3000:]
    line = last_json(r.stdout)
    assert line['n_gpus'] == n
    assert line['process_group_world'] == n
    assert [p['rank'] for p in line['per_rank']] == list(range(n))
    assert line['config']['global_envs'] == 64 * n
    # value = all ranks' env-steps over the slowest rank's time
    steps = sum(p['env_steps'] for p in line['per_rank'])
    assert steps == 64 * 3 * 3 * n
    tmax = max(p['elapsed_s'] for p in line['per_rank'])
    assert abs(line['value'] - steps / tmax) <= 1e-6 * line['value']


def test_world_size_must_match_gpus():
    r = run_bench('--gpus', '2', '--dry-run', env_extra={'WORLD_SIZE': '1', 'RANK': '0',
                                                         'LOCAL_RANK': '0'})
    assert r.returncode != 0
    assert 'WORLD_SIZE=1 but --gpus 2' in r.stderr


def test_split_even():
    sys.path.insert(0, REPO)
    import bench
    assert bench.split_even(20, 20) == [20]
    assert bench.split_even(20, 16) == [10, 10]
    assert bench.split_even(320, 20) == [20] * 16
    assert bench.split_even(21, 20) == [11, 10]
    assert bench.split_even(5, 20) == [5]
    assert bench.split_even(0, 20) == []
    for total in range(1, 90):
        s = bench.split_even(total, 16)
        assert sum(s) == total and max(s) - min(s) <= 1 and max(s) <= 16
