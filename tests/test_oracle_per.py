"""The prioritized-replay oracle against the reference's own PrioritizedReplayBuffer
(tests/golden/prioritized_replay.json) and segment trees (segment_tree.json)."""
import math

from conftest import golden
from oracle.per_ref import PrioritizedReplayRef, min_tree, sum_tree, uniform_indices


def _tree(vals):
    return [math.inf if v is None else v for v in vals]


def test_per_oracle_matches_reference_buffer():
    for case in golden('prioritized_replay.json'):
        ref = PrioritizedReplayRef(case['size'], case['alpha'])
        assert ref.capacity == case['capacity']
        stored = {}
        for op in case['ops']:
            for slot, item in zip(ref.add(len(op['add'])), op['add']):
                stored[slot] = item
            if 'sample' in op:
                s = op['sample']
                idx, w = ref.sample(s['u'], s['beta'])
                assert idx == s['idx']
                assert w == s['weights']                     # same float ops: exact
                assert [stored[i] for i in idx] == s['obs']  # slot -> payload mapping
                ref.update_priorities(op['update']['idx'], op['update']['priorities'])
            assert ref.len == op['len'] and ref.next_idx == op['next_idx']
            assert ref.max_priority == op['max_priority']
            assert ref.it_sum.value == op['sum_tree']
            assert ref.it_min.value == _tree(op['min_tree'])


def test_segment_tree_oracle_matches_reference():
    for case in golden('segment_tree.json'):
        s, m = sum_tree(case['capacity']), min_tree(case['capacity'])
        for op in case['ops']:
            i, v = op['set']
            s[i] = v
            m[i] = v
            a, b = op['range']
            assert s.reduce(a, b) == op['sum']
            assert m.reduce(a, b) == op['min']
            assert s.reduce() == op['total']
            assert s.find_prefixsum_idx(op['prefix']) == op['idx']


def test_uniform_indices():
    assert uniform_indices([0.0, 0.5, 0.999999], 10) == [0, 5, 9]
