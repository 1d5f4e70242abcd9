"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's prioritized
replay (tests/ and bench.py's cpu leg may import this; the product path never
does).  Pinned by tests/golden/prioritized_replay.json, which was produced by
running the reference's own PrioritizedReplayBuffer (tests/golden/make_golden.py).

Follows:
  utils/segment_tree.py:3-91   SegmentTree (2*capacity array, node 1 = root,
                               leaf i at capacity+i; __setitem__ recomputes
                               the path to the root; reduce() recursion)
  utils/segment_tree.py:94-132 SumSegmentTree.sum / find_prefixsum_idx
  utils/segment_tree.py:135-146 MinSegmentTree.min
  utils/buffers.py:140-259     PrioritizedReplayBuffer (add, _sample_proportional,
                               sample weights, update_priorities)
Quirk kept: _sample_proportional scales by sum(0, len - 1), which (reduce's
end -= 1) covers leaves 0 .. len-2 only (buffers.py:180, segment_tree.py:74-76).
"""
import math


class SegmentTreeRef:
    def __init__(self, capacity, op, neutral):
        assert capacity > 0 and capacity & (capacity - 1) == 0
        self.capacity = capacity
        self.value = [neutral] * (2 * capacity)
        self.op = op

    def _reduce(self, start, end, node, ns, ne):           # segment_tree.py:37-50
        if start == ns and end == ne:
            return self.value[node]
        mid = (ns + ne) // 2
        if end <= mid:
            return self._reduce(start, end, 2 * node, ns, mid)
        if mid + 1 <= start:
            return self._reduce(start, end, 2 * node + 1, mid + 1, ne)
        return self.op(self._reduce(start, mid, 2 * node, ns, mid),
                       self._reduce(mid + 1, end, 2 * node + 1, mid + 1, ne))

    def reduce(self, start=0, end=None):                     # segment_tree.py:52-74
        if end is None:
            end = self.capacity
        if end < 0:
            end += self.capacity
        end -= 1
        return self._reduce(start, end, 1, 0, self.capacity - 1)

    def __setitem__(self, idx, val):                         # segment_tree.py:77-87
        idx += self.capacity
        self.value[idx] = val
        idx //= 2
        while idx >= 1:
            self.value[idx] = self.op(self.value[2 * idx], self.value[2 * idx + 1])
            idx //= 2

    def __getitem__(self, idx):
        return self.value[self.capacity + idx]

    def find_prefixsum_idx(self, prefixsum):                 # segment_tree.py:106-132
        idx = 1
        while idx < self.capacity:
            if self.value[2 * idx] > prefixsum:
                idx = 2 * idx
            else:
                prefixsum -= self.value[2 * idx]
                idx = 2 * idx + 1
        return idx - self.capacity


def sum_tree(capacity):
    return SegmentTreeRef(capacity, lambda a, b: a + b, 0.0)


def min_tree(capacity):
    return SegmentTreeRef(capacity, min, float('inf'))


class PrioritizedReplayRef:
    """Index bookkeeping of PrioritizedReplayBuffer (the payload is the caller's)."""

    def __init__(self, size, alpha):
        assert alpha > 0
        self.size, self.alpha = size, alpha
        cap = 1
        while cap < size:
            cap *= 2
        self.capacity = cap
        self.it_sum, self.it_min = sum_tree(cap), min_tree(cap)
        self.max_priority = 1.0
        self.next_idx = 0
        self.len = 0

    def add(self, n=1):
        """n sequential add() calls; returns the slot each one wrote."""
        slots = []
        for _ in range(n):
            idx = self.next_idx
            self.len = min(self.len + 1, self.size)
            self.next_idx = (self.next_idx + 1) % self.size
            self.it_sum[idx] = self.max_priority ** self.alpha
            self.it_min[idx] = self.max_priority ** self.alpha
            slots.append(idx)
        return slots

    def sample(self, us, beta):
        assert beta > 0
        idxes = []
        for u in us:
            mass = u * self.it_sum.reduce(0, self.len - 1)
            idxes.append(self.it_sum.find_prefixsum_idx(mass))
        total = self.it_sum.reduce()
        p_min = self.it_min.reduce() / total
        max_weight = (p_min * self.len) ** (-beta)
        weights = [((self.it_sum[i] / total) * self.len) ** (-beta) / max_weight for i in idxes]
        return idxes, weights

    def update_priorities(self, idxes, priorities):
        for idx, p in zip(idxes, priorities):
            assert p > 0 and 0 <= idx < self.len
            self.it_sum[idx] = p ** self.alpha
            self.it_min[idx] = p ** self.alpha
            self.max_priority = max(self.max_priority, p)


def uniform_indices(us, length):
    """ReplayBuffer.sample's random.randint(0, len - 1) (buffers.py:136) driven
    by uniforms u in [0, 1): floor(u * len)."""
    return [min(int(math.floor(u * length)), length - 1) for u in us]
