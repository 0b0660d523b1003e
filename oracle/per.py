"""CPU ORACLE — test infrastructure only.

NumPy restatement of the prioritized n-step replay (trainer/buffer/prioritized_replay_buffer.py,
csrc/per.hip). **Parity unpinned**: the reference ships no prioritized buffer — its trainer only
calls `buffer.update_batch(idx, new_priority)` after `model_update` returns `(tb, idx, priority)`
(RL/trainer/nstep_off_serial_trainer.py:30,93-95) and the README advertises PER. This oracle
therefore states the published algorithm the engine implements (proportional prioritisation,
Schaul et al., "Prioritized Experience Replay", ICLR 2016, §3.3 + Appendix B.2.1 stratified
sampling) and the engine's own conventions, so the GPU kernels are checked against an independent
sequential restatement:
  * p_i = (|delta_i| + eps)^alpha in float64; a batch naming a leaf twice keeps the LAST entry
    (sequential loop semantics); the running max priority covers every entry of every batch;
  * new windows (the FIFO arc the rollout appended, read from the cursors {ptr, size, total,
    last}) enter with the running max priority (1.0 before any update);
  * sum-tree in heap layout, node k = node 2k + node 2k+1 (one float64 add);
  * draw b of a batch of B: u = (b + U_b) * total / B with U_b the first 32-bit word of
    Philox4x32-10(counter = (b, 9 << 16, draw counter), key = seed) times 2^-32; descend
    (u < left ? left : (u -= left, right)); a leaf at or past `size` is clamped to size - 1;
  * importance weights w_b = (size * p_leaf / total)^-beta / max_b w_b.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """Philox4x32-10 (Salmon et al., SC'11) on uint32 counters `ctr` [..., 4] with key (k0, k1)
    (csrc/philox.h). Vectorised over leading dimensions; returns uint32 [..., 4]."""
    c = [np.asarray(ctr[..., j], np.uint64) for j in range(4)]
    k0, k1 = int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return np.stack([x.astype(np.uint32) for x in c], -1)


def draw_words(seed, units, tick, stream):
    """First-level draw of csrc/philox.h make_rng(seed, unit, tick).draw(stream) for each unit."""
    units = np.asarray(units, np.uint64)
    ctr = np.stack([units & MASK, (units >> np.uint64(32)) ^ np.uint64((stream << 16) & 0xFFFFFFFF),
                    np.full(units.shape, tick & 0xFFFFFFFF, np.uint64),
                    np.full(units.shape, (tick >> 32) & 0xFFFFFFFF, np.uint64)], -1)
    return philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))


class SumTree:
    """Sequential proportional-PER restatement over `capacity` rows (tree = float64 [2 pow2])."""

    def __init__(self, capacity):
        self.capacity = int(capacity)
        pow2 = 1
        while pow2 < self.capacity:
            pow2 <<= 1
        self.pow2 = pow2
        self.tree = np.zeros(2 * pow2, np.float64)
        self.max_prio = 1.0

    @staticmethod
    def build(leaves):
        """Full level-by-level tree from a leaf vector (length a power of two)."""
        pow2 = leaves.size
        tree = np.zeros(2 * pow2, np.float64)
        tree[pow2:] = leaves
        w = pow2 // 2
        while w >= 1:
            tree[w:2 * w] = tree[2 * w:4 * w:2] + tree[2 * w + 1:4 * w:2]
            w //= 2
        return tree

    def _rebuild(self):
        self.tree = self.build(self.tree[self.pow2:].copy())

    def update(self, idx, td, alpha, eps):
        """update_batch(idx, td) (nstep_off_serial_trainer.py:93-95 hook)."""
        a, e = np.float64(np.float32(alpha)), np.float64(np.float32(eps))
        for i, t in zip(np.asarray(idx, np.int64), np.asarray(td, np.float32)):
            if i < 0 or i >= self.pow2:
                continue
            p = (np.float64(abs(t)) + e) ** a
            self.tree[self.pow2 + i] = p
            self.max_prio = max(self.max_prio, p)
        self._rebuild()

    def set_new(self, before, after):
        """Rows appended between two cursor snapshots get the running max priority."""
        cnt = min(int(after[2]) - int(before[2]), self.capacity)
        if cnt <= 0:
            return
        start = (int(after[0]) - cnt) % self.capacity
        rows = (start + np.arange(cnt)) % self.capacity
        self.tree[self.pow2 + rows] = self.max_prio if self.max_prio > 0 else 1.0
        self._rebuild()

    def sample(self, seed, counter, batch, beta, size):
        total = self.tree[1]
        seg = total / np.float64(batch)
        q = draw_words(seed, np.arange(batch), counter, 9)[:, 0]
        u = (np.arange(batch, dtype=np.float64) + q.astype(np.float64) * 2.3283064365386963e-10) * seg
        node = np.ones(batch, np.int64)
        while node[0] < self.pow2:
            left = self.tree[2 * node]
            go_left = u < left
            u = np.where(go_left, u, u - left)
            node = np.where(go_left, 2 * node, 2 * node + 1)
        leaf = node - self.pow2
        leaf = np.where(leaf >= size, max(size - 1, 0), leaf)
        p = self.tree[self.pow2 + leaf] / (total if total > 0 else 1.0)
        wv = (np.float64(max(size, 1)) * np.where(p > 0, p, 1e-300)) ** -np.float64(np.float32(beta))
        mx = wv.max() if wv.max() > 0 else 1.0
        return leaf, (wv / mx).astype(np.float32)
