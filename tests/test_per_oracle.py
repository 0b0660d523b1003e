"""CPU checks of the PER restatement (oracle/per.py; parity unpinned — no reference buffer):
Philox4x32-10 against the Random123 known-answer vectors, the sum-tree against cumulative
sums, the stratified sampler against inverse-CDF lookups, and the FIFO insertion arc."""
import numpy as np

from oracle.per import SumTree, philox4x32_10


def test_philox_known_answers():
    kat = [([0, 0, 0, 0], (0, 0), [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
           ([0xFFFFFFFF] * 4, (0xFFFFFFFF, 0xFFFFFFFF), [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
           ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], (0xA4093822, 0x299F31D0),
            [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1])]
    for ctr, key, out in kat:
        assert philox4x32_10(np.array([ctr], np.uint64), key)[0].tolist() == out


def test_tree_nodes_are_subtree_sums():
    rng = np.random.default_rng(0)
    leaves = rng.uniform(size=256)
    t = SumTree.build(leaves)
    assert np.isclose(t[1], leaves.sum(), rtol=1e-14)
    assert np.isclose(t[2], leaves[:128].sum(), rtol=1e-14)
    assert np.array_equal(t[1:256], t[2:512:2] + t[3:512:2])


def test_sampler_is_inverse_cdf():
    rng = np.random.default_rng(1)
    s = SumTree(300)
    leaves = np.zeros(s.pow2)
    leaves[:300] = rng.uniform(size=300)
    s.tree = SumTree.build(leaves)
    idx, w = s.sample(7, 3, 64, 0.4, 300)
    # stratified: draw b lies in the b-th of 64 equal mass segments -> indices are sorted
    assert np.all(np.diff(idx) >= 0)
    cdf = np.cumsum(leaves[:300])
    lo = np.concatenate([[0.0], cdf[:-1]])
    seg = s.tree[1] / 64
    for b, i in enumerate(idx):
        assert lo[i] <= (b + 1) * seg + 1e-9 and cdf[i] >= b * seg - 1e-9
    assert w.max() == np.float32(1.0)


def test_fifo_arc_and_last_write_wins():
    s = SumTree(10)
    s.set_new([0, 0, 0, 0], [7, 7, 7, 7])
    assert (s.tree[s.pow2:s.pow2 + 7] == 1.0).all() and (s.tree[s.pow2 + 7:] == 0).all()
    s.update([3, 3], [2.0, 5.0], alpha=1.0, eps=0.0)
    assert s.tree[s.pow2 + 3] == 5.0 and s.max_prio == 5.0
    s.set_new([7, 7, 7, 7], [2, 10, 12, 5])  # wraps: rows 7, 8, 9, 0, 1
    rows = s.tree[s.pow2:s.pow2 + 10]
    assert rows.tolist() == [5.0, 5.0, 1.0, 5.0, 1.0, 1.0, 1.0, 5.0, 5.0, 5.0]
