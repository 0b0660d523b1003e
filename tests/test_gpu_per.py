"""Prioritized replay kernels (csrc/per.hip) vs the sequential NumPy restatement (oracle/per.py).

PARITY UNPINNED: the reference ships no prioritized buffer (its trainer only calls
`buffer.update_batch(idx, priority)`, RL/trainer/nstep_off_serial_trainer.py:93-95), so these
tests pin the engine to the published proportional-PER algorithm as restated in oracle/per.py:
sum-tree contents after updates and FIFO insertions (bit-exact), last-write-wins on duplicate
leaves, sampled indices (bit-exact for the same Philox draws), importance weights, proportional
sampling frequencies (chi-square), and config 3 of BASELINE.json (DuctedFan / TwoLink, 65,536
envs, n-step windows + PER) through the trainer.
"""
import os

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from oracle.per import SumTree

pytestmark = pytest.mark.gpu


def _cursor(ptr, size, total, last=0):
    return torch.tensor([ptr, size, total, last], dtype=torch.int64, device="cuda")


class DevTree:
    def __init__(self, capacity):
        self.ref = SumTree(capacity)
        self.cap, self.pow2 = capacity, self.ref.pow2
        self.tree = torch.zeros(2 * self.pow2, dtype=torch.float64, device="cuda")
        self.max_prio = torch.ones(1, dtype=torch.float64, device="cuda")
        self.cur = [0, 0, 0, 0]

    def append(self, cnt):
        before = list(self.cur)
        ptr, size, total, _ = self.cur
        self.cur = [(ptr + cnt) % self.cap, min(size + cnt, self.cap), total + cnt, cnt]
        b, a = _cursor(*before), _cursor(*self.cur)
        N.check(N.lib().mh_per_set_new(N.ptr(self.tree), self.pow2, N.ptr(b), N.ptr(a), self.cap, N.ptr(self.max_prio),
                                       N.stream_of()), "mh_per_set_new")
        self.ref.set_new(before, self.cur)

    def update(self, idx, td, alpha=0.6, eps=1e-6):
        i = torch.as_tensor(np.asarray(idx, np.int64), device="cuda")
        p = torch.as_tensor(np.asarray(td, np.float32), device="cuda")
        N.check(N.lib().mh_per_update(N.ptr(self.tree), self.pow2, N.ptr(i), N.ptr(p), i.numel(), alpha, eps,
                                      N.ptr(self.max_prio), N.stream_of()), "mh_per_update")
        self.ref.update(idx, td, alpha, eps)
        got = self.host()
        # f64 pow: the device's and libm's results may differ in the last ulp
        np.testing.assert_allclose(got[self.pow2:], self.ref.tree[self.pow2:], rtol=2e-15, atol=0)
        np.testing.assert_allclose(float(self.max_prio.item()), self.ref.max_prio, rtol=2e-15)
        # adopt the device's leaves so the structural checks that follow are bit-exact
        self.ref.tree = SumTree.build(got[self.pow2:].copy())
        self.ref.max_prio = float(self.max_prio.item())

    def host(self):
        return self.tree.cpu().numpy()


def _assert_tree_exact(t):
    """Every internal node is exactly the f64 sum of its children (device-side invariant)."""
    pow2 = t.size // 2
    assert np.array_equal(t[1:pow2], t[2:2 * pow2:2] + t[3:2 * pow2:2])


@pytest.mark.parametrize("capacity", [1000, 1024, 100_000, 1 << 17])
def test_fifo_insertion_matches_oracle(capacity):
    """New rows (including arcs that wrap the FIFO and batches larger than the capacity) enter at
    the running max priority; only they change; the tree equals the oracle's bit for bit."""
    rng = np.random.default_rng(capacity)
    d = DevTree(capacity)
    for cnt in (capacity // 3, capacity // 2 + 7, 1, 0, 2 * capacity + 5, capacity // 5):
        d.append(cnt)
        if d.cur[1] > 0:  # raise the running max between appends
            k = 17
            d.update(rng.integers(0, d.cur[1], k), rng.standard_normal(k).astype(np.float32) * (3 + cnt % 11))
        got = d.host()
        _assert_tree_exact(got)
        np.testing.assert_array_equal(got[d.pow2:], d.ref.tree[d.pow2:])
        np.testing.assert_array_equal(got, d.ref.tree)
        assert float(d.max_prio.item()) == d.ref.max_prio
    assert not got[d.pow2 + capacity:].any()  # rows past the capacity never gain mass


@pytest.mark.parametrize("capacity,batch", [(1000, 256), (1 << 20, 256), (50_000, 3000), (4096, 65536)])
def test_update_leaf_to_root_matches_oracle(capacity, batch):
    """update_batch: p = (|td| + eps)^alpha in f64, duplicates keep the last entry, ancestors
    recomputed; the full tree (2 x pow2 nodes) equals the oracle's bit for bit."""
    rng = np.random.default_rng(batch)
    d = DevTree(capacity)
    d.append(capacity)
    for r in range(4):
        idx = rng.integers(0, capacity, batch)
        idx[: batch // 8] = idx[batch // 8: batch // 4]  # forced duplicates at both positions
        td = (rng.standard_normal(batch) * 10 ** rng.uniform(-3, 2, batch)).astype(np.float32)
        d.update(idx, td, alpha=0.6, eps=1e-6)
        got = d.host()  # (leaves vs the oracle's pow: DevTree.update)
        _assert_tree_exact(got)
        # internal nodes from the device's own leaves are bitwise the level-by-level rebuild
        np.testing.assert_array_equal(got, SumTree.build(got[d.pow2:]))


def test_duplicate_leaves_last_write_wins():
    d = DevTree(64)
    d.append(64)
    d.update([5, 9, 5, 5, 9, 63, 5], [1.0, 2.0, 3.0, -4.0, 0.5, 7.0, 0.25], alpha=1.0, eps=0.0)
    got = d.host()
    assert got[d.pow2 + 5] == 0.25 and got[d.pow2 + 9] == 0.5 and got[d.pow2 + 63] == 7.0
    assert float(d.max_prio.item()) == 7.0  # the max covers every entry, overwritten or not
    _assert_tree_exact(got)


def test_update_ignores_out_of_range_and_empty():
    d = DevTree(100)
    d.append(100)
    before = d.host()
    i = torch.tensor([-1, 1 << 40], dtype=torch.int64, device="cuda")
    p = torch.tensor([5.0, 6.0], device="cuda")
    N.check(N.lib().mh_per_update(N.ptr(d.tree), d.pow2, N.ptr(i), N.ptr(p), 2, 0.6, 1e-6, N.ptr(d.max_prio),
                                  N.stream_of()), "update")
    N.check(N.lib().mh_per_update(N.ptr(d.tree), d.pow2, None, None, 0, 0.6, 1e-6, N.ptr(d.max_prio),
                                  N.stream_of()), "update0")
    np.testing.assert_array_equal(d.host(), before)


def _sample(tree, pow2, size, seed, counter, batch, beta):
    cur = _cursor(0, size, size)
    idx = torch.empty(batch, dtype=torch.int64, device="cuda")
    w = torch.empty(batch, dtype=torch.float32, device="cuda")
    N.check(N.lib().mh_per_sample(N.ptr(tree), pow2, N.ptr(cur), seed, counter, batch, beta, N.ptr(idx), N.ptr(w),
                                  N.stream_of()), "mh_per_sample")
    return idx.cpu().numpy(), w.cpu().numpy()


@pytest.mark.parametrize("capacity,size,batch", [(700, 700, 256), (1 << 20, 900_001, 256), (5000, 3000, 1000)])
def test_sample_indices_and_weights_match_oracle(capacity, size, batch):
    rng = np.random.default_rng(size)
    ref = SumTree(capacity)
    leaves = np.zeros(ref.pow2)
    leaves[:size] = rng.gamma(0.5, 1.0, size)
    leaves[:size][rng.uniform(size=size) < 0.1] = 0.0  # zero-priority rows are never drawn
    ref.tree = SumTree.build(leaves)
    tree = torch.as_tensor(ref.tree, device="cuda")
    for counter in (0, 1, 12345, (1 << 33) + 7):
        seed = 0xDEADBEEF12345
        idx, w = _sample(tree, ref.pow2, size, seed, counter, batch, 0.4)
        ridx, rw = ref.sample(seed, counter, batch, 0.4, size)
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_allclose(w, rw, rtol=1e-6)
        assert (leaves[idx] > 0).all() and (idx < size).all()
        # importance weights: (N P(i))^-beta / max over the batch
        p = leaves[idx] / leaves.sum()
        wv = (size * p) ** -0.4
        np.testing.assert_allclose(w, wv / wv.max(), rtol=1e-5)


def test_sampling_frequencies_are_proportional():
    """Chi-square goodness of fit of 204,800 stratified draws against p_i / sum p."""
    from scipy import stats
    rng = np.random.default_rng(3)
    cap = 512
    ref = SumTree(cap)
    leaves = np.zeros(ref.pow2)
    leaves[:cap] = rng.uniform(0.0, 1.0, cap) ** 3
    ref.tree = SumTree.build(leaves)
    tree = torch.as_tensor(ref.tree, device="cuda")
    counts = np.zeros(cap, np.int64)
    draws = 800
    for c in range(draws):
        idx, _ = _sample(tree, ref.pow2, cap, 99, c, 256, 0.4)
        np.add.at(counts, idx, 1)
    n = draws * 256
    expect = n * leaves[:cap] / leaves[:cap].sum()
    keep = expect > 5
    chi2 = ((counts[keep] - expect[keep]) ** 2 / expect[keep]).sum()
    pval = stats.chi2.sf(chi2, keep.sum() - 1)
    assert pval > 1e-3, (chi2, pval)


@pytest.mark.parametrize("env_name", ["DuctedFan", "TwoLink"])
def test_config3_nstep_per_trainer(tmp_path, env_name):
    """BASELINE.json config 3: 65,536 envs, n-step windows (n = 20) + PER through the trainer.
    After every iteration: the tree is consistent (exact node sums, no mass past the capacity),
    the last batch's leaves hold (|td| + eps)^alpha of the update's per-window TD error (last
    duplicate wins), and every other leaf is unchanged or a new row at the running max."""
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    args = default_msacl_args(env_name=env_name, env_num=65536, buffer_name="prioritized_replay_buffer",
                              buffer_warm_size=20000, buffer_max_size=1_000_000, max_iteration=10 ** 6,
                              eval_interval=10 ** 6, log_save_interval=10 ** 6, apprfunc_save_interval=10 ** 6,
                              save_folder=str(tmp_path), seed=0, buffer_warm_max_samples=40)
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(args)
    assert type(buffer).__name__ == "PrioritizedReplayBuffer"
    pow2 = buffer.pow2
    seen_updates = 0
    orig_update = buffer.update_batch

    def spy(idx, prio):
        nonlocal seen_updates
        before = buffer.tree.cpu().numpy()
        orig_update(idx, prio)
        after = buffer.tree.cpu().numpy()
        i = idx.cpu().numpy()
        td = prio.cpu().numpy()
        last = {int(k): float(v) for k, v in zip(i, td)}
        for k, v in last.items():
            expect = (abs(np.float64(np.float32(v))) + np.float64(np.float32(buffer.eps))) ** np.float64(
                np.float32(buffer.alpha))
            np.testing.assert_allclose(after[pow2 + k], expect, rtol=2e-15)
        other = np.ones(pow2, bool)
        other[list(last)] = False
        np.testing.assert_array_equal(after[pow2:][other], before[pow2:][other])
        seen_updates += 1

    buffer.update_batch = spy
    for _ in range(3):
        trainer.step()
        trainer.iteration += 1
        t = buffer.tree.cpu().numpy()
        _assert_tree_exact(t)
        size = buffer.size
        assert (t[pow2 + size:] == 0).all() and (t[pow2:pow2 + size] > 0).all()
        assert float(buffer.max_prio.item()) >= t[pow2:].max()
    assert seen_updates == 3
    b = buffer.sample_batch(256)
    assert b["weight"].max().item() == 1.0 and (b["weight"] > 0).all()
    assert not b["done"][:, :-1].any()
