"""GPU parity of the on-policy path (PPO / POLYC sampler): the GAE kernel (csrc/gae.hip)
against the reference's _finish_trajs outputs and the oracle, and the device OnSampler with
injected actions/resets against the reference's own OnSampler._sample traces
(tests/golden/onpolicy_*.npz)."""
import glob
import os

import numpy as np
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd._native as N
from oracle.onpolicy import finish_trajs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")
TRACES = sorted(glob.glob(os.path.join(G, "onpolicy_*.npz")))
TOL = dict(rtol=1e-5, atol=1e-5)


def gae_gpu(val, val2, rew, done, gamma, lam):
    E, H = rew.shape
    t = lambda a, dt=torch.float32: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device="cuda")  # noqa: E731
    v, v2, r, d = t(val), t(np.nan_to_num(val2, nan=1e30)), t(rew), t(done, torch.uint8)
    adv, ret = torch.empty(E, H, device="cuda"), torch.empty(E, H, device="cuda")
    N.check(N.lib().mh_gae(N.ptr(v), N.ptr(v2), N.ptr(r), N.ptr(d), E, H, gamma, lam, N.ptr(adv), N.ptr(ret),
                           N.stream_of()), "mh_gae")
    return adv.cpu().numpy(), ret.cpu().numpy()


@pytest.mark.parametrize("path", TRACES, ids=os.path.basename)
def test_gae_kernel_matches_reference(path):
    g = np.load(path)
    E, H = g["init_reset"].shape[0], int(g["H"])
    adv, ret = gae_gpu(g["mb_val"].reshape(E, H), g["val2"], g["mb_rew"].reshape(E, H), g["mb_done"].reshape(E, H),
                       float(g["gamma"]), float(g["gae_lambda"]))
    # float64 recurrence rounded once: equal to the reference up to 1 ulp of float32
    np.testing.assert_allclose(adv.reshape(-1), g["mb_adv"], rtol=2e-7, atol=1e-7)
    np.testing.assert_array_equal(ret.reshape(-1), g["mb_ret"])


@pytest.mark.parametrize("E,H", [(1, 1), (63, 33), (130, 64), (257, 100)])
def test_gae_kernel_ragged_shapes_vs_oracle(E, H):
    rng = np.random.default_rng(E * 1000 + H)
    val = rng.standard_normal((E, H)).astype(np.float32)
    val2 = rng.standard_normal((E, H)).astype(np.float32)
    rew = (rng.standard_normal((E, H)) * 5).astype(np.float32)
    done = rng.random((E, H)) < 0.07
    adv, ret = gae_gpu(val, val2, rew, done, 0.99, 0.95)
    a_ref, r_ref = finish_trajs(val, val2, rew, done, 0.99, 0.95)
    np.testing.assert_allclose(adv, a_ref, rtol=2e-7, atol=1e-6)
    np.testing.assert_array_equal(ret, r_ref)


def test_gae_kernel_large_block_properties():
    """E = 65,536 envs x H = 96: spot-check 64 envs against the oracle; the return of a
    segment's last step equals its reward and every segment-end advantage is the one-step TD."""
    E, H = 65536, 96
    rng = np.random.default_rng(3)
    val = rng.standard_normal((E, H)).astype(np.float32)
    val2 = rng.standard_normal((E, H)).astype(np.float32)
    rew = rng.standard_normal((E, H)).astype(np.float32)
    done = rng.random((E, H)) < 0.02
    adv, ret = gae_gpu(val, val2, rew, done, 0.99, 0.95)
    pick = rng.choice(E, 64, replace=False)
    a_ref, r_ref = finish_trajs(val[pick], val2[pick], rew[pick], done[pick], 0.99, 0.95)
    np.testing.assert_allclose(adv[pick], a_ref, rtol=2e-7, atol=1e-6)
    np.testing.assert_array_equal(ret[pick], r_ref)
    end = done.copy()
    end[:, -1] = True
    np.testing.assert_array_equal(ret[end], rew[end])
    td = (rew.astype(np.float64) + 0.99 * val2.astype(np.float64) * (~done)) - val
    np.testing.assert_allclose(adv[end], td[end].astype(np.float32), rtol=1e-6, atol=1e-6)


def _on_sampler(name, E, H, value_sd):
    from msacl_amd.create_pkg.create_sampler import create_sampler
    from msacl_amd.utils.config import default_ppo_args
    from msacl_amd.utils.init_args import init_args
    from msacl_amd.create_pkg.create_envs import create_envs
    args = default_ppo_args(env_name=name, env_num=E, sample_batch_size=H, value_hidden_sizes=[64, 64],
                            policy_hidden_sizes=[64, 64], save_folder="/tmp/msacl_onpolicy_test", seed=0)
    args = init_args(create_envs(**args), **args)
    smp = create_sampler(**args)
    smp.networks.value.load_state_dict(value_sd)
    return smp


@pytest.mark.parametrize("path", TRACES, ids=os.path.basename)
def test_on_sampler_matches_reference_trace(path):
    g = np.load(path)
    name = os.path.basename(path)[9:-4]
    E, H = g["init_reset"].shape[0], int(g["H"])
    vsd = {k[6:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("value/")}
    smp = _on_sampler(name, E, H, vsd)
    smp.obs, _ = smp.envs.reset(reset_states=g["init_reset"])
    smp.envs.set_state(None, None, g["init_steps"])
    out = smp.sample_injected(g["actions"], g["logp_sampled"], g["resets"])
    torch.cuda.synchronize()
    got = {k: v.cpu().numpy() for k, v in out.items()}
    for k in ("obs", "obs2", "act", "rew", "cost", "logp"):
        np.testing.assert_allclose(got[k], g["mb_" + k], **TOL, err_msg=k)
    np.testing.assert_array_equal(got["done"], g["mb_done"])
    assert got["done"].dtype == np.bool_
    # values come from the GPU value MLP (hipBLASLt) vs the reference's CPU torch: GEMM
    # reduction order moves them by ~1e-7 relative, GAE accumulates that over a segment
    np.testing.assert_allclose(got["val"], g["mb_val"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(got["adv"], g["mb_adv"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(got["ret"], g["mb_ret"], rtol=1e-5, atol=1e-5)
