#!/usr/bin/env python3
"""Calibrate the CPU baseline: the reference's own CPU sampler vs the oracle restatement that
bench.py times on the GPU box (tools/cpu_baseline.py), on THIS container's cores.

Build-container only (the reference never travels to the GPU box). The reference path is the
one tools/gen_golden.py executes: BaseSampler._n_step compiled from RL/trainer/sampler/base.py
over reference env objects (tools/refload.py; gymnasium's SyncVectorEnv autoreset restated) with
the reference StochaPolicy (256 x 256, TanhGaussDistribution, torch CPU). Both are timed on
QuadTracking with 64 envs as 1 process x 4 torch threads (init_args.py:16-17) and as P
processes x 1 thread. Writes profiles/r02_cpu_ratio.json: ratio = reference / restatement.
Usage: python tools/cpu_ratio.py [seconds]
"""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import time
import types
from collections import deque

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAME, E = "QuadTracking", 64


def _ref_worker(seconds, threads, seed, evt, q):
    import numpy as np
    import torch
    torch.set_num_threads(threads)
    from oracle import envs as OE
    from tools import gen_golden as GG
    from tools.refload import REF, load_env
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from RL.apprfunc.mlp import StochaPolicy
    from RL.utils.act_distribution_cls import TanhGaussDistribution
    cls = OE.ENVS[NAME]
    rng = np.random.default_rng(seed)
    torch.manual_seed(seed)
    mod = load_env(NAME)
    draw = lambda k: cls.reset_draw(rng, k, gauss=lambda m: rng.standard_normal((m, 3)))  # noqa: E731

    class Venv(GG.RefVectorEnv):  # unbounded reset pool, no per-step logs
        def step(self, actions):
            obs, finals = [], np.empty(self.E, dtype=object)
            rewards = np.zeros(self.E, np.float64)
            terms = np.zeros(self.E, bool)
            truncs = np.zeros(self.E, bool)
            for i, env in enumerate(self.envs):
                o, r, te, tr, _ = env.step(actions[i])
                rewards[i], terms[i], truncs[i] = r, te, tr
                o = np.asarray(o, np.float32).copy()
                if te or tr:
                    finals[i] = o
                    o = GG.ref_reset(self.mod, env, self.name, draw(1)[0])
                obs.append(o)
            return np.stack(obs).astype(np.float32), rewards, terms, truncs, {"final_observation": finals}

    venv = Venv(mod, NAME, E, draw(E), np.zeros(E, np.int64), draw(1))
    policy = StochaPolicy(obs_dim=cls.obs_dim, act_dim=cls.act_dim, hidden_sizes=[256, 256], hidden_activation="relu",
                          output_activation="linear", min_log_std=-20, max_log_std=1, act_high_lim=cls.act_high.copy(),
                          act_low_lim=cls.act_low.copy(), action_distribution_cls=TanhGaussDistribution)

    class Net:
        def __init__(self):
            self.policy = policy

        def create_action_distributions(self, logits):
            return policy.get_act_dist_cls(logits)

    smp = types.SimpleNamespace(env_id=NAME, num_envs=E, envs=venv, networks=Net(), noise_params=None,
                                action_type="continu", reward_scale=100.0, cost_scale=100.0, target_value=0.0,
                                n_step=20, n_step_buffers=[deque(maxlen=20) for _ in range(E)],
                                obs=venv.obs0.astype(np.float32).copy())
    n_step = types.MethodType(GG.load_n_step(), smp)
    with torch.no_grad():
        n_step()
        evt.wait()
        steps, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            n_step()
            steps += E
        q.put((steps, time.perf_counter() - t0))


def _port_worker(seconds, threads, seed, evt, q):
    from tools.cpu_baseline import _worker
    _worker(NAME, E, seconds, threads, seed, evt, q)


def _run(target, seconds, threads, procs):
    ctx = mp.get_context("spawn")
    q, evt = ctx.Queue(), ctx.Event()
    ps = [ctx.Process(target=target, args=(seconds, threads, 500 + i, evt, q)) for i in range(procs)]
    for p in ps:
        p.start()
    time.sleep(3.0)  # imports
    evt.set()
    res = [q.get(timeout=seconds * 4 + 300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    return sum(r[0] for r in res) / max(r[1] for r in res)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    from tools.cpu_baseline import host_topology
    topo = host_topology()
    P = topo.get("physical_cores") or os.cpu_count()
    out = {"env": NAME, "envs_per_process": E, "seconds": seconds, "host": topo}
    for label, threads, procs in (("1proc_4thr", 4, 1), (f"{P}proc_1thr", 1, P)):
        ref = _run(_ref_worker, seconds, threads, procs)
        port = _run(_port_worker, seconds, threads, procs)
        out[label] = {"reference_env_steps_per_s": round(ref, 1), "restatement_env_steps_per_s": round(port, 1),
                      "ratio_reference_over_restatement": round(ref / port, 4)}
        print(label, out[label], flush=True)
    path = os.path.join(ROOT, "profiles", "r02_cpu_ratio.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
