"""CPU baseline of record for bench.py (SURVEY 8(d) "CPU path timing").

Times the oracle's faithful restatement of the reference CPU sampler (oracle/sampler.py
PerEnvCpuSampler: per-env Python env objects stepped one at a time like gymnasium's
SyncVectorEnv, per-env deques building n-step windows like BaseSampler._n_step, NumPy
StochaPolicy MLP with the reference's default 256 x 256 shape) on the host cores of the box:

  * 1 process x 4 threads   — the reference's own setting (init_args.py:16-17 sets 4 torch
                              threads for serial trainers);
  * P processes x 1 thread  — P = the physical cores this process may use (affinity and the
                              box's per-GPU CPU share of 16 bound it), each its own env batch,
                              started together; the node-aggregate env-steps/s is the baseline.

The CPU work runs ONLY in spawned child processes (the parent may hold the GPU). nproc and the
lscpu topology are recorded with the numbers. The oracle is test infrastructure: this module is
the bench's checker-side `cpu_baseline` leg, never the product path.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _policy_weights(obs_dim, act_dim, hidden=(256, 256), seed=0):
    """Random StochaPolicy weights with torch.nn.Linear's default init (U(+-1/sqrt(fan_in)))."""
    import numpy as np
    rng = np.random.default_rng(seed)
    sizes = [obs_dim, *hidden, 2 * act_dim]
    out = []
    for i in range(len(sizes) - 1):
        bound = 1.0 / np.sqrt(sizes[i])
        out.append((rng.uniform(-bound, bound, (sizes[i + 1], sizes[i])).astype(np.float32),
                    rng.uniform(-bound, bound, sizes[i + 1]).astype(np.float32)))
    return out


def _worker(env_name, n_envs, seconds, threads, seed, start_evt, q):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    for var in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[var] = str(threads)
    from threadpoolctl import threadpool_limits

    from oracle import envs as OE
    from oracle.sampler import CpuPolicy, PerEnvCpuSampler
    cls = OE.ENVS[env_name]
    pol = CpuPolicy(_policy_weights(cls.obs_dim, cls.act_dim, seed=seed))
    with threadpool_limits(limits=threads):
        smp = PerEnvCpuSampler(env_name, n_envs, 20, pol, seed=seed)
        smp.step()  # warm
        if start_evt is not None:
            start_evt.wait()
        steps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            smp.step()
            steps += n_envs
        dt = time.perf_counter() - t0
    q.put((steps, dt))


def host_topology():
    info = {"nproc": os.cpu_count(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "max_jobs": os.environ.get("MAX_JOBS")}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["nproc"]
    try:
        txt = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        kv = {}
        for ln in txt.splitlines():
            if ":" in ln:
                k, v = ln.split(":", 1)
                kv[k.strip()] = v.strip()
        info["model"] = kv.get("Model name")
        sockets = int(kv.get("Socket(s)", "1") or 1)
        cores = int(kv.get("Core(s) per socket", "0") or 0)
        tpc = int(kv.get("Thread(s) per core", "1") or 1)
        info.update(sockets=sockets, cores_per_socket=cores, threads_per_core=tpc,
                    physical_cores=sockets * cores if cores else None)
    except (OSError, ValueError, subprocess.SubprocessError):
        info["physical_cores"] = None
    return info


def _run(ctx, env_name, n_envs, seconds, threads, procs):
    q = ctx.Queue()
    evt = ctx.Event()
    ps = [ctx.Process(target=_worker, args=(env_name, n_envs, seconds, threads, 1000 + i, evt, q)) for i in range(procs)]
    for p in ps:
        p.start()
    time.sleep(0.2)
    evt.set()
    res = [q.get(timeout=seconds * 4 + 120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    return sum(r[0] for r in res), max(r[1] for r in res)


def measure(env_name="QuadTracking", seconds=6.0, n_envs=64, procs=None, box_share=16):
    """-> dict for bench.py's cpu_baseline (value = P-process node aggregate)."""
    topo = host_topology()
    ctx = mp.get_context("spawn")
    s1, t1 = _run(ctx, env_name, n_envs, seconds, 4, 1)
    if procs is None:
        cand = [c for c in (topo.get("physical_cores"), topo.get("affinity"), box_share) if c]
        procs = max(1, min(cand))
    sp, tp = _run(ctx, env_name, n_envs, seconds, 1, procs)
    s11, t11 = _run(ctx, env_name, n_envs, seconds, 1, 1)
    single = s1 / t1
    agg = sp / tp
    one = s11 / t11
    phys = topo.get("physical_cores")
    proj = None
    if phys and phys > procs:
        # SURVEY 8(d) asks for P = the physical cores; the pool caps a GPU box's worker pools at
        # its per-GPU CPU share (16 of the host's cores are this GPU's), so the physical-core
        # figure is the measured per-process rate times the core count, with the measured
        # P-process efficiency (aggregate / (P x the 1-process rate)) shown beside it
        proj = {"cores": phys, "value": round(agg / procs * phys, 1),
                "method": (f"measured {procs}-process per-process rate x {phys} physical cores (linear; "
                           f"not run: the pool limits a one-GPU box's worker pools to its {box_share}-CPU share)"),
                "efficiency_at_measured_procs": round(agg / (procs * one), 3)}
    return {
        "value": round(agg, 1), "unit": "env_steps/s", "cores": procs, "kind": "port",
        "sample": (f"{env_name}: oracle restatement of the reference CPU sampler (per-env SyncVectorEnv loop + "
                   f"_n_step deques + NumPy 256x256 StochaPolicy), {procs} processes x 1 thread x {n_envs} envs, "
                   f"{seconds:.0f} s each, started together; value = node aggregate"),
        "one_process_4_threads": round(single, 1),
        "one_process_1_thread": round(one, 1),
        "per_process": round(agg / procs, 1),
        "projected_physical_cores": proj,
        "host": topo,
        "procs_rule": "min(physical cores, CPU affinity, the box's per-GPU CPU share of 16)",
    }


if __name__ == "__main__":
    import json
    print(json.dumps(measure(sys.argv[1] if len(sys.argv) > 1 else "QuadTracking")))
