#!/usr/bin/env python3
"""Headline benchmark: env steps/sec (whole node), QuadrotorTracking, 65,536 envs per GPU.

A "step" is one NstepOffSerialTrainer.step() of the MSACL pipeline built exactly like
example/msacl_train.py (create_envs -> init_args -> create_alg/sampler/buffer/trainer):
sample() = 20 lockstep steps of all envs (policy MLP + fused HIP rollout/n-step emission),
add_batch, replay sample_batch(256) and the full MSACL model_update (twin-Q, Lyapunov, 2x
policy + alpha on even iterations). Env-steps per step = envs x horizon (20).

Run: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under torch.distributed.run
(one rank per GPU, RCCL). Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PEAK_F32_MFMA_TFS = 157.3  # MI355X dense f32 matrix peak (v_mfma_f32_*_f32)
PEAK_F16_MFMA_TFS = 2500.0  # MI355X dense f16 matrix peak (v_mfma_f32_32x32x16_f16), MI355X_MICROARCH.md
PMC_TRAFFIC = "r06_pmc_traffic_v2.json"  # the PMC summary of the current kernels (tools/pmc.sh + tools/pmc_summary.py)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--env", default="QuadTracking")
    p.add_argument("--envs", type=int, default=65536, help="parallel envs per GPU")
    p.add_argument("--policy", choices=["init", "hover"], default="init",
                   help="init: PyTorch default init (SURVEY 8d); hover: action mean [mg,0,0,0], long episodes")
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="per CPU-baseline leg (1x4 threads, Px1)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-4m", action="store_true", help="skip the 4,194,304-env lockstep-kernel measurement")
    p.add_argument("--no-twin-streams", action="store_true",
                   help="alg_twin_streams off: q1 / q2 branches of the update on one stream (A/B)")
    p.add_argument("--overlap", action="store_true",
                   help="trainer_overlap_sampling: sampling beside the policy-free updates (A/B; off by default)")
    p.add_argument("--dp-rehearsal", action="store_true",
                   help="one GPU: a world-size-1 RCCL process group with the update's gradient / statistics "
                        "all-reduces issued anyway (the data-parallel step's per-rank cost without the wire)")
    p.add_argument("--graph-collectives", action="store_true",
                   help="the all-reduces inside the captured update graph (MSACL_GRAPH_COLLECTIVES=1) instead of "
                        "graph segments cut at them")
    p.add_argument("--graph-segments", action="store_true",
                   help="capture the update as graphs cut at its all-reduces (the world size > 1 path)")
    p.add_argument("--eager-update", action="store_true",
                   help="run the model update eagerly (no HIP-graph replay), as with world size > 1")
    p.add_argument("--update-gemm", dest="update_gemm", choices=["auto", "hip", "blas"], default=None,
                   help="GEMMs of the update MLPs: auto (default: mh_gemm_f32 where faster), hip or blas")
    p.add_argument("--blas", choices=["hipblaslt", "rocblas"], default=None,
                   help="GEMM library of the PyTorch parts (update MLPs); default: the config's (rocblas)")
    return p.parse_args()


def set_hover_policy(policy, mg):
    """SURVEY 8d second variant: mean = [mg, 0, 0, 0] (tanh-squashed centre of the box is mg
    for the thrust), std = (2, 0.5, 0.5, 0.5) in pre-tanh units scaled to the box."""
    import math
    import torch
    last = policy.policy[-2]
    with torch.no_grad():
        last.weight.zero_()
        last.bias.zero_()
        A = last.bias.numel() // 2
        stds = [2.0 / mg, 0.5 / 10.0, 0.5 / 10.0, 0.5 / 10.0][:A]
        for i, s in enumerate(stds):
            last.bias[A + i] = math.log(s)


def cpu_baseline(env_name, seconds):
    """SURVEY 8(d) CPU baseline of record (tools/cpu_baseline.py): the oracle restatement of the
    reference CPU sampler as 1 process x 4 threads and as P processes x 1 thread (P = physical
    cores usable here, <= the box's per-GPU share of 16), in spawned children; value = the
    P-process node aggregate. The restatement/reference speed ratio was measured in the build
    container, where the reference itself runs (tools/cpu_ratio.py -> profiles/r02_cpu_ratio.json),
    and scales the value to a reference-equivalent figure."""
    from tools.cpu_baseline import measure
    out = measure(env_name, seconds=seconds)
    path = os.path.join(ROOT, "profiles", "r02_cpu_ratio.json")
    try:
        cal = json.load(open(path))
        key = next(k for k in cal if k.endswith("proc_1thr") and not k.startswith("1proc"))
        ratio = float(cal[key]["ratio_reference_over_restatement"])
        out["reference_equivalent_value"] = round(out["value"] * ratio, 1)
        out["calibration"] = {"ratio_reference_over_restatement": ratio, "source": "profiles/r02_cpu_ratio.json",
                              "measured": f"{cal['env']}, {cal['envs_per_process']} envs/process, {key}, build container",
                              "calibration_cpu": cal["host"].get("model"),
                              "note": "ratio measured on the build container's CPU (the reference cannot run on "
                                      "the GPU box), applied to this host's CPU: a cross-CPU estimate"}
    except (OSError, ValueError, StopIteration, KeyError):
        out["calibration"] = None
    return out


def main():
    a = parse()
    import torch
    import msacl_amd  # noqa: F401
    import msacl_amd._native as N
    from msacl_amd.utils import dist as D
    from msacl_amd.utils.config import build_pipeline, default_msacl_args

    D.init_from_env()
    rank, world = D.rank(), D.world_size()
    local = D.local_device_index()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if a.graph_collectives:
        D.set_graph_collectives(True)
    dp_rehearsal = None
    if a.dp_rehearsal and world == 1:
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                             device_id=dev)
        D.force_collectives(True)
        dp_rehearsal = {"backend": torch.distributed.get_backend(), "world": 1,
                        "collectives": "in the update graph" if D.collectives_in_graph() else "graph segments"}
    # self-check of the launch: every rank joins one all-reduce of a ones tensor over the data-path
    # backend (RCCL on the MI355X node); the count must equal --gpus, else the line is not valid
    dist_backend = torch.distributed.get_backend() if world > 1 else None
    ranks_seen = int(round(D.sum_over_ranks(1.0))) if world > 1 else 1
    if ranks_seen != a.gpus or world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the process group has {world} ranks and an all-reduce over "
              f"{dist_backend} counted {ranks_seen}", file=sys.stderr, flush=True)
        if world > 1:
            torch.distributed.destroy_process_group()
        sys.exit(3)
    horizon = 20
    tmp = tempfile.mkdtemp(prefix=f"msacl_bench_r{rank}_")
    cfg = default_msacl_args(env_name=a.env, env_num=a.envs, env_seed=1 + rank * 1000003, seed=rank * 1000000,
                             sample_batch_size=horizon, n_step=20, replay_batch_size=256, buffer_max_size=int(1e6),
                             buffer_warm_size=5000, max_iteration=10 ** 9, eval_interval=10 ** 9,
                             log_save_interval=10 ** 9, apprfunc_save_interval=10 ** 9, save_folder=tmp,
                             num_eval_episode=1, sampler_sync_timing=False, device=dev)
    if a.blas is not None:
        cfg["blas_backend"] = a.blas
    if a.update_gemm is not None:
        cfg["update_gemm"] = a.update_gemm
    if a.eager_update:
        cfg["alg_use_graph"] = False
    if a.overlap:
        cfg["trainer_overlap_sampling"] = True
    if a.no_twin_streams:
        cfg["alg_twin_streams"] = False
    if a.graph_segments:
        cfg["alg_force_graph_segments"] = True
    if a.policy == "hover":
        cfg["buffer_warm_size"] = 0
    args, alg, sampler, buffer, evaluator, trainer = build_pipeline(cfg)
    if a.policy == "hover":
        set_hover_policy(alg.networks.policy, float(sampler.envs.single_action_space.high[0]) / 2)

    def one_step():
        trainer.step()
        trainer.iteration += 1

    for _ in range(a.warmup):
        one_step()
    # the horizon emission alone (k_emit_cells via mh_sample_horizon_emit) on the last warm-up
    # step's horizon, before the timed region: it rewrites the same store rows (idempotent) and
    # moves no env state, and the window count is then one of the trainer's own steps (after the
    # timed region the init policy's episodes have mostly become short and horizons emit ~1 k)
    from tools.gputime import time_launches
    trainer.finish_pending()
    emit_diag = None
    if (hasattr(sampler, "_pack_policy") and getattr(sampler, "_fused_horizon_ok", None)
            and sampler._fused_horizon_ok(bool(sampler._pack_policy()))):
        h_e, st_e = sampler.envs.handle(), N.stream_of(dev)
        win_dev = torch.zeros(1, dtype=torch.int64, device=dev)

        def k_emit_only():
            N.check(N.lib().mh_sample_horizon_emit(h_e, sampler.horizon, ctypes.byref(buffer.ws), N.ptr(win_dev),
                                                   st_e), "mh_sample_horizon_emit")
        k_emit_only()
        torch.cuda.synchronize()
        emit_diag = (time_launches(k_emit_only, 20) * 1e-3, int(win_dev.item()))
    win0 = int(buffer.cursor[2].item())
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one_step()
    torch.cuda.synchronize()  # every stream: an overlapped sampling still in flight is inside the timed region
    if world > 1:
        torch.distributed.barrier()
    t1 = time.perf_counter()
    windows_timed = int(buffer.cursor[2].item()) - win0
    elapsed = D.max_over_ranks(t1 - t0)
    env_steps_total = world * a.envs * horizon * a.steps
    value = env_steps_total / elapsed

    trainer.finish_pending()

    # ---- phase split (diagnostic, after the timed region): sample() vs replay sample + update,
    # each synchronised, over PH_PAIRS (policy-free, policy) step pairs; per pair the two steps'
    # mean, and the median over the pairs (single pairs swing by +-10 % on one box)
    PH_PAIRS = 8
    pair_s, pair_u, u_by_kind = [], [], {True: [], False: []}
    for _ in range(PH_PAIRS):
        ps = pu = 0.0
        for _ in range(2):
            torch.cuda.synchronize()
            ta = time.perf_counter()
            samples, _ = sampler.sample()
            buffer.add_batch(samples)
            torch.cuda.synchronize()
            tb_ = time.perf_counter()
            policy_step = trainer.iteration % trainer.policy_frequency == 0
            trainer.replay_and_update()  # as step() does (the draw inside the replayed update graph)
            trainer.iteration += 1
            torch.cuda.synchronize()
            ps += tb_ - ta
            du = time.perf_counter() - tb_
            pu += du
            u_by_kind[policy_step].append(du)
        pair_s.append(ps)
        pair_u.append(pu)
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    ph_s, ph_u = med(pair_s), med(pair_u)
    # host enqueue rate: the host time of trainer steps without a sync (it only blocks when the
    # device queue is full or a call waits) against the same steps' wall time: equal = host-bound
    k_host = 6
    host_parts = {}

    def timed(obj, name):  # wrap a bound method with a host timer (restored below)
        fn = getattr(obj, name)

        def w(*args, **kw):
            t = time.perf_counter()
            try:
                return fn(*args, **kw)
            finally:
                host_parts[name] = host_parts.get(name, 0.0) + time.perf_counter() - t
        setattr(obj, name, w)
        return name

    wrapped = [(trainer, timed(trainer, "_sample")), (trainer, timed(trainer, "_replay_batch")),
               (alg, timed(alg, "model_update")), (alg, timed(alg, "model_update_drawn")),
               (buffer, timed(buffer, "add_batch")), (trainer, timed(trainer, "_graph_step"))]
    torch.cuda.synchronize()
    th0 = time.perf_counter()
    for _ in range(k_host):
        one_step()
    th1 = time.perf_counter()
    torch.cuda.synchronize()
    th2 = time.perf_counter()
    for obj, name in wrapped:
        delattr(obj, name)
    phases = {"sample_ms": round(ph_s / 2 * 1e3, 3), "replay_and_update_ms": round(ph_u / 2 * 1e3, 3),
              "replay_and_update_ms_policy_free_policy": [round(med(u_by_kind[False]) * 1e3, 3),
                                                          round(med(u_by_kind[True]) * 1e3, 3)],
              "phase_pairs": PH_PAIRS,
              "sampler_only_env_steps_per_s": round(a.envs * horizon / (ph_s / 2), 1),
              "update_to_data_ratio": round(1.0 / (a.envs * horizon), 9),
              "host_enqueue_ms_per_step": round((th1 - th0) / k_host * 1e3, 3),
              "wall_ms_per_step_same_steps": round((th2 - th0) / k_host * 1e3, 3),
              "host_ms_per_step_by_call": {k: round(v / k_host * 1e3, 3) for k, v in host_parts.items()}}

    # ---- per-kernel durations, right after the timed region: HIP events on the launch stream
    # around R back-to-back launches of the engine's lockstep kernels on the live pipeline state
    # (the graph replays carry no per-kernel events). The stream is parked on a GPU spin while
    # the host enqueues, so the events bracket device time (tools/gputime.py).
    from tools.gputime import time_launches
    h = sampler.envs.handle()
    st = N.stream_of(dev)
    with torch.no_grad():
        logits, _raw = sampler._policy_raw()
    reps = 20

    def k_roll():  # k_rollout<Env> alone (no store: ring push, no emission)
        N.lib().mh_rollout_step(h, N.ptr(logits), None, None, None, N.ptr(sampler.obs), None, None, None, st)

    def k_pair():  # k_rollout<Env> + k_emit_fused into the replay store
        N.lib().mh_rollout_step(h, N.ptr(logits), None, None, None, N.ptr(sampler.obs), ctypes.byref(buffer.ws),
                                None, None, st)

    have_fused = sampler._pack_policy() if hasattr(sampler, "_pack_policy") else False
    pol_out = torch.empty(a.envs, 2 * sampler.envs.act_dim, dtype=torch.float32, device=dev)

    def k_policy():  # the sampler's fused f32-MFMA policy forward (csrc/policy_mlp.hip)
        N.lib().mh_policy_forward(N.ptr(sampler._packed), N.ptr(sampler.obs), a.envs, sampler.envs.obs_dim,
                                  2 * sampler.envs.act_dim, N.ptr(pol_out), st)

    def k_defer():  # the sampler's lockstep kernel: k_rollout<Env> + its emitter waves copying the
        # previous launch's windows into the replay store (mh_rollout_step_deferred)
        N.lib().mh_rollout_step_deferred(h, N.ptr(logits), None, None, None, N.ptr(sampler.obs),
                                         ctypes.byref(buffer.ws), None, None, st)

    fused_h = bool(have_fused and getattr(sampler, "_fused_horizon_ok", None) and sampler._fused_horizon_ok(True))
    H = sampler.horizon
    noise_ptr = N.ptr(sampler._noise) if getattr(sampler, "_noise", None) is not None else None

    t_emit_h, windows_emit = emit_diag if emit_diag is not None else (None, None)

    def k_fused():  # the fused horizon kernel alone (its windows are not emitted)
        N.lib().mh_sample_horizon(h, N.ptr(sampler._packed), sampler.envs.obs_dim, 2 * sampler.envs.act_dim,
                                  N.ptr(sampler.obs), H, None, noise_ptr, None, None, st)

    t_fh = None
    if fused_h:
        # one launch per measurement (each after the stream's spin), averaged: five back-to-back
        # persistent MFMA launches ran ~10 % slower than the same kernel inside the trainer's
        # steps (rocprofv3 average), where the update's launches sit between horizons
        k_fused()
        t_fh = sum(time_launches(k_fused, 1, warm=0) for _ in range(5)) / 5 * 1e-3
    t_pol = time_launches(k_policy, reps) * 1e-3 if have_fused else None
    t_step = time_launches(k_roll, reps) * 1e-3
    win1 = int(buffer.cursor[2].item())
    t_pair = time_launches(k_pair, reps, warm=0) * 1e-3
    windows = (int(buffer.cursor[2].item()) - win1) / reps
    t_emit = max(t_pair - t_step, 1e-9)
    win2 = int(buffer.cursor[2].item())
    t_defer = time_launches(k_defer, reps, warm=0) * 1e-3
    N.check(N.lib().mh_rollout_flush(h, st), "mh_rollout_flush")
    torch.cuda.synchronize()
    windows_defer = (int(buffer.cursor[2].item()) - win2) / reps

    # ---- live roofline of the engine's kernels (algorithmic bytes / measured device time)
    info = sampler.envs.info
    S, XS, D_, A_, F = info.state_dim, info.xstate_dim, info.obs_dim, info.act_dim, info.record_floats
    n = sampler.n_step
    bytes_step_kernel = a.envs * ((S * 4 + XS * 8 + 4 + 2 * A_ * 4 + D_ * 4 + 8)
                                  + (S * 4 + XS * 8 + 4 + D_ * 4 + F * 4 + 8 + 4))
    bytes_window = n * F * 4 + n * (2 * D_ + A_ + 4) * 4  # ring records read + 7 store arrays written
    bytes_emit = windows * bytes_window
    bytes_defer = bytes_step_kernel + windows_defer * bytes_window
    kernels = {
        "rollout_emit": {"avg_us": round(t_defer * 1e6, 3), "bytes": round(bytes_defer, 1),
                         "windows": windows_defer, "GBps": round(bytes_defer / t_defer / 1e9, 1),
                         "note": "the sampler's lockstep kernel (mh_rollout_step_deferred): the env step of "
                                 "every env + the previous launch's windows into the replay store"},
        "rollout_step": {"avg_us": round(t_step * 1e6, 3), "bytes": bytes_step_kernel,
                         "GBps": round(bytes_step_kernel / t_step / 1e9, 1)},
        "window_emit": {"avg_us": round(t_emit * 1e6, 3), "bytes": bytes_emit, "windows": windows,
                        "GBps": round(bytes_emit / t_emit / 1e9, 1),
                        "note": "separate emission launch (mh_rollout_step), not used by the sampler"},
        "method": f"HIP events around {reps} back-to-back launches after a GPU spin; emit = (rollout+emit) - rollout",
    }
    D0, A2 = sampler.envs.obs_dim, 2 * sampler.envs.act_dim
    flops_lockstep = 2.0 * a.envs * (D0 * 256 + 256 * 256 + 256 * A2)
    if fused_h:
        # the fused horizon kernel: per lockstep the policy's split-f16 MFMA work (3 f16 products
        # per f32-equivalent product) beside the env step; HBM traffic per horizon: the ring
        # records and the per-horizon state / observation load + store (W2 is re-read from L2)
        bytes_fh = a.envs * (H * F * 4 + 2 * (S * 4 + XS * 8 + 16) + 2 * D_ * 4)
        kernels["sample_fused"] = {
            "avg_us_per_horizon": round(t_fh * 1e6, 2), "avg_us_per_lockstep": round(t_fh / H * 1e6, 3),
            "f16_mfma_TFLOPs": round(3 * flops_lockstep * H / t_fh / 1e12, 1),
            "frac_f16_mfma_peak": round(3 * flops_lockstep * H / t_fh / 1e12 / PEAK_F16_MFMA_TFS, 4),
            "hbm_bytes": bytes_fh, "GBps": round(bytes_fh / t_fh / 1e9, 1),
            "note": "k_sample_fused<Env>: the whole horizon (policy MLP + sample + env step + ring push for "
                    f"{H} locksteps) in one persistent launch, without its window emission"}
    if fused_h and t_emit_h is not None:
        bytes_win = windows_emit * bytes_window
        kernels["emit_horizon"] = {"avg_us": round(t_emit_h * 1e6, 2), "windows": windows_emit, "bytes": bytes_win,
                                   "GBps": round(bytes_win / t_emit_h / 1e9, 1),
                                   "frac": round(bytes_win / t_emit_h / 1e9 / PEAK_HBM_GBS, 4),
                                   "note": "k_emit_cells alone (mh_sample_horizon_emit) on the last warm-up step's "
                                           "horizon, before the timed region: its windows, ring records -> replay "
                                           "store rows"}
    if t_pol is not None:
        flops = flops_lockstep
        # split-f16 arithmetic: every f32 product is 3 f16 MFMA products (hi.hi + hi.lo + lo.hi),
        # so the kernel's own ceiling is the dense f16 peak / 3 in f32-equivalent flop/s
        kernels["policy_forward"] = {"avg_us": round(t_pol * 1e6, 3), "flops": flops,
                                     "TFLOPs": round(flops / t_pol / 1e12, 2),
                                     "f16_mfma_TFLOPs": round(3 * flops / t_pol / 1e12, 2),
                                     "frac_f16_mfma_peak": round(3 * flops / t_pol / 1e12 / PEAK_F16_MFMA_TFS, 4),
                                     "vs_f32_mfma_peak": round(flops / t_pol / 1e12 / PEAK_F32_MFMA_TFS, 4),
                                     "note": "per lockstep step; f32-accurate split-f16 MFMA (3 products per f32 "
                                             "product): bound by the f16 MFMA rate, not HBM; flops = f32-equivalent"}
    # the same lockstep kernel over 4,194,304 envs (SURVEY 8(d)'s second size): its 2.4 GB of state,
    # observations and ring records exceed the 256 MB Infinity Cache, so this fraction is HBM's
    # (at 65,536 envs the 37 MB working set is cache-resident)
    if not a.no_4m and a.env == "QuadTracking" and world == 1:
        import contextlib
        import io
        from tools.kernel_bench import bench_rollout
        with contextlib.redirect_stdout(io.StringIO()):  # (kernel_bench prints its rows)
            rows4 = bench_rollout(a.env, 4_194_304, reps, dev)
        r4 = [r for r in rows4 if r["kernel"] == "rollout_step"]
        if r4:
            r4 = r4[0]
            kernels["rollout_step_4m"] = {"avg_us": r4["avg_us"], "env_steps": r4["env_steps"],
                                          "bytes": r4["env_steps"] * r4["bytes_per_unit"], "GBps": r4["GBps"],
                                          "frac": r4["frac"],
                                          "note": "k_rollout<QuadTracking> at 4,194,304 envs (beyond the Infinity Cache)"}
    dom = "sample_fused" if fused_h else "rollout_emit"
    ach = kernels[dom]["f16_mfma_TFLOPs"] if fused_h else kernels[dom]["GBps"]
    # HBM bytes per launch: PMC counters cannot be read from inside this process (rocprofv3 --pmc
    # wraps the whole command), so `traffic` is the committed measurement of this same command
    # (tools/pmc.sh: separate FETCH_SIZE / WRITE_SIZE passes, tools/pmc_summary.py applies the
    # gfx950 FETCH_SIZE correction), named in traffic_source; null when none matches the config
    traffic, traffic_src = None, None
    pmc_path = os.path.join(ROOT, "profiles", PMC_TRAFFIC)
    if a.env == "QuadTracking" and a.envs == 65536 and os.path.exists(pmc_path):
        try:
            from tools.kernel_hash import rollout_sources_sha
            pmc = json.load(open(pmc_path))
            if pmc.get("rollout_sources_sha") == rollout_sources_sha():
                traffic = pmc.get(dom, {}).get("bytes_per_launch")
                traffic = None if traffic is None else round(float(traffic), 1)
                traffic_src = (f"profiles/{PMC_TRAFFIC} (rocprofv3 --pmc passes of this bench command on the same "
                               f"kernel sources, sha {pmc['rollout_sources_sha']}; not measured live)")
            else:  # the kernel changed since the PMC passes: no stale figure
                traffic_src = f"profiles/{PMC_TRAFFIC} is for other kernel sources (stale): not reported"
        except (OSError, ValueError):
            traffic = None
    if fused_h:
        roof = {"bound": "mfma", "kernel": "k_sample_fused<%s>" % a.env, "achieved": round(ach, 1),
                "peak": PEAK_F16_MFMA_TFS, "unit": "TFLOP/s", "frac": round(ach / PEAK_F16_MFMA_TFS, 4),
                "traffic": traffic, "traffic_source": traffic_src,
                "flops_note": "f16 MFMA flops of the policy's split-f16 arithmetic (3 per f32-equivalent product) "
                              "over the fused kernel's device time; its env VALU work overlaps on the same SIMDs",
                "hbm_GBps": kernels[dom]["GBps"]}
    else:
        roof = {"bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": traffic, "traffic_source": traffic_src}
    if "rollout_step_4m" in kernels:
        roof["frac_4m_envs"] = kernels["rollout_step_4m"]["frac"]

    out = {
        "metric": "env steps/sec (whole node), QuadrotorTracking 65536 envs, 1/2/4/8 MI355X",
        "value": round(value, 1), "unit": "env_steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{a.env} MSACL NstepOffSerialTrainer.step: {a.envs} envs/GPU x horizon {horizon}, "
                               f"n-step {n} windows, replay batch 256, full MSACL update",
                   "env": a.env, "envs_per_gpu": a.envs, "horizon": horizon, "n_step": n, "replay_batch": 256,
                   "policy": a.policy, "parallelism": f"dp{world}"},
        "roofline": roof,
        "dist_backend": dist_backend, "rccl_ranks": ranks_seen, "dp_rehearsal": dp_rehearsal,
        "kernels": kernels,
        "windows_per_step": round(windows_timed / a.steps, 1),
        "phases": phases,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.env, a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    elif dp_rehearsal is not None:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
