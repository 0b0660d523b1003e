#!/usr/bin/env python3
"""Does the even-iteration MSACL update lose time to its graph's structure? Times, at the bench
config, (a) the update replayed as the trainer does (one graph per branch), (b) the same body
captured as ONE graph by this tool, (c) the body's pieces captured as separate graphs (critic ||
Lyapunov + targets; policy step 1 + alpha; policy step 2 + alpha) replayed back to back, and
(d) each piece alone. Diagnostic only (parameters are updated by every replay)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import msacl_amd  # noqa: F401
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    dev = torch.device("cuda", 0)
    cfg = default_msacl_args(env_name="QuadTracking", env_num=65536, sample_batch_size=20, n_step=20,
                             replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=5000,
                             max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                             apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), seed=0, device=dev,
                             sampler_sync_timing=False)
    _, alg, sampler, buffer, _, trainer = build_pipeline(cfg)
    for _ in range(4):
        trainer.step()
        trainer.iteration += 1
    torch.cuda.synchronize()

    def timeit(fn, reps=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3  # us

    batch = buffer.sample_batch(256)
    res = {"trainer_even": timeit(lambda: alg.model_update(batch, 0)),
           "trainer_odd": timeit(lambda: alg.model_update(batch, 1))}
    data = alg._static

    def capture(fn):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        return g

    def critic_lya():
        side = alg._side_stream()
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            alg._lyapunov_update(data)
        alg._q_update(data, stats=True)
        alg._target_update()
        main.wait_stream(side)

    def pol(k):
        def f():
            _, ent = alg._policy_update(data=data, reuse_adv=k > 0)
            alg._alpha_update(entropy=ent)
        return f

    whole = capture(lambda: alg._update_body(data, True, True))
    res["one_graph_even"] = timeit(whole.replay)
    pieces = [capture(critic_lya), capture(pol(0)), capture(pol(1))]

    def chain():
        for g in pieces:
            g.replay()
    res["three_graphs_even"] = timeit(chain)
    for name, g in zip(("critic||lya", "policy1", "policy2"), pieces):
        res[name] = timeit(g.replay)
    for k, v in res.items():
        print(f"{k:20s} {v:9.1f} us", flush=True)


if __name__ == "__main__":
    main()
