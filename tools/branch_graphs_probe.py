#!/usr/bin/env python3
"""Can the critic and Lyapunov branches of the policy-free MSACL update overlap better as TWO
graphs replayed on two streams than as two branches of one graph? At the bench config, times
(HIP events, back-to-back replays, device time with the stream parked first): the trainer's odd
update graph; the Lyapunov update and the critic update (+ Polyak) each captured alone; and the
two captured graphs replayed concurrently on two streams (fork / join by events).
Diagnostic only (parameters are updated by every replay)."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import msacl_amd  # noqa: F401
    from msacl_amd.utils.config import build_pipeline, default_msacl_args
    from msacl_amd.utils import dist as D
    from tools.gputime import time_launches
    dev = torch.device("cuda", 0)
    cfg = default_msacl_args(env_name="QuadTracking", env_num=65536, sample_batch_size=20, n_step=20,
                             replay_batch_size=256, buffer_max_size=int(1e6), buffer_warm_size=5000,
                             max_iteration=10 ** 9, eval_interval=10 ** 9, log_save_interval=10 ** 9,
                             apprfunc_save_interval=10 ** 9, save_folder=tempfile.mkdtemp(), seed=0, device=dev,
                             sampler_sync_timing=False)
    _, alg, sampler, buffer, _, trainer = build_pipeline(cfg)
    for _ in range(6):
        trainer.step()
        trainer.iteration += 1
    torch.cuda.synchronize()
    data = alg._static

    def capture(fn):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with D.cuda_graph(g):
            fn()
        torch.cuda.synchronize()
        return g

    def critic():
        alg._q_update(data, stats=False)
        alg._target_update()

    g_l = capture(lambda: alg._lyapunov_update(data))
    g_c = capture(critic)
    odd = [k for k in alg._graphs if not k[1]][0]
    g_odd = alg._graphs[odd][0]
    side = torch.cuda.Stream(device=dev)

    def both():
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            g_l.replay()
        g_c.replay()
        main.wait_stream(side)

    def both_rev():
        main = torch.cuda.current_stream(dev)
        side.wait_stream(main)
        g_c.replay()
        with torch.cuda.stream(side):
            g_l.replay()
        main.wait_stream(side)

    res = {}
    for name, fn in (("odd_graph", g_odd.replay), ("lyapunov_alone", g_l.replay), ("critic_alone", g_c.replay),
                     ("two_graphs_two_streams", both), ("two_graphs_two_streams_critic_first", both_rev),
                     ("odd_graph_again", g_odd.replay)):
        res[name] = round(time_launches(fn, 30, host_us_per_call=1500.0, warm=3) * 1e3, 1)
    print(res, flush=True)


if __name__ == "__main__":
    main()
