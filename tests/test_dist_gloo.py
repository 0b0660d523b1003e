"""CPU, world_size 2 over gloo: the data-parallel gradient path (utils/dist.py) makes two
ranks with half batches produce exactly the gradient of the full batch, and the advantage
statistic all-reduce gives the global batch's mean/std (msacl.py:400 semantics)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import msacl_amd  # noqa: F401
    from msacl_amd.utils import dist as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 1))
    if rank == 1:  # different init: broadcast must make them equal
        with torch.no_grad():
            for p in net.parameters():
                p.add_(1.0)
    D.broadcast_module(net)
    g = torch.Generator().manual_seed(123)
    x = torch.randn(64, 6, generator=g)
    y = torch.randn(64, 1, generator=g)
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    net.zero_grad()
    ((net(xs) - ys) ** 2).mean().backward()
    D.allreduce_grads(list(net.parameters()))
    local = [p.grad.clone() for p in net.parameters()]
    net.zero_grad()
    ((net(x) - y) ** 2).mean().backward()
    full = [p.grad.clone() for p in net.parameters()]
    adv = torch.randn(64, generator=g)
    mine = adv.chunk(world)[rank].double()
    st = torch.stack([mine.sum(), (mine * mine).sum()])
    D.allreduce_(st)
    n = 64.0
    mean = st[0] / n
    std = ((st[1] - n * mean * mean) / (n - 1)).sqrt()
    ok_stats = abs(mean.item() - adv.double().mean().item()) < 1e-12 and abs(std.item() - adv.double().std().item()) < 1e-9
    q.put((rank, max((a - b).abs().max().item() for a, b in zip(local, full)), ok_stats, D.world_size()))
    dist.destroy_process_group()


def test_two_rank_gradient_average_equals_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, err, ok_stats, ws in res:
        assert ws == 2
        assert err < 1e-6, (rank, err)
        assert ok_stats


def _alg_worker(rank, world, port, tag, q):
    """Rank r updates on rows [r*B/2, (r+1)*B/2) of the reference's fixture batch with the
    matching rows of the recorded rsample noise; the all-reduced update must equal the
    reference's single-process full-batch update (tests/golden/<tag>_update.npz)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import numpy as np
    import torch.distributions.normal as tdn
    import msacl_amd  # noqa: F401
    from tests.test_algorithms import G, make_alg
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = np.load(os.path.join(G, f"{tag}_update.npz"))
        alg = make_alg(tag, "cpu")
        alg.networks.load_state_dict({k[5:]: torch.as_tensor(g[k]) for k in g.files if k.startswith("init/")})
        eps = iter([g[f"eps{i}"] for i in range(int(g["n_eps"]))])

        def draw(shape, dtype, device):
            e = torch.as_tensor(next(eps), dtype=dtype)
            return e.chunk(world)[rank].reshape(shape)
        tdn._standard_normal = draw
        keys = [k[3:] for k in g.files if k.startswith("in_")]
        data = {k: torch.as_tensor(g["in_" + k]).chunk(world)[rank].contiguous() for k in keys}
        alg.model_update(data, 0)
        mine = alg.networks.state_dict()
        worst = 0.0
        for k in g.files:
            if k.startswith("after0/"):
                ref = torch.as_tensor(g[k])
                got = mine[k[7:]]
                bad = (~torch.isclose(got, ref, rtol=1e-4, atol=3e-5)).float().mean().item()
                worst = max(worst, bad)
        q.put((rank, worst))
    finally:
        dist.destroy_process_group()


def _run(tag):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_alg_worker, args=(r, 2, port, tag, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    return res


def test_two_rank_sac_update_equals_reference_full_batch():
    for rank, worst in _run("sac"):
        assert worst < 2e-3, (rank, worst)


def test_two_rank_lac_update_equals_reference_full_batch():
    for rank, worst in _run("lac"):
        assert worst < 2e-3, (rank, worst)
