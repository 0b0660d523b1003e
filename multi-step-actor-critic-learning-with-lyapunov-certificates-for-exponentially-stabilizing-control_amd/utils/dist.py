"""Data-parallel plumbing: one process per GPU, torch.distributed with the "nccl" backend
(= RCCL over xGMI on ROCm), or "gloo" for the CPU tests.

The reference is single-process (no torch.distributed anywhere); the only exchange this engine
adds is the gradient all-reduce of each optimiser step plus the 2-float (sum, sumsq) all-reduce
of the stability-advantage normalisation. Gradients of one optimiser step go out as ONE flat
bucket (at the reference config 0.54-0.56 MB for Q/Lyapunov, 0.28 MB for the policy): at these
sizes a ring all-reduce over xGMI is latency-bound, so one call per step beats per-tensor calls.
"""
from __future__ import annotations

import contextlib
import gc
import os

import torch
import torch.distributed as dist


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def local_device_index() -> int:
    """This rank's GPU: LOCAL_RANK, wrapped onto the visible devices (one rank per GPU in
    production; several ranks per GPU only in the gloo rehearsal)."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = torch.cuda.device_count()
    return local % n if n > 0 else local


def init_from_env(backend=None):
    """Initialise from torchrun-style env vars (RANK, WORLD_SIZE, MASTER_ADDR/PORT)."""
    if is_initialized() or int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return False
    if backend is None:
        # MSACL_DIST_BACKEND=gloo: rehearse the multi-rank path with several ranks on one GPU
        # (RCCL refuses two ranks per device)
        backend = os.environ.get("MSACL_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    kw = {}
    if backend == "nccl":
        local = local_device_index()
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend=backend, **kw)
    return True


@contextlib.contextmanager
def cuda_graph(g, **kw):
    """torch.cuda.graph with the cyclic garbage collector paused while the stream captures.
    torch.cuda.graph collects once before the capture, but an allocation inside the capture can
    trigger another collection, which may finalise graphs, events or streams of pipelines that
    died in reference cycles: HIP calls that are illegal during a capture (seen as aborts and a
    host segfault in a later replay during one full test session)."""
    was = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(g, **kw):
            yield
    finally:
        if was:
            gc.enable()


class GraphSegments:
    """A model update captured as a chain of HIP graphs cut at its collectives (data parallel,
    world size > 1). While active (`capturing(seg)`), every allreduce_ / allreduce_grads call ends
    the graph being captured, is recorded, and the capture continues in a new graph of the same
    memory pool; replay() runs graph 0, collective 0 (eagerly, RCCL on the current stream), graph
    1, ... So a rank's update costs a handful of graph launches plus its all-reduces instead of
    ~250 Python-issued kernels, and no collective is ever inside a captured graph."""

    def __init__(self):
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs, self.ops = [], []
        self._ctx = None

    def _begin(self):
        g = torch.cuda.CUDAGraph()
        self._ctx = torch.cuda.graph(g, pool=self.pool, capture_error_mode="thread_local")
        self._ctx.__enter__()
        self.graphs.append(g)

    def _cut(self, op):
        self._ctx.__exit__(None, None, None)
        self.ops.append(op)
        self._begin()

    def reset(self):
        """Free every captured graph now (idempotent)."""
        graphs, self.graphs, self.ops = self.graphs, [], []
        for g in graphs:
            g.reset()

    def replay(self):
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.ops):
                self.ops[i]()


_SEG = {"active": None, "force": False}


def force_graph_segments(on: bool) -> None:
    """Test switch: cut update graphs at their collectives even with one rank."""
    _SEG["force"] = bool(on)


def graph_segments_wanted() -> bool:
    return world_size() > 1 or _SEG["force"]


class capturing:
    """Context: capture the enclosed update into `seg` (GraphSegments)."""

    def __init__(self, seg: GraphSegments):
        self.seg = seg

    def __enter__(self):
        self._gc = gc.isenabled()
        _SEG["active"] = self.seg
        try:
            self.seg._begin()
        except BaseException:
            _SEG["active"] = None
            raise
        gc.disable()  # as cuda_graph: no collection while a segment captures (only once it began)
        return self.seg

    def __exit__(self, *exc):
        try:
            self.seg._ctx.__exit__(*exc)
        finally:
            self.seg._ctx = None
            _SEG["active"] = None
            if self._gc:
                gc.enable()
        return False


def segment_capture_active() -> bool:
    return _SEG["active"] is not None


def _allreduce_now(t, average):
    if world_size() > 1:
        dist.all_reduce(t)
        if average:
            t.div_(world_size())
    return t


def allreduce_(t: torch.Tensor, average: bool = False) -> torch.Tensor:
    seg = _SEG["active"]
    if seg is not None:
        seg._cut(lambda: _allreduce_now(t, average))
        return t
    return _allreduce_now(t, average)


def allreduce_grads(params) -> None:
    """Average the .grad of `params` across ranks with a single flat all-reduce."""
    seg = _SEG["active"]
    if seg is not None:
        # the gradient tensors the captured graphs write, bound now: another capture (the other
        # branch of the update) re-points p.grad at tensors of its own memory pool
        grads = [p.grad for p in params if p.grad is not None]
        seg._cut(lambda: _allreduce_tensors_now(grads))
        return
    _allreduce_tensors_now([p.grad for p in params if p.grad is not None])


def _allreduce_tensors_now(grads) -> None:
    if world_size() <= 1:
        return
    if not grads:
        return
    flat = torch._utils._flatten_dense_tensors(grads)
    dist.all_reduce(flat)
    flat.div_(world_size())
    for g, f in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
        g.copy_(f)


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Make every rank start from rank `src`'s parameters and buffers."""
    if world_size() <= 1:
        return
    tensors = [p.data for p in module.parameters()] + [b for b in module.buffers()]
    flat = torch._utils._flatten_dense_tensors(tensors)
    dist.broadcast(flat, src)
    for t, f in zip(tensors, torch._utils._unflatten_dense_tensors(flat, tensors)):
        t.copy_(f)


def max_over_ranks(x: float) -> float:
    if world_size() <= 1:
        return float(x)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float) -> float:
    if world_size() <= 1:
        return float(x)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return float(t.item())
