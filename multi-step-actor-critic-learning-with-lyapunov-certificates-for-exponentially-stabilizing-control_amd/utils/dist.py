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
import ctypes
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


# live side streams: id(stream) -> (hipStream_t handle, device index). Not weak references: a
# weakref to a torch.cuda.Stream was seen returning an unrelated object after the stream died
# (its referent not cleared on this image), so each stream unregisters itself when it is freed.
_SIDE_STREAMS: "dict[int, tuple[int, int]]" = {}


class _SideStream(torch.cuda.Stream):
    def __del__(self):
        _SIDE_STREAMS.pop(id(self), None)


def side_stream(device) -> "torch.cuda.Stream":
    """A new stream for work forked off the current stream inside an update (twin critics, the
    critic / Lyapunov branches, the stability advantage). Registered, so that a capture ending
    with one of them still forked is caught (cuda_graph, GraphSegments) instead of reaching
    hipStreamEndCapture with a dangling branch."""
    s = _SideStream(device=device)
    _SIDE_STREAMS[id(s)] = (int(s.cuda_stream), int(s.device.index))
    return s


def unjoined_forks(join: bool = True):
    """The registered side streams that take part in the current stream's capture with work the
    current stream does not (transitively) wait for: forks never joined back
    (mh_capture_unjoined walks the captured graph's dependencies). Returns their hipStream_t
    handles. join=True makes the current stream wait for each of them, so the capture can still
    end with a well-formed graph."""
    cur = torch.cuda.current_stream()
    handles = [h for h, d in list(_SIDE_STREAMS.values()) if d == cur.device.index]
    if not handles:
        return []
    from .. import _native as N
    arr = (ctypes.c_void_p * len(handles))(*handles)
    out = (ctypes.c_int32 * len(handles))()
    N.check(N.lib().mh_capture_unjoined(ctypes.c_void_p(cur.cuda_stream), arr, len(handles), out),
            "mh_capture_unjoined")
    bad = [h for h, u in zip(handles, out) if u]
    if join:
        for h in bad:
            cur.wait_stream(torch.cuda.ExternalStream(h, device=cur.device))
    return bad


class UnjoinedForkError(RuntimeError):
    pass


class NestedForkError(RuntimeError):
    pass


def _unjoined_message(bad):
    return (f"HIP graph capture ended with {len(bad)} forked stream(s) not joined back to the capture "
            f"stream ({', '.join(hex(h) for h in bad)}): every side-stream branch must end "
            f"with current_stream().wait_stream(side) before the capture ends (the graph was joined "
            f"and discarded)")


# hipStream_t of the stream each active capture began on (innermost last)
_CAPTURE_ORIGIN: "list[int]" = []


@contextlib.contextmanager
def fork(side):
    """Run the enclosed work on `side`, forked off the current stream (side waits for it); the
    caller joins it later with current_stream().wait_stream(side). During a capture the fork must
    come from the capture's own stream: a fork of a fork (a stream forked from a side stream, even
    when every branch is joined back) makes hipStreamEndCapture crash on this ROCm
    (tools/probes/capture_unjoined_probe.py, mode nested_joined: SIGSEGV), so it is
    refused with NestedForkError before anything is enqueued."""
    cur = torch.cuda.current_stream(side.device)
    if _CAPTURE_ORIGIN and torch.cuda.is_current_stream_capturing() and int(cur.cuda_stream) != _CAPTURE_ORIGIN[-1]:
        raise NestedForkError(
            f"fork of stream {hex(int(cur.cuda_stream))} inside a HIP graph capture that began on "
            f"{hex(_CAPTURE_ORIGIN[-1])}: forks of forks are refused (hipStreamEndCapture crashes on them); "
            f"fork from the capture stream instead")
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        yield side


@contextlib.contextmanager
def cuda_graph(g, **kw):
    """torch.cuda.graph with the cyclic garbage collector paused while the stream captures, and
    with the capture's forks checked before it ends.

    gc: torch.cuda.graph collects once before the capture, but an allocation inside the capture
    can trigger another collection, which may finalise graphs, events or streams of pipelines that
    died in reference cycles: HIP calls that are illegal during a capture (seen as aborts and a
    host segfault in a later replay during one full test session).

    forks ("capture hygiene"): a registered side stream (side_stream) whose captured work
    the capture stream does not wait for would end the capture with a dangling branch; the check
    joins such streams, lets the capture end, discards the graph and raises UnjoinedForkError (the
    same join runs when the body raised, so the capture always ends on a well-formed graph).
    Forks of forks are refused earlier, by fork()."""
    was = gc.isenabled()
    gc.disable()
    bad = []
    try:
        with torch.cuda.graph(g, **kw):
            _CAPTURE_ORIGIN.append(int(torch.cuda.current_stream().cuda_stream))
            try:
                yield
            finally:
                _CAPTURE_ORIGIN.pop()
                bad = unjoined_forks(join=True)
    finally:
        if was:
            gc.enable()
    if bad:
        g.reset()
        raise UnjoinedForkError(_unjoined_message(bad))


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
        _CAPTURE_ORIGIN.append(int(torch.cuda.current_stream().cuda_stream))
        self.graphs.append(g)

    def _end(self):
        _CAPTURE_ORIGIN.pop()
        bad = unjoined_forks(join=True)
        ctx, self._ctx = self._ctx, None
        ctx.__exit__(None, None, None)
        if bad:
            self.reset()
            raise UnjoinedForkError(_unjoined_message(bad))

    def _cut(self, op):
        self._end()
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


# Collectives inside the captured update graph (RCCL supports stream capture): opt-in with
# MSACL_GRAPH_COLLECTIVES=1 on the nccl (RCCL) backend. The update is then ONE graph at any world
# size (no segment cuts, the trainer's graphed step applies). `force`: issue the collectives even
# with one rank (a world-size-1 process group: the one-GPU rehearsal of the data-parallel step).
_COLL = {"in_graph": os.environ.get("MSACL_GRAPH_COLLECTIVES", "0") == "1", "force": False}


def set_graph_collectives(on: bool) -> None:
    _COLL["in_graph"] = bool(on)


def force_collectives(on: bool) -> None:
    """Issue the gradient collectives even when the (initialised) process group has one rank."""
    _COLL["force"] = bool(on)


def collectives_active() -> bool:
    """The update's gradient / statistics all-reduces are issued (world > 1, or forced)."""
    return world_size() > 1 or (_COLL["force"] and is_initialized())


def collectives_in_graph() -> bool:
    return _COLL["in_graph"] and collectives_active() and is_initialized() and dist.get_backend() == "nccl"


def graph_segments_wanted() -> bool:
    return _SEG["force"] or (collectives_active() and not collectives_in_graph())


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
            if exc[0] is None:
                self.seg._end()
            elif self.seg._ctx is not None:
                _CAPTURE_ORIGIN.pop()
                unjoined_forks(join=True)  # end the capture on a well-formed graph, then re-raise
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
    if collectives_active():
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
    if not collectives_active():
        return
    if not grads:
        return
    flat = torch._utils._flatten_dense_tensors(grads)
    dist.all_reduce(flat)
    flat.div_(world_size())
    for g, f in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
        g.copy_(f)


# count of parameter writes that torch's version counters do not see (copies through .data,
# kernels writing parameter storage through raw pointers outside an optimiser): every such writer
# calls parameters_written(), and caches of parameter values (the sampler's packed policy) compare it
_PARAM_EPOCH = [0]


def parameters_written() -> None:
    _PARAM_EPOCH[0] += 1


def param_epoch() -> int:
    return _PARAM_EPOCH[0]


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Make every rank start from rank `src`'s parameters and buffers."""
    if world_size() <= 1:
        return
    parameters_written()  # (written through .data below: invisible to the version counters)
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
