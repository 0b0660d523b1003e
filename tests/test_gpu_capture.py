"""HIP-graph capture hygiene (utils/dist.py cuda_graph / GraphSegments, mh_capture_unjoined).

The update is captured with work forked onto side streams (twin critics, the critic / Lyapunov
branches, the policy step's stability advantage: RL/algorithm/msacl.py:174-224 is the update being
captured). A fork that is not joined back before the capture ends leaves a dangling branch; the
guard detects it from the captured graph's dependencies, joins it, lets the capture end, discards
the graph and raises UnjoinedForkError, instead of handing hipStreamEndCapture that state.
"""
import pytest
import torch

import msacl_amd  # noqa: F401
import msacl_amd.utils.dist as D

pytestmark = pytest.mark.gpu


def _fork(side, fn):
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()


def test_joined_fork_captures_and_replays():
    side = D.side_stream(torch.device("cuda"))
    x = torch.zeros(4096, device="cuda")
    y = torch.zeros(4096, device="cuda")
    g = torch.cuda.CUDAGraph()
    with D.cuda_graph(g):
        x.add_(1.0)
        _fork(side, lambda: y.add_(2.0))
        x.mul_(3.0)
        torch.cuda.current_stream().wait_stream(side)  # joined
        x.add_(y)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    # x <- 3 (x + 1) + y, y <- y + 2, three times from zero
    xr = yr = 0.0
    for _ in range(3):
        yr += 2.0
        xr = 3.0 * (xr + 1.0) + yr
    assert torch.all(x == xr) and torch.all(y == yr)


def test_unjoined_fork_raises_instead_of_ending_the_capture():
    side = D.side_stream(torch.device("cuda"))
    x = torch.zeros(4096, device="cuda")
    y = torch.zeros(4096, device="cuda")
    g = torch.cuda.CUDAGraph()
    with pytest.raises(D.UnjoinedForkError, match="not joined back"):
        with D.cuda_graph(g):
            x.add_(1.0)
            _fork(side, lambda: y.add_(2.0))  # never joined
            x.mul_(3.0)
    # the stream and the device are usable afterwards: eager work and a new capture
    assert not torch.cuda.is_current_stream_capturing()
    x.fill_(1.0)
    g2 = torch.cuda.CUDAGraph()
    with D.cuda_graph(g2):
        x.add_(1.0)
    g2.replay()
    torch.cuda.synchronize()
    assert torch.all(x == 2.0)


def test_unjoined_fork_in_a_graph_segment_raises():
    side = D.side_stream(torch.device("cuda"))
    x = torch.zeros(1024, device="cuda")
    y = torch.zeros(1024, device="cuda")
    seg = D.GraphSegments()
    with pytest.raises(D.UnjoinedForkError):
        with D.capturing(seg):
            x.add_(1.0)
            _fork(side, lambda: y.add_(1.0))
    assert not torch.cuda.is_current_stream_capturing()
    assert not seg.graphs
    # a joined segment chain still works
    seg2 = D.GraphSegments()
    with D.capturing(seg2):
        x.add_(1.0)
        _fork(side, lambda: y.add_(1.0))
        torch.cuda.current_stream().wait_stream(side)
    x.zero_()
    y.zero_()
    seg2.replay()
    torch.cuda.synchronize()
    assert torch.all(x == 1.0) and torch.all(y == 1.0)


def test_unjoined_query_outside_a_capture_is_an_error():
    import msacl_amd._native as N
    import ctypes
    s = torch.cuda.current_stream()
    rc = N.lib().mh_capture_unjoined(ctypes.c_void_p(s.cuda_stream), None, 0, None)
    assert rc != 0


def test_nested_fork_is_refused_before_it_reaches_the_capture():
    """A fork of a fork (a stream forked from a side stream) is refused inside a capture: HIP's
    hipStreamEndCapture crashes on it even when every branch is joined back
    (tools/probes/capture_unjoined_probe.py, mode nested_joined: SIGSEGV). The refusal comes before
    the nested fork is enqueued, the open branch is joined, and the capture ends normally."""
    dev = torch.device("cuda")
    side, twin = D.side_stream(dev), D.side_stream(dev)
    x = torch.zeros(1024, device="cuda")
    g = torch.cuda.CUDAGraph()
    with pytest.raises(D.NestedForkError, match="forks of forks"):
        with D.cuda_graph(g):
            with D.fork(side):
                x.add_(1.0)
                with D.fork(twin):
                    x.add_(1.0)
    assert not torch.cuda.is_current_stream_capturing()
    # outside a capture nested forks are plain stream ordering
    x.zero_()
    with D.fork(side):
        x.add_(1.0)
        with D.fork(twin):
            x.add_(1.0)
        side.wait_stream(twin)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert torch.all(x == 2.0)
    # and two single-level forks from the capture stream are fine
    y = torch.zeros(1024, device="cuda")
    g2 = torch.cuda.CUDAGraph()
    with D.cuda_graph(g2):
        with D.fork(side):
            x.add_(1.0)
        with D.fork(twin):
            y.add_(1.0)
        cur = torch.cuda.current_stream()
        cur.wait_stream(side)
        cur.wait_stream(twin)
        x.add_(y)
    x.zero_()
    y.zero_()
    g2.replay()
    torch.cuda.synchronize()
    assert torch.all(x == 2.0) and torch.all(y == 1.0)
