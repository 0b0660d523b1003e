"""Device-time measurement of back-to-back kernel launches with HIP events.

Events are recorded on torch's current stream (the stream every engine call is launched on).
Before the first event the stream is parked on a GPU spin long enough for the host to enqueue
every launch of the batch, so the two events bracket device execution only (no host launch
latency between kernels) — the same quantity rocprofv3's kernel trace reports per dispatch,
plus the ~1 us dispatch gaps between consecutive kernels.
"""
from __future__ import annotations

import torch

CLOCK_HZ = 2.4e9  # torch.cuda._sleep counts shader clock cycles (8.3 ms for 2e7 measured)


def time_launches(fn, reps: int = 20, host_us_per_call: float = 60.0, warm: int = 1) -> float:
    """Average device milliseconds per call of `fn` (which only enqueues GPU work)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    spin = int(max(2e-3, 2.0 * reps * host_us_per_call * 1e-6) * CLOCK_HZ)
    torch.cuda._sleep(spin)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps
