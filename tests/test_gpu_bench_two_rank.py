"""GPU: bench.py's multi-rank path end to end (torch.distributed.run, 2 ranks, barrier +
max-over-ranks timing, world-size-scaled value, the data-parallel MSACL update with its graph
cut at the merged all-reduces). RCCL refuses two ranks on one device, so this rehearsal runs the
gloo backend (MSACL_DIST_BACKEND=gloo) with both ranks on GPU 0; the 8-GPU RCCL run is the
driver's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo_rehearsal():
    env = dict(os.environ, MSACL_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints exactly one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and out["value"] > 0
    # the launch self-check: both ranks counted by an all-reduce over the data-path backend
    assert out["dist_backend"] == "gloo" and out["rccl_ranks"] == 2
    # value = env-steps of BOTH ranks over the max-over-ranks time
    assert abs(out["value"] - 2 * 65536 * 20 * 2 / (out["ms_per_step"] * 2 / 1e3)) / out["value"] < 0.01


def test_bench_rank_count_mismatch_fails():
    """--gpus that disagrees with the process group: bench.py exits non-zero before timing."""
    env = dict(os.environ, MSACL_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29519", os.path.join(ROOT, "bench.py"),
           "--gpus", "3", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "counted 2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
