"""Content hash of the sources the lockstep kernel is built from, so a committed PMC traffic
summary (tools/pmc_summary.py) can be matched against the kernel a bench run executes: bench.py
reports `roofline.traffic` only when the summary's hash equals the current sources' hash."""
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd",
                    "csrc")
# the kernels' own sources and build flags (the C ABI glue in capi.hip changes no kernel's traffic)
ROLLOUT_SOURCES = ("rollout.hip", "env_math.h", "reset_draw.h", "philox.h", "Makefile",
                   "sample_fused.hip", "sample_fused.h", "policy_x3.h", "policy_mlp.hip")


def rollout_sources_sha(names=ROLLOUT_SOURCES) -> str:
    h = hashlib.sha256()
    for n in names:
        with open(os.path.join(CSRC, n), "rb") as f:
            h.update(n.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]
