"""What hipStreamEndCapture does with a fork that was never joined back, WITHOUT the engine's guard
(utils/dist.py cuda_graph). Runs the raw torch.cuda.graph capture in a child process (it may crash)
and reports how it ended: a Python error (the runtime returned hipErrorStreamCaptureUnjoined) or a
signal. Usage: python tools/probes/capture_unjoined_probe.py [joined|unjoined|unjoined_kernel]
(parent mode runs all three children)."""
import subprocess
import sys

CHILD = r"""
import sys, torch
mode = sys.argv[1]
side = torch.cuda.Stream()
twin = torch.cuda.Stream()
x = torch.zeros(4096, device="cuda"); y = torch.zeros(4096, device="cuda")
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
print("capture begin", flush=True)
try:
    with torch.cuda.graph(g):
        x.add_(1.0)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            if mode != "unjoined_empty":
                y.add_(2.0)
            if mode.startswith("nested"):  # a fork of the fork (the twin critics inside a side branch)
                twin.wait_stream(side)
                with torch.cuda.stream(twin):
                    y.mul_(2.0)
                if mode != "nested_twin_unjoined":
                    side.wait_stream(twin)
        x.mul_(3.0)
        if mode in ("joined", "nested_joined", "nested_twin_unjoined"):
            torch.cuda.current_stream().wait_stream(side)
        print("capture end", flush=True)
    print("capture ended normally", flush=True)
    g.replay(); torch.cuda.synchronize()
    print("replayed: x[0] =", float(x[0]), "y[0] =", float(y[0]), flush=True)
except Exception as e:
    print("python error:", type(e).__name__, str(e).splitlines()[0][:300], flush=True)
"""


def main():
    modes = sys.argv[1:] or ["joined", "unjoined_empty", "unjoined", "nested_joined", "nested_unjoined",
                             "nested_twin_unjoined"]
    for m in modes:
        p = subprocess.run([sys.executable, "-c", CHILD, m], capture_output=True, text=True, timeout=120)
        out = (p.stdout + p.stderr).strip().splitlines()
        print(f"== {m}: exit {p.returncode}")
        for ln in out[-6:]:
            print("   ", ln[:300])


if __name__ == "__main__":
    main()
