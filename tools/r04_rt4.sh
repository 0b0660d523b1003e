#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for rt in 2 4; do
  MH_MLP_RT=$rt timeout -k 10 300 python tools/mlp3_bench.py --reps 40 2> gpurun_out/rt.err | grep k_mlp3_fwd | sed "s/^/RT=$rt /" || { tail -5 gpurun_out/rt.err; exit 1; }
done
timeout -k 10 300 python tools/mlp3_bench.py --reps 40 2> gpurun_out/rt.err | grep -v k_mlp3_fwd || { tail -5 gpurun_out/rt.err; exit 1; }
