#!/bin/bash
# Forward row-tile count vs row count for the Lyapunov-shaped wide MLP (tools/mlp3_bench.py)
set -o pipefail
mkdir -p gpurun_out
C="8192,12,256,1,1;10240,12,256,1,1;12288,12,256,1,1;16384,12,256,1,1"
for rt in 2 3 4; do
  echo "== MH_MLP_RT=$rt"
  MH_MLP_RT=$rt timeout -k 10 120 python tools/mlp3_bench.py --cases "$C" > gpurun_out/rt3_$rt.log 2>&1 || { tail -5 gpurun_out/rt3_$rt.log; exit 1; }
  grep -v per_layer gpurun_out/rt3_$rt.log | cut -c1-140
done
