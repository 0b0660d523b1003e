#!/bin/bash
# Forward row-tile count for the update's other fused-MLP shapes (tools/mlp3_bench.py)
set -o pipefail
mkdir -p gpurun_out
C="5120,16,1,1,2;5120,16,1,0,2;5120,12,8,1,1;5376,12,256,0,1;5120,16,1,1,4;2560,12,8,1,1;20480,12,256,1,1"
for rt in 2 3 1; do
  echo "== MH_MLP_RT=$rt"
  MH_MLP_RT=$rt timeout -k 10 120 python tools/mlp3_bench.py --cases "$C" > gpurun_out/rt3b_$rt.log 2>&1 || { tail -5 gpurun_out/rt3b_$rt.log; exit 1; }
  grep k_mlp3_fwd gpurun_out/rt3b_$rt.log | cut -c1-140
done
