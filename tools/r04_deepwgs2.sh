#!/bin/bash
# Deep-product workgroup target (MH_DEEP_WGS) in the concurrent update: standalone weight-gradient
# times, then a bench A/B of 128 vs 96 vs 64
set -o pipefail
mkdir -p gpurun_out
for w in 128 96 64; do
  MH_DEEP_WGS=$w timeout -k 10 120 python tools/mlp3_bench.py --cases "10240,12,256,1,1;5120,16,1,1,1" > gpurun_out/dw_$w.log 2>&1 || { tail -5 gpurun_out/dw_$w.log; exit 1; }
  echo "MH_DEEP_WGS=$w $(grep weight_grads gpurun_out/dw_$w.log | tr '\n' ' ' | cut -c1-300)"
done
for cfg in "MH_DEEP_WGS=128" "MH_DEEP_WGS=96" "MH_DEEP_WGS=64" "MH_DEEP_WGS=128" "MH_DEEP_WGS=96" "MH_DEEP_WGS=64"; do
  env $cfg timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
