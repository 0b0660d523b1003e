#!/bin/bash
# Fused forward row tiles (MH_MLP_RT 2 vs 1) in the concurrent update: bench A/B
set -o pipefail
mkdir -p gpurun_out
for cfg in "MH_MLP_RT=2" "MH_MLP_RT=1" "MH_MLP_RT=2" "MH_MLP_RT=1" "MH_MLP_RT=2" "MH_MLP_RT=1"; do
  env $cfg timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
