#!/bin/bash
# Bench A/B: the fused sampler with policy waves at issue priority 1 (exp_libs/fused-prio1) vs base
set -o pipefail
mkdir -p gpurun_out
for v in base prio1 base prio1 base prio1; do
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['kernels']['sample_fused']['avg_us_per_horizon'])"
done
