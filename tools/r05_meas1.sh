#!/bin/bash
# Round 5 measurements: (1) all six env steps at 65,536 and 4,194,304 envs at HEAD with SURVEY §8(d)'s
# bytes beside the builder's (tools/kernel_bench.py); (2) QuadTracking's 4 M-env step and rollout
# kernels, round-3 sources (cb29cf2) vs HEAD, alternating; (3) the hover bench variant
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/kernel_bench.py --skip rollout,gather,msacl,policy,gae --out gpurun_out/r05_env_step_4m.json \
  > gpurun_out/r05_env_step.log 2>&1 || { tail -5 gpurun_out/r05_env_step.log; exit 1; }
cat gpurun_out/r05_env_step.log | cut -c1-260
for i in 1 2; do
  for d in exp_libs/rev-* exp_libs/work; do
    n=$(basename $d)
    MSACL_HIP_LIB=$PWD/$d/libmsacl_hip.so timeout -k 10 300 python tools/kernel_bench.py --envs QuadTracking --sizes 4194304 \
      --skip gather,msacl,policy,gae > gpurun_out/r05_ab4m_${n}_$i.log 2>&1 || { tail -5 gpurun_out/r05_ab4m_${n}_$i.log; exit 1; }
    python -c "
import json,sys
for l in open('gpurun_out/r05_ab4m_${n}_$i.log'):
    if l.startswith('{'):
        d=json.loads(l); d['lib']='$n'; d['round']=$i; print(json.dumps(d))" | tee -a gpurun_out/r05_rollout_4m_ab.jsonl | cut -c1-200
  done
done
timeout -k 10 600 python bench.py --policy hover --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r05_hover.log 2>&1 \
  || { tail -5 gpurun_out/r05_hover.log; exit 1; }
tail -1 gpurun_out/r05_hover.log > gpurun_out/r05_bench_hover.json; cut -c1-300 gpurun_out/r05_bench_hover.json
