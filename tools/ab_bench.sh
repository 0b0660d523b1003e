#!/bin/bash
# bench.py A/B on one box: alternates the default and "$AB_FLAG" (bench flags) / "$AB_ENV"
# (environment assignments, e.g. MSACL_FUSED_BACKWARD=1) ${AB_REPS:-3} times each,
# writes gpurun_out/ab_bench.json (value, ms_per_step and phases per run).
mkdir -p gpurun_out
: > gpurun_out/ab_bench.jsonl
for i in $(seq ${AB_REPS:-3}); do
  for arm in A B; do
    m=""; envs=""
    [ $arm = B ] && { m="$AB_FLAG"; envs="$AB_ENV"; }
    env $envs timeout -k 10 240 python bench.py --steps ${AB_STEPS:-40} --warmup 5 --no-cpu-baseline $m > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    tail -1 gpurun_out/ab_run.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'flags': '$m $envs'.strip() or 'default', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'phases': d['phases'], 'policy_us': d['kernels'].get('policy_forward', {}).get('avg_us'), 'rollout_us': d['kernels']['rollout_step']['avg_us']}))" | tee -a gpurun_out/ab_bench.jsonl
  done
done
