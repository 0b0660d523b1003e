#!/bin/bash
# bench.py --policy hover A/B of the working tree vs an older tree in $AB_TREE (git archive, engine
# built in place), alternating ${AB_REPS:-3} times on one box: gpurun_out/ab_hover.jsonl
mkdir -p gpurun_out
: > gpurun_out/ab_hover.jsonl
ROOT=$(pwd)
for i in $(seq ${AB_REPS:-3}); do
  for arm in head old; do
    d=$ROOT; [ $arm = old ] && d=$ROOT/$AB_TREE
    (cd "$d" && timeout -k 10 240 python bench.py --policy hover --steps ${AB_STEPS:-40} --warmup 5 --no-cpu-baseline) > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    tail -1 gpurun_out/ab_run.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'tree': '$arm', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'windows_per_step': d.get('windows_per_step'), 'phases': d['phases']}))" | tee -a gpurun_out/ab_hover.jsonl
  done
done
