#!/bin/bash
# bench.py A/B of two engine libraries on one box: the in-tree build vs $AB_LIB (e.g. a variant in
# exp_libs/), alternating ${AB_REPS:-3} times; gpurun_out/ab_lib.jsonl.
mkdir -p gpurun_out
: > gpurun_out/ab_lib.jsonl
for i in $(seq ${AB_REPS:-3}); do
  for arm in tree alt; do
    if [ $arm = alt ]; then export MSACL_HIP_LIB="$AB_LIB"; else unset MSACL_HIP_LIB; fi
    timeout -k 10 240 python bench.py --steps ${AB_STEPS:-40} --warmup 5 --no-cpu-baseline > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    tail -1 gpurun_out/ab_run.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'lib': '$arm', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'phases': d['phases']}))" | tee -a gpurun_out/ab_lib.jsonl
  done
done
unset MSACL_HIP_LIB
