#!/bin/bash
# The round's late changes end to end: bench lines alternating between this tree and the tree at
# 15bcf8c (exp_tree/, its own library build), three rounds on one box
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
for v in head start; do
  if [ $v = head ]; then d=.; else d=exp_tree; fi
  (cd $d && timeout -k 10 300 python bench.py --no-cpu-baseline) > gpurun_out/sess_bench.log 2>&1 || { tail -5 gpurun_out/sess_bench.log; exit 1; }
  tail -1 gpurun_out/sess_bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); k = d['kernels']['sample_fused']; print('bench $v', d['value'], d['ms_per_step'], k['avg_us_per_horizon'], d['phases']['replay_and_update_ms_policy_free_policy'])"
done
done
