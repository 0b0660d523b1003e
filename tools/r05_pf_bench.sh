#!/bin/bash
# MLP weight-ring depth variants: standalone kernels, then the bench alternating
set -o pipefail
mkdir -p gpurun_out
for v in base pf2t2 pft2; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/mlp_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/mlp3_bench.py --reps 30 > gpurun_out/pf_$v.log 2>&1 || { tail -5 gpurun_out/pf_$v.log; exit 1; }
  echo "== $v $(grep kernel gpurun_out/pf_$v.log | python3 -c "
import sys, json
print(' '.join(f\"{d['kernel'][7:10]}{d.get('M')}/{d.get('N3')}/{d.get('groups', '')}={d.get('us')}\" for d in map(json.loads, sys.stdin) if d['kernel'] in ('k_mlp3_fwd', 'k_mlp3_bwd')))")"
done
for r in 1 2; do
for v in base pf2 pf2t2; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/mlp_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/pfb.log 2>&1 || { tail -5 gpurun_out/pfb.log; exit 1; }
  tail -1 gpurun_out/pfb.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms'])"
done
done
