#!/bin/bash
# weight-ring depth variants of the fused MLP kernels (MH_MLP_PF), standalone, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for v in base pf3 pf2; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/mlp_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/mlp3_bench.py --reps 30 > gpurun_out/pf_$v.log 2>&1 || { tail -5 gpurun_out/pf_$v.log; exit 1; }
  echo "== $v $(grep kernel gpurun_out/pf_$v.log | python3 -c "
import sys, json
print(' '.join(f\"{d['kernel'][:9]}{d.get('M')}/{d.get('N3')}/{d.get('groups', '')}={d.get('us')}\" for d in map(json.loads, sys.stdin) if d['kernel'] in ('k_mlp3_fwd', 'k_mlp3_bwd')))")"
done
done
