#!/bin/bash
# weight-gradient chunk prefetch distance (MH_DEEP_AHEAD1): gemm + MLP tests on the variant,
# standalone kernel times, then bench lines alternating
set -o pipefail
mkdir -p gpurun_out
MSACL_HIP_LIB=$PWD/exp_libs/gemm-ahead1/libmsacl_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_mlp3.py > gpurun_out/deep_tests.log 2>&1
rc=$?; tail -1 gpurun_out/deep_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base ahead1; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/gemm-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/mlp3_bench.py --reps 30 > gpurun_out/deep_$v.log 2>&1 || { tail -5 gpurun_out/deep_$v.log; exit 1; }
  echo "== $v $(grep weight_grads gpurun_out/deep_$v.log | python3 -c "
import sys, json
print(' '.join(f\"{d.get('M')}/{d.get('N3')}={d.get('us')}\" for d in map(json.loads, sys.stdin)))")"
done
for r in 1 2; do
for v in base ahead1; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/gemm-$v/libmsacl_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/deep_ab.log 2>&1 || { tail -5 gpurun_out/deep_ab.log; exit 1; }
  tail -1 gpurun_out/deep_ab.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms'])"
done
done
