#!/bin/bash
# Layer 3 on 16x16x32 (row-half W3 layout): parity tests, per-segment cycles (TACC builds) of the old and new pass, and the fused kernel
# time of fold-schedule variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_horizon.py \
  tests/test_gpu_sampler_oracle.py tests/test_gpu_policy_mlp.py > gpurun_out/l3b_tests.log 2>&1
rc=$?; tail -3 gpurun_out/l3b_tests.log; [ $rc -eq 0 ] || exit $rc
for v in old-tacc sample_fused-tacc sample_fused-k2x3tacc; do
  MSACL_HIP_LIB=$PWD/exp_libs/$v/libmsacl_hip.so timeout -k 10 120 python tools/probes/fused_tacc.py > gpurun_out/l3b_tacc_$v.log 2>&1 \
    || { tail -5 gpurun_out/l3b_tacc_$v.log; exit 1; }
  echo "tacc $v $(tail -1 gpurun_out/l3b_tacc_$v.log)"
done
for r in 1 2; do
for v in new old sample_fused-k2x3 sample_fused-k2x4; do
  if [ $v = new ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py --reps 5 > gpurun_out/l3b_fab_$v.log 2>&1 || { tail -5 gpurun_out/l3b_fab_$v.log; exit 1; }
  echo "fused $v $(tail -1 gpurun_out/l3b_fab_$v.log | cut -c1-160)"
done
done
for r in 1 2; do
for v in new old; do
  if [ $v = new ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/old/libmsacl_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/l3b_bench_$v.log 2>&1 || { tail -5 gpurun_out/l3b_bench_$v.log; exit 1; }
  tail -1 gpurun_out/l3b_bench_$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('bench $v', d['value'], d['ms_per_step'], d['kernels']['sample_fused']['avg_us_per_horizon'])"
done
done
