#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_fused_horizon.py tests/test_gpu_nstep.py tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_mlp3.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it9_tests.log 2>&1
rc=$?; tail -2 gpurun_out/it9_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in build nots; do
  if [ $v = build ]; then L=""; else L="MSACL_HIP_LIB=exp_libs/sample_fused-$v/libmsacl_hip.so"; fi
  env $L timeout -k 10 200 python tools/fused_ab.py --reps 5 --rounds 2 > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
  tail -1 gpurun_out/ab_one.log | cut -c1-200
done; done
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'], d['kernels']['emit_horizon']['avg_us'], d['kernels']['sample_fused']['avg_us_per_horizon'])"
done
for w in 256 512 1024; do
  MH_DEEP_WGS=$w timeout -k 10 200 python tools/mlp3_bench.py --reps 50 2> gpurun_out/rt.err | grep weight_grads | sed "s/^/WGS=$w /" || { tail -5 gpurun_out/rt.err; exit 1; }
done
