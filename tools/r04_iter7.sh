#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_fused_horizon.py tests/test_gpu_sampler_oracle.py tests/test_gpu_nstep.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it7_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it7_tests.log; [ $rc -eq 0 ] || exit $rc
MH_MLP_BWD_RT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp3.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > gpurun_out/rt_tests2.log 2>&1
rc=$?; tail -2 gpurun_out/rt_tests2.log; [ $rc -eq 0 ] || exit $rc
for rt in 1 2; do
  MH_MLP_BWD_RT=$rt timeout -k 10 200 python tools/mlp3_bench.py --reps 50 2> gpurun_out/rt.err | grep -v k_mlp3_fwd | sed "s/^/BWD_RT=$rt /" || { tail -5 gpurun_out/rt.err; exit 1; }
done
for cfg in "MSACL_MLP3_WIDE=0" "MSACL_MLP3_WIDE=1" "MH_MLP_BWD_RT=1" "MSACL_MLP3_WIDE=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'], d['kernels']['emit_horizon']['avg_us'])"
done
