#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp3.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > gpurun_out/rt_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rt_tests.log; [ $rc -eq 0 ] || exit $rc
MH_MLP_BWD_RT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp3.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > gpurun_out/rt_tests2.log 2>&1
rc=$?; tail -3 gpurun_out/rt_tests2.log; [ $rc -eq 0 ] || exit $rc
for rt in 1 2; do
  MH_MLP_BWD_RT=$rt timeout -k 10 200 python tools/mlp3_bench.py --reps 50 2> gpurun_out/rt.err | grep -v k_mlp3_fwd | sed "s/^/BWD_RT=$rt /" || { tail -5 gpurun_out/rt.err; exit 1; }
done
