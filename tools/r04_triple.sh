#!/bin/bash
# Triple-buffered W2 chunks in k_sample_fused (MH_FUSED_TRIPLE): bit-exactness of the fused-horizon
# tests on the variant library, then the kernel's device time A/B (tools/fused_ab.py)
set -o pipefail
mkdir -p gpurun_out
MSACL_HIP_LIB=$PWD/exp_libs/fused-triple/libmsacl_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_horizon.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/triple_tests.log 2>&1
rc=$?; tail -3 gpurun_out/triple_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base triple base triple; do
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/fused_ab.py --reps 5 --rounds 3 > gpurun_out/triple_ab.log 2>&1 || { tail -5 gpurun_out/triple_ab.log; exit 1; }
  tail -1 gpurun_out/triple_ab.log | cut -c1-300
done
