#!/bin/bash
# Round 5, fused sampler restructure: bit-exactness of the fused path (fused-horizon + sampler-oracle
# tests on the in-tree build = the new sources), then the kernel's device time A/B against the
# round-4 library (exp_libs/fused-base) with tools/fused_ab.py, alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_horizon.py tests/test_gpu_sampler_oracle.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -rf > gpurun_out/r05_it1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_it1_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base new base new; do
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/fused_ab.py --reps 5 --rounds 3 \
    > gpurun_out/r05_it1_ab.log 2>&1 || { tail -5 gpurun_out/r05_it1_ab.log; exit 1; }
  tail -1 gpurun_out/r05_it1_ab.log | cut -c1-300
done
