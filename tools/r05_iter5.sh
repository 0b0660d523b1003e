#!/bin/bash
# Round 5: fused-path parity on the in-tree build, then kernel time A/B (base = round 4, new = the
# first restructure, new2 = + compile-time logits store, zero-C first MFMAs, bias reads ahead of
# the ring reads) and the register-accumulated segment accounting of new2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy_mlp.py tests/test_gpu_sampler_oracle.py tests/test_gpu_fused_horizon.py -m gpu -q \
  --timeout 300 --timeout-method thread -rf > gpurun_out/r05_it6_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_it6_tests.log; [ $rc -eq 0 ] || exit $rc
MSACL_HIP_LIB=$PWD/exp_libs/fused-tacc3/libmsacl_hip.so timeout -k 10 120 python tools/probes/fused_tacc.py \
  2> gpurun_out/r05_tacc3.err > gpurun_out/r05_tacc3.json || { tail -5 gpurun_out/r05_tacc3.err; exit 1; }
tr -d '\n' < gpurun_out/r05_tacc3.json; echo
VARIANTS="new2 new3 new2 new3" bash tools/r05_iter3.sh
