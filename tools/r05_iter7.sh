#!/bin/bash
# Round 5: the sampler-oracle QuadTracking case on the in-tree build, then TACC + kernel A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler_oracle.py -m gpu -q --timeout 300 --timeout-method thread -rf \
  > gpurun_out/r05_it8_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r05_it8_tests.log; [ $rc -eq 0 ] || exit $rc
MSACL_HIP_LIB=$PWD/exp_libs/fused-tacc3/libmsacl_hip.so timeout -k 10 120 python tools/probes/fused_tacc.py \
  2> gpurun_out/r05_tacc3.err > gpurun_out/r05_tacc3.json || { tail -5 gpurun_out/r05_tacc3.err; exit 1; }
tr -d '\n' < gpurun_out/r05_tacc3.json; echo
VARIANTS="base new2 new3 mfma16 base new2 new3 mfma16" bash tools/r05_iter3.sh
