#!/bin/bash
# Round 5: the full GPU suite on the in-tree build, then the TACC accounting and the kernel A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf \
  > gpurun_out/r05_it7_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r05_it7_tests.log; [ $rc -eq 0 ] || exit $rc
MSACL_HIP_LIB=$PWD/exp_libs/fused-tacc3/libmsacl_hip.so timeout -k 10 120 python tools/probes/fused_tacc.py \
  2> gpurun_out/r05_tacc3.err > gpurun_out/r05_tacc3.json || { tail -5 gpurun_out/r05_tacc3.err; exit 1; }
tr -d '\n' < gpurun_out/r05_tacc3.json; echo
VARIANTS="base new2 new3 base new2 new3" bash tools/r05_iter3.sh
