#!/bin/bash
mkdir -p gpurun_out
for v in 0 1 2 4 7; do
  echo "== variant $v"
  MSACL_HIP_LIB=$PWD/exp_libs/lib_exp$v.so timeout -k 10 300 python3 tools/kernel_bench.py --envs QuadTracking --sizes 65536,1048576 --skip gather,msacl > gpurun_out/exp_$v.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/exp_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/exp_$v.log
done
