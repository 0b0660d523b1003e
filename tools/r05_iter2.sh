#!/bin/bash
# Round 5: s_memtime stamps of the restructured fused kernel's policy passes (with and without
# the env waves), per-phase cycle breakdown (tools/probes/fused_stamps.py)
set -o pipefail
mkdir -p gpurun_out
for v in noenv_stamps stamps; do
  echo "== stamps $v"
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/probes/fused_stamps.py \
    2> gpurun_out/r05_stamps_$v.err > gpurun_out/r05_stamps_$v.json || { tail -5 gpurun_out/r05_stamps_$v.err; exit 1; }
  tr -d '\n' < gpurun_out/r05_stamps_$v.json; echo
done
for v in noenv new; do
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/fused_ab.py --reps 5 --rounds 3 \
    > gpurun_out/r05_it2_ab.log 2>&1 || { tail -5 gpurun_out/r05_it2_ab.log; exit 1; }
  tail -1 gpurun_out/r05_it2_ab.log | cut -c1-200
done
