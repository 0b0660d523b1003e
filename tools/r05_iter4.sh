#!/bin/bash
# Round 5: per-segment cycle accounting of the fused kernel's policy passes (register-accumulated
# s_memtime deltas, tools/probes/fused_tacc.py), with and without env waves, + their kernel times
set -o pipefail
mkdir -p gpurun_out
for v in noenv_tacc tacc; do
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/probes/fused_tacc.py \
    2> gpurun_out/r05_tacc_$v.err > gpurun_out/r05_tacc_$v.json || { tail -5 gpurun_out/r05_tacc_$v.err; exit 1; }
  echo "== $v"; tr -d '\n' < gpurun_out/r05_tacc_$v.json; echo
done
VARIANTS="tacc new noenv_tacc noenv" bash tools/r05_iter3.sh
