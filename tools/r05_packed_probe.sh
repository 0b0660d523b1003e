#!/bin/bash
# Fragment-ordered weight addresses (MH_MLP_EXP_PACKED: wrong values, the packed copy's access
# pattern) against the shipped row-major loads, standalone at the bench's shapes
set -o pipefail
mkdir -p gpurun_out
for v in base packed base packed; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/mlp_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/mlp3_bench.py --reps 50 > gpurun_out/packed_probe_$v.log 2>&1 || { tail -5 gpurun_out/packed_probe_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/packed_probe_$v.log | grep kernel | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['kernel'], d.get('M'), d.get('N3'), d.get('groups', ''), d.get('us'))"
done
