#!/bin/bash
# Fused sampler cost attribution at the round's final sources: parts compiled out (garbage
# results, timing only), fused kernel us per horizon, two rounds
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for v in base noenv nopol nodma nosync nomfma; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py --reps 5 > gpurun_out/attrib_fab.log 2>&1 || { tail -5 gpurun_out/attrib_fab.log; exit 1; }
  echo "fused $v $(tail -1 gpurun_out/attrib_fab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_horizon"], d["all_us"])')"
done
done
