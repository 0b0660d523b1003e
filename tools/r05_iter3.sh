#!/bin/bash
# Round 5: cost attribution of the restructured fused kernel (variants with parts compiled out,
# tools/fused_variants.sh), device time per horizon with tools/fused_ab.py
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-new burst nosync nodma nosyncdma nomfma nopol noenv new burst}; do
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/fused_ab.py --reps 5 --rounds 3 \
    > gpurun_out/r05_ab_$v.log 2>&1 || { tail -5 gpurun_out/r05_ab_$v.log; exit 1; }
  tail -1 gpurun_out/r05_ab_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['us_per_horizon'], d['all_us'], d['err_words'])" | tee -a gpurun_out/r05_ab.txt
done
