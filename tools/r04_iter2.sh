set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in build poldma; do
    if [ $v = build ]; then L=""; else L="MSACL_HIP_LIB=exp_libs/fused-$v/libmsacl_hip.so"; fi
    env $L timeout -k 10 200 python tools/fused_ab.py --reps 5 --rounds 2 > gpurun_out/ab_one.log 2>&1 || { tail -5 gpurun_out/ab_one.log; exit 1; }
    tail -1 gpurun_out/ab_one.log >> gpurun_out/it2_ab.jsonl
  done
done
cut -c1-200 gpurun_out/it2_ab.jsonl
PROF=1 bash tools/r03_iter.sh
