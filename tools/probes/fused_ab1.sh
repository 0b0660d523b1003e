set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fused_ab.jsonl
true
true
for v in noenv nomfma serial build; do
  if [ $v = build ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py >> gpurun_out/fused_ab.jsonl 2> gpurun_out/fused_ab_$v.err || { echo "fail $v"; tail -5 gpurun_out/fused_ab_$v.err; exit 1; }
done
unset MSACL_HIP_LIB
cat gpurun_out/fused_ab.jsonl
bash tools/fused_pmc.sh && bash tools/update_trace.sh && PROF=1 BENCH_STEPS=20 bash tools/r03_iter.sh
