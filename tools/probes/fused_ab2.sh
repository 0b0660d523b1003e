set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fused_ab2.jsonl
for v in noenv noenv_nosync noenv_nodma nosync build; do
  if [ $v = build ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py 2> gpurun_out/fused_ab_$v.err | grep '^{' >> gpurun_out/fused_ab2.jsonl || { echo "fail $v"; tail -5 gpurun_out/fused_ab_$v.err; exit 1; }
done
unset MSACL_HIP_LIB
cut -c1-200 gpurun_out/fused_ab2.jsonl
LIBS="noenv=$PWD/exp_libs/fused-noenv/libmsacl_hip.so" bash tools/fused_pmc.sh
