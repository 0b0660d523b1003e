set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fused_ab.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_grouped.py tests/test_gpu_linear_backward.py tests/test_gpu_adam.py tests/test_gpu_msacl_bench.py tests/test_gpu_msacl.py tests/test_gpu_policy_mlp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_upd.log 2>&1; rc=$?; tail -3 gpurun_out/t_upd.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b1.log 2>&1; rc=$?; tail -1 gpurun_out/b1.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for v in build nopol noenv nomfma serial; do
  if [ $v = build ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py >> gpurun_out/fused_ab.jsonl 2> gpurun_out/fused_ab_$v.err || { echo "fail $v"; tail -5 gpurun_out/fused_ab_$v.err; exit 1; }
done
unset MSACL_HIP_LIB
cat gpurun_out/fused_ab.jsonl
bash tools/fused_pmc.sh && bash tools/update_trace.sh
