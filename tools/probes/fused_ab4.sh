set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fused_ab4.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_horizon.py tests/test_gpu_sampler_oracle.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_f4.log 2>&1; rc=$?; tail -2 gpurun_out/t_f4.log; [ $rc -eq 0 ] || exit $rc
for v in build noenv; do
  if [ $v = build ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py 2> gpurun_out/fused_ab_$v.err | grep '^{' | sed "s/^{/{\"v\": \"$v\", /" >> gpurun_out/fused_ab4.jsonl || { echo "fail $v"; tail -5 gpurun_out/fused_ab_$v.err; exit 1; }
done
unset MSACL_HIP_LIB
cut -c1-140 gpurun_out/fused_ab4.jsonl
bash tools/probes/fused_stamps.sh > gpurun_out/stamps4.log 2>&1; grep -v created gpurun_out/stamps4.log | grep -v "global seed"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/b4.log 2>&1; tail -1 gpurun_out/b4.log | cut -c1-200
