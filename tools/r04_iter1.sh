set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_fused_horizon.py tests/test_gpu_sampler_oracle.py tests/test_gpu_msacl_bench.py tests/test_gpu_msacl.py tests/test_gpu_policy_mlp.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it1_tests.log 2>&1; rc=$?; tail -8 gpurun_out/it1_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in build poldma; do
    if [ $v = build ]; then L=""; else L="MSACL_HIP_LIB=exp_libs/fused-$v/libmsacl_hip.so"; fi
    env $L timeout -k 10 200 python tools/fused_ab.py --reps 5 --rounds 2 >> gpurun_out/it1_ab.jsonl 2>/dev/null || exit 1
  done
done
tail -4 gpurun_out/it1_ab.jsonl | cut -c1-200
PROF=1 bash tools/r03_iter.sh
