set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_fused_horizon.py tests/test_gpu_msacl_bench.py tests/test_gpu_msacl.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it3_tests.log 2>&1; rc=$?; tail -8 gpurun_out/it3_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04_iter2.sh
