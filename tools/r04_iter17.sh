#!/bin/bash
# Deep-product target 128: the update's GPU tests, then the round-end bench record + profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_trainer.py tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it17_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it17_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04_record.sh
