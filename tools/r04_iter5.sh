#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp3.py -m gpu -x -q --timeout 200 --timeout-method thread -rf > gpurun_out/it5_tests.log 2>&1
rc=$?; tail -4 gpurun_out/it5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/mlp3_bench.py --reps 50 > gpurun_out/mlp3_bench.jsonl 2> gpurun_out/mlp3_bench.err; rc=$?
cat gpurun_out/mlp3_bench.jsonl; [ $rc -eq 0 ] || { tail -20 gpurun_out/mlp3_bench.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/it5_bench.log 2>&1; rc=$?
tail -1 gpurun_out/it5_bench.log | cut -c1-300; exit $rc
