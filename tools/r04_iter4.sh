#!/bin/bash
# r04: fused-MLP kernels with the enforced load ring + policy-DMA sampler default.
# GPU tests of the touched paths, then bench A/B (fused MLP on / per-layer), then a traced bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_mlp3.py tests/test_gpu_fused_horizon.py tests/test_gpu_msacl.py \
  tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it4_tests.log 2>&1
rc=$?; tail -8 gpurun_out/it4_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/it4_ab.txt
for r in 1 2; do
  for m in 1 0; do
    MSACL_MLP3=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1 \
      || { tail -5 gpurun_out/ab_bench.log; exit 1; }
    echo "MLP3=$m $(tail -1 gpurun_out/ab_bench.log | cut -c1-160)" >> gpurun_out/it4_ab.txt
  done
done
cat gpurun_out/it4_ab.txt
PROF=1 bash tools/r03_iter.sh
