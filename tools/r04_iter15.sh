#!/bin/bash
# Relaxed arrivals without agent-scope fences (row-kernel partial sums as coherent atomic stores,
# the head's draw counter): GPU tests, then a bench A/B against the fenced build (exp_libs/fenced)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_policy_head_rng.py tests/test_gpu_trainer.py tests/test_gpu_mlp3.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it15_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it15_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/head_bench.py 2>&1 | grep case
for v in relaxed fenced relaxed fenced relaxed fenced; do
  lib=""; [ $v = fenced ] && lib="MSACL_HIP_LIB=$PWD/exp_libs/fenced/libmsacl_hip.so"
  env $lib timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/ab_bench.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_bench.log').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
done
