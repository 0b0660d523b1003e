#!/bin/bash
# Fused sampler's tail without agent-scope fences: fused-horizon tests on the default build, then
# the kernel's device time vs the fenced tail (tools/fused_ab.py), then a bench A/B
set -o pipefail
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_horizon.py tests/test_gpu_sampler_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base tailfenced base tailfenced; do
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/fused_ab.py --reps 5 --rounds 3 > gpurun_out/tail_ab.log 2>&1 || { tail -5 gpurun_out/tail_ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/tail_ab.log').read().strip().splitlines()[-1]); print('$v', d['us_per_horizon'], d['all_us'])"
done
