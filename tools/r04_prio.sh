#!/bin/bash
# Policy waves at a higher issue priority than the env waves sharing their SIMDs (s_setprio,
# MH_FUSED_POLPRIO): fused-horizon tests on the variant, then the kernel's device time A/B
set -o pipefail
mkdir -p gpurun_out
MSACL_HIP_LIB=$PWD/exp_libs/fused-prio3/libmsacl_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_horizon.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/prio_tests.log 2>&1
rc=$?; tail -2 gpurun_out/prio_tests.log; [ $rc -eq 0 ] || exit $rc
for v in base prio3 prio1 base prio3 prio1; do
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/fused_ab.py --reps 5 --rounds 3 > gpurun_out/prio_ab.log 2>&1 || { tail -5 gpurun_out/prio_ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/prio_ab.log').read().strip().splitlines()[-1]); print('$v', d['us_per_horizon'], d['all_us'])"
done
