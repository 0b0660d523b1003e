#!/bin/bash
# Fused sampler layer-2 step order: two output blocks interleaved (MH_FUSED_ILV) vs block-major:
# fused-horizon tests on the variant (bit-identical to the lockstep kernels), fused kernel time
set -o pipefail
mkdir -p gpurun_out
MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-ilv/libmsacl_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_fused_horizon.py > gpurun_out/ilv_tests.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/ilv_tests.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
for v in base ilv; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py --reps 5 > gpurun_out/ilv_fab.log 2>&1 || { tail -5 gpurun_out/ilv_fab.log; exit 1; }
  echo "fused $v $(tail -1 gpurun_out/ilv_fab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_horizon"], d["all_us"])')"
done
done
