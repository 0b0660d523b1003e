#!/bin/bash
# Fold-schedule variants of the fused sampler's last phase / layer 3 at the final sources
# (MH_FOLD_K3: pairs split per layer-3 block and VALU per MFMA group; MH_FOLD_K2: pairs per
# layer-2 step): fused-horizon tests on one variant, fused kernel time alternating
set -o pipefail
mkdir -p gpurun_out
MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-k3x8/libmsacl_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_fused_horizon.py > gpurun_out/fold_tests.log 2>&1
rc=$?; echo "tests k3x8: $(tail -1 gpurun_out/fold_tests.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in base k3x4 k3x8 k2x1; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py --reps 5 > gpurun_out/fold_fab.log 2>&1 || { tail -5 gpurun_out/fold_fab.log; exit 1; }
  echo "fused $v $(tail -1 gpurun_out/fold_fab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["us_per_horizon"], d["all_us"])')"
done
done
