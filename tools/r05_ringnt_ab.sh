#!/bin/bash
# cache policy of the fused kernel's ring-record stores (MH_RING_STORE_CPOL): fused-horizon tests
# on the variant, bench lines alternating, then one trace per variant (fused + emission times)
set -o pipefail
mkdir -p gpurun_out
MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-nt/libmsacl_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_fused_horizon.py > gpurun_out/nt_tests.log 2>&1
rc=$?; tail -1 gpurun_out/nt_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in base nt sc1; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/nt_ab.log 2>&1 || { tail -5 gpurun_out/nt_ab.log; exit 1; }
  tail -1 gpurun_out/nt_ab.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms'], d['kernels']['sample_fused']['avg_us_per_horizon'])"
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base nt; do
  if [ $v = base ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-$v/libmsacl_hip.so; fi
  rm -rf gpurun_out/prof_$v
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o bench --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$v.log 2>&1 || { tail -5 gpurun_out/prof_$v.log; exit 1; }
  echo "== $v"; grep -E "k_sample_fused|k_emit_cells" "$(find gpurun_out/prof_$v -name '*kernel_stats.csv' | head -1)" | cut -d, -f1-4
done
