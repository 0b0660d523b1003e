#!/bin/bash
# Policy pack launches (k_policy_scales: 32 workgroups x 8 waves, one W2 row per wave; k_policy_pack_x3:
# one thread per fragment pair and lane, 16-byte loads and stores) vs HEAD before (exp_libs/old):
# policy / sampler parity tests, then the kernels' times from a kernel trace of a short bench run and bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_policy_mlp.py \
  tests/test_gpu_fused_horizon.py tests/test_gpu_sampler_oracle.py > gpurun_out/pack_tests.log 2>&1
rc=$?; tail -2 gpurun_out/pack_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${PROF_VARIANTS:-new old}; do
  if [ $v = new ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/old/libmsacl_hip.so; fi
  rm -rf gpurun_out/packprof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/packprof_$v -o p --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/packprof_$v.log 2>&1 || { tail -5 gpurun_out/packprof_$v.log; exit 1; }
  grep -h "policy_scales\|policy_pack" $(find gpurun_out/packprof_$v -name '*kernel_stats.csv') | cut -d, -f1-4 | sed "s/^/$v /"
done
unset MSACL_HIP_LIB
for r in $(seq 1 ${BENCH_ROUNDS:-2}); do
for v in new old; do
  if [ $v = new ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/old/libmsacl_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/pack_bench_$v.log 2>&1 || { tail -5 gpurun_out/pack_bench_$v.log; exit 1; }
  tail -1 gpurun_out/pack_bench_$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('bench $v', d['value'], d['ms_per_step'], d['phases']['sample_ms'])"
done
done
