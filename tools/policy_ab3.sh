#!/bin/bash
# policy-forward kernels on one box: numerics of the default (split-f16, 8 waves) kernel and of
# the 4-wave variant, the microbenchmark of every variant, then bench.py with the default.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy_mlp.py -x -q --timeout 200 --timeout-method thread -k "fused_policy" > gpurun_out/pm.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pm.log; exit 1; }
tail -1 gpurun_out/pm.log
MH_POLICY_WAVES=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_policy_mlp.py -x -q --timeout 200 --timeout-method thread -k "fused_policy" > gpurun_out/pm4.log 2>&1 || { echo "pytest (4 waves) failed"; tail -40 gpurun_out/pm4.log; exit 1; }
tail -1 gpurun_out/pm4.log
for k in "x3 8" "x3 4" "x6 4" "f32 4"; do
  set -- $k
  MH_POLICY_KERNEL=$1 MH_POLICY_WAVES=$2 timeout -k 10 120 python tools/policy_bench.py 65536 50 | sed "s/^/waves=$2 /" || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_x3.log 2>&1 || exit 1
tail -1 gpurun_out/b_x3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernels']['policy_forward'], d['phases'])"
