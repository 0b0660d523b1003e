set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_env.py tests/test_gpu_nstep.py tests/test_gpu_sampling.py tests/test_gpu_offpolicy.py tests/test_gpu_onpolicy.py tests/test_gpu_trainer.py tests/test_gpu_policy_mlp.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -15 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/b2.log 2>&1; rc=$?; tail -1 gpurun_out/b2.log | cut -c1-2500; exit $rc
