mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py -x -v --timeout 300 --timeout-method thread -k "overlapped or train_loop" > gpurun_out/ov_tests.log 2>&1 || { tail -30 gpurun_out/ov_tests.log; exit 1; }
tail -3 gpurun_out/ov_tests.log
for m in "--overlap" "" "--overlap" ""; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline $m > gpurun_out/b_ov.log 2>&1 || exit 1
  tail -1 gpurun_out/b_ov.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value'], d['ms_per_step'], d['phases'])"
done
