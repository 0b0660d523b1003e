#!/bin/bash
# Emission-only relaunch entry (mh_sample_horizon_emit): its test and the fused-horizon tests, a
# short bench line (kernels.emit_horizon at the trainer's window count), then PMC passes (v3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused_horizon.py tests/test_capi.py -m "gpu or not gpu" -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/it18_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it18_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/it18_bench.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/it18_bench.log; exit $rc; }
python3 -c "
import json; d=json.loads(open('gpurun_out/it18_bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['windows_per_step'], json.dumps(d['kernels']['emit_horizon'])[:300])"
bash tools/r04_pmc.sh
