#!/bin/bash
# Item-parallel horizon emission: the fused-horizon / sampler / n-step parity tests, the emission
# scan probe (emission time vs window count), then the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_horizon.py \
  tests/test_gpu_sampler_oracle.py tests/test_gpu_nstep.py tests/test_gpu_trainer.py > gpurun_out/emit1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/emit1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/probes/emit_scan.py > gpurun_out/emit_scan2.log 2>&1 || { tail -5 gpurun_out/emit_scan2.log; exit 1; }
grep '^{' gpurun_out/emit_scan2.log | head -12 | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/emit1_bench.log 2>&1 || { tail -5 gpurun_out/emit1_bench.log; exit 1; }
tail -1 gpurun_out/emit1_bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms'])"
