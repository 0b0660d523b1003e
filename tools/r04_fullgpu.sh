#!/bin/bash
# the whole GPU suite and the smoke, as the driver runs them at round end
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/full_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/full_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; exit $rc
