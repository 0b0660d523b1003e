#!/bin/bash
# Round-end record at HEAD: the whole GPU suite, smoke(), the bench with its CPU-baseline leg and
# a rocprofv3 kernel trace of the bench command (tools/r04_record.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread -rf > gpurun_out/final_tests.log 2>&1
rc=$?; tail -2 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04_record.sh
