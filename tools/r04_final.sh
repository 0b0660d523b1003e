#!/bin/bash
# Round-end record: the whole GPU suite, smoke(), then the PMC traffic passes of the bench command
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/final_tests.log 2>&1
rc=$?; tail -4 gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/final_smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04_pmc.sh
