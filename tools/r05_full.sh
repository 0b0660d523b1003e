#!/bin/bash
# Full GPU suite + smoke at HEAD (round-end record)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r05_gpu_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/r05_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.txt 2>&1
rc=$?; tail -3 gpurun_out/r05_smoke.txt; exit $rc
