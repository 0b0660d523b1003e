#!/bin/bash
# Round-5 closing record after the Python-side step changes (kernel sources unchanged since
# r05_pmc_traffic_v3): full GPU suite + smoke, the default bench line with the CPU-baseline leg
set -o pipefail
mkdir -p gpurun_out
bash tools/r05_full.sh || exit $?
timeout -k 10 900 python bench.py > gpurun_out/final_bench.log 2>&1
rc=$?; tail -1 gpurun_out/final_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/final_bench.log > gpurun_out/r05_bench_final.json
