set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1; rc=$?; tail -3 gpurun_out/full_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/full_bench.log 2>&1; rc=$?; tail -1 gpurun_out/full_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
PROF=1 BENCH_STEPS=20 bash tools/r03_iter.sh && bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out gpurun_out/pmc_traffic.json
