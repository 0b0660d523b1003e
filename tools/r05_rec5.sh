#!/bin/bash
# Round-5 closing record at HEAD (after the flat chunked replay gather): full GPU suite + smoke, the PMC traffic passes (v3, copied into
# profiles/ on the box so the bench line reads it), the default bench line with the CPU-baseline
# leg, and a kernel trace + stats of the bench command
set -o pipefail
mkdir -p gpurun_out
bash tools/r05_full.sh || exit $?
bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out gpurun_out/r05_pmc_traffic_v4.json || exit 1
cp gpurun_out/r05_pmc_traffic_v4.json profiles/
timeout -k 10 900 python bench.py > gpurun_out/final_bench.log 2>&1
rc=$?; tail -1 gpurun_out/final_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
tail -1 gpurun_out/final_bench.log > gpurun_out/r05_bench_final.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
  python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof_bench.log; exit $rc; }
tail -1 gpurun_out/prof_bench.log > gpurun_out/r05_bench_final_prof.json
python3 tools/trace_split.py "$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)" gpurun_out/trace_split.csv
python3 tools/step_timeline.py "$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)" gpurun_out/step_timeline.txt
cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/kernel_stats.csv
