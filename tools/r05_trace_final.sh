#!/bin/bash
# Kernel trace + stats of the bench command at the round's final sources (step timeline, trace split)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
  python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof_bench.log; exit $rc; }
tail -1 gpurun_out/prof_bench.log > gpurun_out/r05_bench_final_prof.json
python3 tools/trace_split.py "$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)" gpurun_out/trace_split.csv
python3 tools/step_timeline.py "$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)" gpurun_out/step_timeline.txt
cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/kernel_stats.csv
head -24 gpurun_out/step_timeline.txt
