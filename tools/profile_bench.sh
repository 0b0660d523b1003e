#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (profiles/ gets the stats CSV).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps ${BENCH_STEPS:-5} --warmup ${BENCH_WARMUP:-2} --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo "rocprof rc=$?"
find gpurun_out/prof -name "*stats*" | head
