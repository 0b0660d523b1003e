#!/bin/bash
# One GPU call: rocprofv3 kernel trace (+stats) of the bench command, then the FETCH_SIZE and
# WRITE_SIZE PMC passes of the same command (separate runs, no trace domains with --pmc).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
  python3 bench.py --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-5} --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/prof_bench.log; exit $rc; }
tail -1 gpurun_out/prof_bench.log | cut -c1-400
python3 tools/trace_split.py "$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)" gpurun_out/trace_split.csv
bash tools/pmc.sh
