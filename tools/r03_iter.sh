#!/bin/bash
# One GPU iteration: selected GPU tests, a bench line, then a rocprofv3 kernel trace of the same
# bench command (stats + per-grid split). Stops at the first failing step.
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread -rf \
    > gpurun_out/iter_tests.log 2>&1; rc=$?; tail -6 gpurun_out/iter_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-5} --no-cpu-baseline ${BENCH_ARGS} \
  > gpurun_out/iter_bench.log 2>&1; rc=$?; tail -1 gpurun_out/iter_bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
    python3 bench.py --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-5} --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/prof_bench.log 2>&1; rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/trace_split.py "$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)" gpurun_out/trace_split.csv
  python3 tools/step_timeline.py "$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)" gpurun_out/step_timeline.txt && head -25 gpurun_out/step_timeline.txt
fi
