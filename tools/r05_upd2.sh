#!/bin/bash
# Replay draw inside the update graph: the buffer / trainer / MSACL parity tests, then the bench
# line, the host-overhead probe and a kernel trace with the step timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nstep.py \
  tests/test_gpu_trainer.py tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_gpu_offpolicy.py \
  tests/test_gpu_per.py > gpurun_out/upd2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/upd2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/upd2_bench.log 2>&1
rc=$?; tail -1 gpurun_out/upd2_bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/probes/update_host.py > gpurun_out/update_host2.log 2>&1
rc=$?; tail -2 gpurun_out/update_host2.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
  python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof_bench.log; exit $rc; }
python3 tools/step_timeline.py "$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)" gpurun_out/step_timeline.txt
cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/kernel_stats.csv
