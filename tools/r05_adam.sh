#!/bin/bash
# float4 Adam / Polyak units: the optimiser and MSACL parity tests, then the bench line + timeline
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_adam.py \
  tests/test_gpu_msacl.py tests/test_gpu_msacl_bench.py tests/test_algorithms.py tests/test_gpu_trainer.py \
  > gpurun_out/adam_tests.log 2>&1
rc=$?; tail -3 gpurun_out/adam_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/adam_bench.log 2>&1 || { tail -5 gpurun_out/adam_bench.log; exit 1; }
tail -1 gpurun_out/adam_bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
  python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof_bench.log; exit $rc; }
python3 tools/step_timeline.py "$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)" gpurun_out/step_timeline.txt
cp "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" gpurun_out/kernel_stats.csv
grep -E "k_adam|k_polyak" gpurun_out/kernel_stats.csv | cut -c1-160
