#!/bin/bash
# bench's live fused-kernel timing (one launch per measurement) vs the rocprofv3 average of the same run
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
  python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-4m > gpurun_out/fh_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/fh_bench.log; exit $rc; }
grep '^{"metric"' gpurun_out/fh_bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['kernels']['sample_fused']['avg_us_per_horizon'], d['roofline']['frac'])"
grep k_sample_fused "$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1)" | cut -c1-120
