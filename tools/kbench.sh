#!/bin/bash
# Kernel microbenchmarks (tools/kernel_bench.py) and their rocprofv3 kernel-trace summary.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kprof
timeout -k 10 600 python3 tools/kernel_bench.py --out gpurun_out/kernel_bench.json > gpurun_out/kernel_bench.log 2>&1
rc=$?; echo "kernel_bench rc=$rc"; tail -n 40 gpurun_out/kernel_bench.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof -o kb --output-format csv -- python3 tools/kernel_bench.py > gpurun_out/kprof.log 2>&1
echo "rocprof rc=$?"
