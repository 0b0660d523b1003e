#!/bin/bash
# Graphed step with the policy pack skipped after policy-free updates: trainer tests, then bench
# lines against the previous HEAD (exp_libs/old is the same kernels; the change is Python-side, so
# the A/B is MSACL_PACK_A (this tree) vs the tree at HEAD~ checked out beside it under exp_tree/)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_trainer.py \
  > gpurun_out/pskip_tests.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/pskip_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pskip_tests.log; exit $rc; }
for r in 1 2; do
for v in new old; do
  if [ $v = new ]; then d=.; else d=exp_tree; fi
  (cd $d && timeout -k 10 300 python bench.py --no-cpu-baseline) > gpurun_out/pskip_bench.log 2>&1 || { tail -5 gpurun_out/pskip_bench.log; exit 1; }
  tail -1 gpurun_out/pskip_bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('bench $v', d['value'], d['ms_per_step'], d['phases']['host_enqueue_ms_per_step'])"
done
done
