#!/bin/bash
# The first policy step's forward chains inside the update's branches (stability advantage on the
# Lyapunov branch, policy head + critics' forward on the critic branch) vs HEAD before (exp_tree/):
# MSACL parity / graph-path / trainer tests, a kernel trace of the policy step, bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_msacl.py \
  tests/test_gpu_msacl_bench.py tests/test_gpu_trainer.py > gpurun_out/early_tests.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/early_tests.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/early_tests.log; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/early_prof
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/early_prof -o bench --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/early_prof.log 2>&1 || { tail -5 gpurun_out/early_prof.log; exit 1; }
python3 tools/step_timeline.py "$(find gpurun_out/early_prof -name '*kernel_trace.csv' | head -1)" gpurun_out/early_timeline.txt
head -24 gpurun_out/early_timeline.txt | tail -8
for r in 1 2 3; do
for v in new old; do
  if [ $v = new ]; then d=.; else d=exp_tree; fi
  (cd $d && timeout -k 10 300 python bench.py --no-cpu-baseline) > gpurun_out/early_bench.log 2>&1 || { tail -5 gpurun_out/early_bench.log; exit 1; }
  tail -1 gpurun_out/early_bench.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('bench $v', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms_policy_free_policy'])"
done
done
