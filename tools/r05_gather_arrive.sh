#!/bin/bash
# Replay gather on a flat chunked grid (one workgroup per GATHER_CHUNK vectors of one output) vs
# the previous fixed (x, 9) grid (exp_libs/old): the replay/trainer GPU tests on the new library,
# then k_gather's average duration in a short bench run per library (K = 4 default, 2, 8), then
# alternating bench lines new/old
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_nstep.py tests/test_gpu_trainer.py > gpurun_out/garr_tests.log 2>&1
rc=$?; tail -2 gpurun_out/garr_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in new old rollout-k2 rollout-k8; do
  if [ $v = new ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/$v/libmsacl_hip.so; fi
  rm -rf gpurun_out/garr_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/garr_$v -o p --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/garr_$v.log 2>&1 || { tail -5 gpurun_out/garr_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
for r in csv.DictReader(open(glob.glob(f'gpurun_out/garr_{v}/*kernel_stats.csv')[0])):
    if 'k_gather' in r['Name']:
        print(v, r['Name'][:30], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us')
PY
done
unset MSACL_HIP_LIB
for r in 1 2; do
for v in new old; do
  if [ $v = new ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/old/libmsacl_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/garr_bench_$v.log 2>&1 || { tail -5 gpurun_out/garr_bench_$v.log; exit 1; }
  tail -1 gpurun_out/garr_bench_$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('bench $v', d['value'], d['ms_per_step'], d['phases']['replay_and_update_ms_policy_free_policy'])"
done
done
