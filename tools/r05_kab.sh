#!/bin/bash
# Generic kernel A/B against exp_libs/old (the previous HEAD build): $TESTS on the new library, then
# rocprofv3 kernel stats of a short bench run per library for kernels matching $KPAT, then
# $BENCH_ROUNDS alternating bench lines
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/kab_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/kab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in new old; do
  if [ $v = new ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/old/libmsacl_hip.so; fi
  rm -rf gpurun_out/kabprof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kabprof_$v -o p --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/kabprof_$v.log 2>&1 || { tail -5 gpurun_out/kabprof_$v.log; exit 1; }
  python3 - "$v" "$KPAT" <<'PY'
import csv, glob, re, sys
v, pat = sys.argv[1], sys.argv[2]
f = glob.glob(f'gpurun_out/kabprof_{v}/*kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    if re.search(pat, r['Name']):
        print(v, r['Name'][:48], r['Calls'], round(float(r['AverageNs']) / 1e3, 2), 'us')
PY
done
unset MSACL_HIP_LIB
for r in $(seq 1 ${BENCH_ROUNDS:-2}); do
for v in new old; do
  if [ $v = new ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/old/libmsacl_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/kab_bench_$v.log 2>&1 || { tail -5 gpurun_out/kab_bench_$v.log; exit 1; }
  tail -1 gpurun_out/kab_bench_$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print('bench $v', d['value'], d['ms_per_step'], d['phases']['sample_ms'], d['phases']['replay_and_update_ms_policy_free_policy'])"
done
done
