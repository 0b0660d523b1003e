#!/bin/bash
# Horizon emission with cooperative (line-contiguous) ring reads (MH_EMIT_COOP=1, the build) vs one
# record per lane (exp_libs/sample_fused-nocoop): emission tests, emission time vs window count per
# trainer step (tools/probes/emit_scan.py), bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_horizon.py \
  tests/test_gpu_sampler_oracle.py > gpurun_out/ecoop_tests.log 2>&1
rc=$?; echo "tests: $(tail -1 gpurun_out/ecoop_tests.log)"; [ $rc -eq 0 ] || exit $rc
for v in coop nocoop coop nocoop; do
  if [ $v = coop ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 300 python tools/probes/emit_scan.py > gpurun_out/ecoop_scan_$v.jsonl 2> gpurun_out/ecoop_scan_$v.err \
    || { tail -5 gpurun_out/ecoop_scan_$v.err; exit 1; }
  python3 -c "
import json
rows=[json.loads(l) for l in open('gpurun_out/ecoop_scan_$v.jsonl') if l.startswith('{')]
w=sum(r['windows_hdr'] for r in rows)/len(rows); c=sum(r['emit_us_cold'] for r in rows)/len(rows); h=sum(r['emit_us_warm'] for r in rows)/len(rows)
print('scan $v', len(rows), 'steps; mean windows', round(w), 'cold us', round(c,2), 'warm us', round(h,2))"
done
for r in 1 2; do
for v in coop nocoop; do
  if [ $v = coop ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/sample_fused-$v/libmsacl_hip.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ecoop_bench_$v.log 2>&1 || { tail -5 gpurun_out/ecoop_bench_$v.log; exit 1; }
  tail -1 gpurun_out/ecoop_bench_$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); e = d['kernels'].get('emit_horizon') or {}; print('bench $v', d['value'], d['ms_per_step'], e.get('avg_us'), e.get('windows'), e.get('frac'))"
done
done
