set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fused_ab5.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_horizon.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_f5.log 2>&1; rc=$?; tail -2 gpurun_out/t_f5.log; [ $rc -eq 0 ] || exit $rc
for v in prev build prev build; do
  if [ $v = build ]; then unset MSACL_HIP_LIB; else export MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so; fi
  timeout -k 10 120 python tools/fused_ab.py 2> gpurun_out/fused_ab_$v.err | grep '^{' | sed "s/^{/{\"v\": \"$v\", /" >> gpurun_out/fused_ab5.jsonl || { echo "fail $v"; tail -5 gpurun_out/fused_ab_$v.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/fused_ab5.jsonl'):
    d=json.loads(l); print(d['v'], d['us_per_horizon'], d['all_us'])
"
