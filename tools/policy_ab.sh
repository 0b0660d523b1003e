#!/bin/bash
# policy-forward kernel A/B on one box: the fused-policy numerics test, then bench.py with the
# split-bf16 layer-2 kernel (default) and with the all-f32 kernel (MH_POLICY_KERNEL=f32).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy_mlp.py -x -q --timeout 200 --timeout-method thread -k "fused" > gpurun_out/pm.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pm.log; exit 1; }
tail -2 gpurun_out/pm.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_x6.log 2>&1 || exit 1
MH_POLICY_KERNEL=f32 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_f32.log 2>&1 || exit 1
python - <<'PY'
import json
for f in ("gpurun_out/b_x6.log", "gpurun_out/b_f32.log"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["kernels"]["policy_forward"]["avg_us"], d["phases"])
PY
