#!/bin/bash
# A/B of mh_gemm_f32 per update shape between exp_libs/* (tools/ab_libs.sh build): device time
# of tools/gemm_shapes.py with each library.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for d in "$ROOT"/exp_libs/*; do
  n=$(basename "$d")
  MSACL_HIP_LIB="$d/libmsacl_hip.so" timeout -k 10 200 python3 "$ROOT/tools/gemm_shapes.py" > "$ROOT/gpurun_out/gab_$n.log" 2>&1
  echo "== $n"; grep '"M"' "$ROOT/gpurun_out/gab_$n.log" | python3 -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r['M'], r['N'], r['K'], r['ta'], r['tb'], 'hip', r['hip_us'], 'blas', r['blas_us'])"
done
