#!/bin/bash
# policy_bench.py with every library under exp_libs/ (tools/ab_libs.sh build ...), twice, alternating.
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for i in 1 2; do
  for d in "$ROOT"/exp_libs/*/; do
    n=$(basename "$d")
    MSACL_HIP_LIB="$d/libmsacl_hip.so" timeout -k 10 120 python "$ROOT/tools/policy_bench.py" 65536 50 | sed "s/^/$n: /" || exit 1
  done
done
