#!/bin/bash
# determinism of the fused horizon (QuadTracking) for each exp_libs variant
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  echo "== $v"
  MSACL_HIP_LIB=$PWD/exp_libs/$v/libmsacl_hip.so timeout -k 10 120 python -u tools/probes/fused_determinism_probe.py QuadTracking 2>&1 | grep "vs" || exit 1
done
