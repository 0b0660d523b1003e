#!/bin/bash
# SQ counters of k_rollout<QuadTracking> for each exp_libs/ variant (cost attribution).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-base NO_POLAR NO_DESIRED NO_SAMPLE NO_SUBSTEPS NO_RESET}; do
  echo "== $v"
  MSACL_HIP_LIB="$GRAFT_REPO_ROOT/exp_libs/$v/libmsacl_hip.so" bash tools/pmc_sq_rollout.sh | tail -1
done
