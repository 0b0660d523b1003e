#!/bin/bash
cd "$GRAFT_REPO_ROOT"
for n in "$@"; do
  for r in 1 2; do
    timeout -k 10 120 python -u tools/probes/fused_determinism_probe.py $n 2>&1 | grep "vs" || exit 1
  done
done
