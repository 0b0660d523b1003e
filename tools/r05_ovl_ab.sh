#!/bin/bash
# trainer_overlap_sampling A/B at HEAD (alternating runs on one box)
set -o pipefail
mkdir -p gpurun_out
for m in "--overlap" "" "--overlap" ""; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $m > gpurun_out/ovl_ab.log 2>&1 || { tail -5 gpurun_out/ovl_ab.log; exit 1; }
  tail -1 gpurun_out/ovl_ab.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); print('overlap' if '$m' else 'serial', d['value'], d['ms_per_step'])"
done
