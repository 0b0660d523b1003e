#!/bin/bash
# Late round-5 record at HEAD: full GPU suite + smoke, then the PMC traffic passes of the bench command
set -o pipefail
mkdir -p gpurun_out
bash tools/r05_full.sh || exit $?
bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out gpurun_out/r05_pmc_traffic_v2.json && \
  python3 -c "
import json
d = json.load(open('gpurun_out/r05_pmc_traffic_v2.json'))
for k in ('sample_fused', 'emit_horizon', 'replay_gather'):
    print(k, json.dumps(d.get(k) or d.get('kernels', {}).get(k))[:300])"
