#!/bin/bash
# One bench line (emission window trace), then the PMC traffic passes of the bench command
# (tools/pmc.sh: FETCH_SIZE, WRITE_SIZE in separate passes) summarised per kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05_pmcb.log 2>&1 || { tail -5 gpurun_out/r05_pmcb.log; exit 1; }
tail -1 gpurun_out/r05_pmcb.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['kernels']['emit_horizon']))"
bash tools/pmc.sh && python3 tools/pmc_summary.py gpurun_out gpurun_out/r05_pmc_traffic_v1.json && \
  python3 -c "
import json
d = json.load(open('gpurun_out/r05_pmc_traffic_v1.json'))
for k in ('sample_fused', 'emit_horizon', 'replay_gather'):
    print(k, json.dumps(d.get(k))[:300])"
