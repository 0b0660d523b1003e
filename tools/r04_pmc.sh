#!/bin/bash
# PMC traffic passes of the bench command (FETCH_SIZE, WRITE_SIZE in separate runs), then the
# summary into profiles/r04_pmc_traffic_v3.json
set -o pipefail
mkdir -p gpurun_out
bash tools/pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out gpurun_out/r04_pmc_traffic_v3.json
