#!/bin/bash
# bench line (default) and the hover variant with the emission timed on the last warm-up horizon
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05_b3.log 2>&1 || { tail -5 gpurun_out/r05_b3.log; exit 1; }
tail -1 gpurun_out/r05_b3.log > gpurun_out/r05_bench_v3.json
timeout -k 10 600 python bench.py --policy hover --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r05_hover2.log 2>&1 \
  || { tail -5 gpurun_out/r05_hover2.log; exit 1; }
tail -1 gpurun_out/r05_hover2.log > gpurun_out/r05_bench_hover_v2.json
for f in gpurun_out/r05_bench_v3.json gpurun_out/r05_bench_hover_v2.json; do python3 -c "
import json
d = json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['windows_per_step'], json.dumps(d['kernels']['emit_horizon'])[:200], d['roofline']['traffic'])"; done
