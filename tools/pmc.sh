#!/bin/bash
# HBM traffic of the bench's kernels from rocprofv3 PMC counters, one counter per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass; no trace domains here).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$c
  timeout -k 10 900 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o pmc --output-format csv -- \
    python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1
  rc=$?
  echo "pmc $c rc=$rc"
  [ $rc -ne 0 ] && { tail -20 gpurun_out/pmc_$c.log; exit $rc; }
done
find gpurun_out/pmc_* -name "*counter_collection*"
