#!/bin/bash
# One GPU session, parameterised (the single driver for GPU calls; records go to gpurun_out/):
#   STEPS="tests smoke bench"   which steps, in order (also: hover, capture_probe, prof, pmc)
#   TESTS="tests/x.py ..."      test files for `tests` (default: the whole -m gpu suite)
#   BENCH_STEPS / BENCH_WARMUP / BENCH_ARGS   bench.py arguments
#   TAG                          suffix of the log names (default: none)
# Stops at the first crash-class exit status (fault/abort/segv/timeout) and at a failing test run.
mkdir -p gpurun_out
TAG=${TAG:+_$TAG}
run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name$TAG.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 5 "gpurun_out/$name$TAG.log" | cut -c1-3000
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests smoke bench"}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -x --timeout 300 --timeout-method thread -rf -p no:cacheprovider ;;
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-5} ${BENCH_ARGS:---no-cpu-baseline} ;;
    hover) run bench_hover 900 python bench.py --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-5} --policy hover --no-cpu-baseline ;;
    capture_probe) run capture_probe 300 python -u tools/probes/capture_unjoined_probe.py ;;
    prof) run prof 600 bash tools/profile_bench.sh ;;
    pmc) run pmc 900 bash tools/pmc.sh ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
