#!/bin/bash
# One GPU session: gpu tests, smoke, short bench. Stops at the first crash-class exit status
# (fault/abort/segv/timeout); a plain test failure (rc 1) does not stop the later steps.
mkdir -p gpurun_out
run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests smoke bench"}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 840 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf ;;
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py --steps ${BENCH_STEPS:-10} --warmup ${BENCH_WARMUP:-3} ;;
    hover) run bench_hover 900 python bench.py --steps ${BENCH_STEPS:-10} --warmup ${BENCH_WARMUP:-3} --policy hover --no-cpu-baseline ;;
  esac
done
