#!/bin/bash
# Round 5 re-measure at HEAD: (1) the six env steps at 65,536 / 4,194,304 envs with SURVEY §8(d)'s
# bytes beside the builder's; (2) SQ instruction-mix counters of the TwoLink / SingleTrackCar 4 M
# env steps (three separate PMC passes, no trace domains): totals, then f64 vs f32 VALU by op kind;
# (3) the hover bench variant (emission-heavy), with k_emit_cells on a horizon that emits windows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/kernel_bench.py --skip rollout,gather,msacl,policy,gae --out gpurun_out/r05_env_step_4m.json \
  > gpurun_out/r05_env_step.log 2>&1 || { tail -5 gpurun_out/r05_env_step.log; exit 1; }
python3 -c "
import json
for d in json.load(open('gpurun_out/r05_env_step_4m.json')):
    if d['env_steps'] > 1e6: print(d['env'], d['avg_us'], d['survey_bytes_per_unit'], d['survey_frac'], d['bytes_per_unit'], d['frac'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
pass() {  # name, counters...
  local name=$1; shift
  rm -rf gpurun_out/pmc_$name
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o sq --output-format csv -- python3 tools/kernel_bench.py \
    --envs TwoLink,SingleTrackCar --sizes 4194304 --skip rollout,gather,msacl,policy,gae --reps 3 > gpurun_out/pmc_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || return $rc
  python3 tools/pmc_per_wave.py "$(find gpurun_out/pmc_$name -name '*counter_collection.csv' | head -1)" k_rollout | tee -a gpurun_out/r05_sq_env_mix.txt
}
rm -f gpurun_out/r05_sq_env_mix.txt
pass sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES &&
pass sqb SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 &&
pass sqc SQ_WAVES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_BRANCH || exit 1
timeout -k 10 600 python bench.py --policy hover --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/r05_hover.log 2>&1 \
  || { tail -5 gpurun_out/r05_hover.log; exit 1; }
tail -1 gpurun_out/r05_hover.log > gpurun_out/r05_bench_hover.json; cut -c1-200 gpurun_out/r05_bench_hover.json
