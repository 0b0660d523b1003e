#!/bin/bash
# SQ counters of the update's fused MLP kernels standalone (tools/mlp3_bench.py, two shapes),
# separate PMC passes (no trace domains)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f gpurun_out/r05_mlp_pmc.txt
pass() {
  local name=$1; shift
  rm -rf gpurun_out/pmc_mlp_$name
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_mlp_$name -o sq --output-format csv -- python3 tools/mlp3_bench.py \
    --reps 5 --cases "10240,12,256,1,1;5120,16,1,1,2" > gpurun_out/pmc_mlp_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || return $rc
  python3 tools/pmc_per_wave.py "$(find gpurun_out/pmc_mlp_$name -name '*counter_collection.csv' | head -1)" k_mlp3 | tee -a gpurun_out/r05_mlp_pmc.txt
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES &&
pass b SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU &&
pass c SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_CYCLES
