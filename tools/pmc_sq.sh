#!/bin/bash
# SQ instruction/stall counters for the env-step kernels at 4M envs (separate PMC pass).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc_sq
timeout -k 10 900 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  -d gpurun_out/pmc_sq -o sq --output-format csv -- python3 tools/kernel_bench.py --sizes ${SIZES:-4194304} --skip rollout,gather,msacl --reps 3 > gpurun_out/pmc_sq.log 2>&1
echo "pmc sq rc=$?"
