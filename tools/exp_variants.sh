#!/bin/bash
# Cost attribution of k_rollout<QuadTracking>: build variant libraries with parts compiled out
# (MH_EXP_* macros; results are NOT physically valid) into exp_libs/, then (on the GPU box,
# `tools/exp_variants.sh run`) time rollout_step at E = 65,536 with each.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS="$ROOT/multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd/csrc"
VARIANTS=${VARIANTS:-"base NO_POLAR NO_DESIRED NO_SAMPLE NO_SUBSTEPS"}
if [ "$1" != "run" ]; then
  for v in $VARIANTS; do
    out="$ROOT/exp_libs/$v"; mkdir -p "$out"
    def=""; [ "$v" != "base" ] && def="-DMH_EXP_$v"
    ( cd "$CS" && for f in rollout capi msacl_kernels per gae policy_mlp mlp_grad optim dist_kernels gemm; do
        /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
          -I"$ROOT/include" -I. $def ${EXTRA_FLAGS} -c $f.hip -o "$out/$f.o" & done; wait
      /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/libmsacl_hip.so" "$out"/*.o )
    echo "built $v"
  done
  exit 0
fi
mkdir -p "$ROOT/gpurun_out"
for v in $VARIANTS; do
  MSACL_HIP_LIB="$ROOT/exp_libs/$v/libmsacl_hip.so" timeout -k 10 120 python "$ROOT/tools/kernel_bench.py" \
    --envs QuadTracking --skip env_step,gather,msacl,gae --reps 50 > "$ROOT/gpurun_out/exp_$v.log" 2>&1
  echo "$v $(grep rollout_step "$ROOT/gpurun_out/exp_$v.log")"
done
