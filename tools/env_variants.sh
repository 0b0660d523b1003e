#!/bin/bash
# A/B of env-step kernel build variants (e.g. occupancy floors): build variant libraries into
# exp_libs/<name> (`tools/env_variants.sh` here, VARIANTS="name:-DFLAG ..."), then on the GPU box
# (`tools/env_variants.sh run`) time env_step + rollout_step at E = 4,194,304 / 65,536 with each.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS="$ROOT/multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd/csrc"
VARIANTS=${VARIANTS:-"base:"}
if [ "$1" != "run" ]; then
  for vv in $VARIANTS; do
    v=${vv%%:*}; def=${vv#*:}; def=${def//,/ }
    out="$ROOT/exp_libs/$v"; mkdir -p "$out"
    ( cd "$CS" && for f in rollout capi msacl_kernels per gae policy_mlp mlp_grad optim dist_kernels gemm; do
        /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
          -I"$ROOT/include" -I. $def -c $f.hip -o "$out/$f.o" & done; wait
      /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/libmsacl_hip.so" "$out"/*.o )
    echo "built $v ($def)"
  done
  exit 0
fi
mkdir -p "$ROOT/gpurun_out"
for rep in 1 2; do
for vv in $VARIANTS; do
  v=${vv%%:*}
  MSACL_HIP_LIB="$ROOT/exp_libs/$v/libmsacl_hip.so" timeout -k 10 120 python "$ROOT/tools/kernel_bench.py" \
    --envs ${ENVS:-SingleTrackCar,TwoLink} --sizes ${SIZES:-4194304} --skip gather,msacl,gae,policy --reps 20 \
    > "$ROOT/gpurun_out/envv_$v.log" 2>&1
  echo "== $v"; grep -E '"(env_step|rollout_step)"' "$ROOT/gpurun_out/envv_$v.log" | cut -c1-150
done
done
