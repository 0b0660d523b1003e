#!/bin/bash
# Build the engine library with extra compile flags into exp_libs/<name>/libmsacl_hip.so (A/B runs
# load it through MSACL_HIP_LIB). Usage: tools/build_variant.sh <name> "<flags>"
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
SRC="$ROOT/multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd/csrc"
OUT="$ROOT/exp_libs/$1"
mkdir -p "$OUT/obj"
for f in rollout sample_fused capi msacl_kernels per gae policy_mlp mlp_grad optim dist_kernels gemm mlp_fused; do
  extra=""; [ "$f" = sample_fused ] && extra="-fno-slp-vectorize"  # as the Makefile
  /opt/rocm/bin/hipcc $extra -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -Wno-unused-function \
    -I"$ROOT/include" -I"$SRC" $2 -c "$SRC/$f.hip" -o "$OUT/obj/$f.o" &
done
for j in $(jobs -p); do wait $j || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$OUT/libmsacl_hip.so" "$OUT"/obj/*.o
rm -rf "$OUT/obj"
echo "built $OUT/libmsacl_hip.so"
