#!/bin/bash
# Cost attribution of k_sample_fused: compile csrc/sample_fused.hip with experiment flags and link
# each variant with the main build's other objects into exp_libs/fused-<name>/libmsacl_hip.so
# (build here, on the CPU; tools/fused_ab.py times them on the GPU box through MSACL_HIP_LIB).
# Usage: tools/fused_variants.sh "name=-DFLAG%-DFLAG2 name2=..."
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
SRC="$ROOT/multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd/csrc"
for v in $1; do
  name=${v%%=*}; flags="$(echo ${v#*=} | tr % ' ')"
  out="$ROOT/exp_libs/fused-$name"; mkdir -p "$out"
  ( /opt/rocm/bin/hipcc -fno-slp-vectorize -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
      -Wno-unused-function -I"$ROOT/include" -I"$SRC" $flags -c "$SRC/sample_fused.hip" -o "$out/sample_fused.o" &&
    objs=$(ls "$SRC"/build/*.o | grep -v sample_fused.o) &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/libmsacl_hip.so" "$out/sample_fused.o" $objs &&
    rm -f "$out/sample_fused.o" && echo "built $out" ) &
done
for j in $(jobs -p); do wait $j || { echo "variant build failed"; exit 1; }; done
