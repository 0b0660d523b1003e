#!/bin/bash
# Variants of one csrc source file: compile it with extra flags and link it with the main build's
# other objects into exp_libs/<src>-<name>/libmsacl_hip.so (load with MSACL_HIP_LIB=...).
# Usage: tools/src_variants.sh mlp_fused "pf6=-DMH_MLP_PF=6 pft4=-DMH_MLP_PFT=4%-DX"
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
SRC="$ROOT/multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd/csrc"
base=$1
extra=""; [ "$base" = sample_fused ] && extra="-fno-slp-vectorize"
for v in $2; do
  name=${v%%=*}; flags="$(echo ${v#*=} | tr % ' ')"
  out="$ROOT/exp_libs/$base-$name"; mkdir -p "$out"
  ( /opt/rocm/bin/hipcc $extra -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
      -Wno-unused-function -I"$ROOT/include" -I"$SRC" $flags -c "$SRC/$base.hip" -o "$out/$base.o" &&
    objs=$(ls "$SRC"/build/*.o | grep -v "/$base.o") &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$out/libmsacl_hip.so" "$out/$base.o" $objs &&
    rm -f "$out/$base.o" && echo "built $out" ) &
done
for j in $(jobs -p); do wait $j || { echo "variant build failed"; exit 1; }; done
