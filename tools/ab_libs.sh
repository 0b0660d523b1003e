#!/bin/bash
# A/B of the engine library against a git revision: `tools/ab_libs.sh build REV` compiles
# csrc/ at REV into exp_libs/REV-<sha>/ and the working tree into exp_libs/work/;
# `tools/ab_libs.sh run ARGS...` (GPU box) times tools/kernel_bench.py ARGS (AB_TOOL=fused_ab.py:
# the fused horizon kernel) with each library, alternating twice (AB_ROUNDS), into
# gpurun_out/ab_<lib>_<i>.log.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=multi-step-actor-critic-learning-with-lyapunov-certificates-for-exponentially-stabilizing-control_amd
SRCS="rollout sample_fused capi msacl_kernels per gae policy_mlp mlp_grad optim dist_kernels gemm mlp_fused"
build_dir() {  # $1 = csrc dir, $2 = include dir, $3 = out dir
  mkdir -p "$3"
  ( cd "$1" && for f in $SRCS; do
      [ -f $f.hip ] || continue
      x="-fno-slp-vectorize"  # as the Makefile (every unit since round 6)
      /opt/rocm/bin/hipcc $x -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
        -I"$2" -I. ${EXTRA_FLAGS} -c $f.hip -o "$3/$f.o" & done; wait
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$3/libmsacl_hip.so" "$3"/*.o )
}
if [ "$1" = "build" ]; then
  rev=${2:-HEAD}; sha=$(git -C "$ROOT" rev-parse --short "$rev")
  tmp=$(mktemp -d); git -C "$ROOT" archive "$rev" "$PKG/csrc" include | tar -x -C "$tmp"
  rm -rf "$ROOT"/exp_libs/rev-* "$ROOT"/exp_libs/work*
  build_dir "$tmp/$PKG/csrc" "$tmp/include" "$ROOT/exp_libs/rev-$sha"
  build_dir "$ROOT/$PKG/csrc" "$ROOT/include" "$ROOT/exp_libs/work"
  for v in $VARIANTS; do  # extra working-tree variants: VARIANTS="NAME=-DFLAG ..."
    EXTRA_FLAGS="$(echo ${v#*=} | tr % " ")" build_dir "$ROOT/$PKG/csrc" "$ROOT/include" "$ROOT/exp_libs/work-${v%%=*}"
  done
  rm -rf "$tmp"; echo "built rev-$sha and work"; exit 0
fi
shift
mkdir -p "$ROOT/gpurun_out"
for i in $(seq 1 ${AB_ROUNDS:-2}); do
  for d in "$ROOT"/exp_libs/rev-* "$ROOT"/exp_libs/work*; do
    n=$(basename "$d")
    MSACL_HIP_LIB_AB=1 MSACL_HIP_LIB="$d/libmsacl_hip.so" timeout -k 10 120 python "$ROOT/tools/${AB_TOOL:-kernel_bench.py}" "$@" \
      > "$ROOT/gpurun_out/ab_${n}_$i.log" 2>&1 || { tail -5 "$ROOT/gpurun_out/ab_${n}_$i.log"; exit 1; }
    echo "== $n ($i)"; grep -E '"avg_us"|"us_per_horizon"' "$ROOT/gpurun_out/ab_${n}_$i.log" | cut -c1-200
  done
done
