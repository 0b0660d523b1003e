#!/bin/bash
# env_step timing of SingleTrackCar (and TwoLink) at 4,194,304 envs with the main library and each
# exp_libs/<name> variant given in $VARIANTS, two passes: gpurun_out/carv.jsonl
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/gpurun_out"
: > "$ROOT/gpurun_out/carv.jsonl"
for rep in 1 2; do
  for v in base $VARIANTS; do
    lib="$ROOT/exp_libs/$v/libmsacl_hip.so"; [ $v = base ] && lib=""
    MSACL_HIP_LIB=${lib:-$ROOT/lib/libmsacl_hip.so} \
      timeout -k 10 120 python "$ROOT/tools/kernel_bench.py" --envs ${ENVS:-SingleTrackCar} --sizes ${SIZES:-4194304} \
      --skip gather,msacl,gae,policy,rollout --reps 20 > "$ROOT/gpurun_out/carv_run.log" 2>&1 || { tail -20 "$ROOT/gpurun_out/carv_run.log"; exit 1; }
    grep '"env_step"' "$ROOT/gpurun_out/carv_run.log" | sed "s/^{/{\"variant\": \"$v\", /" | tee -a "$ROOT/gpurun_out/carv.jsonl" | cut -c1-200
  done
done
