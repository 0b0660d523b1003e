set -o pipefail
mkdir -p gpurun_out
for v in noenv_stamps; do
  echo "== $v"
  MSACL_HIP_LIB=$PWD/exp_libs/fused-$v/libmsacl_hip.so timeout -k 10 120 python tools/probes/fused_stamps.py 2> gpurun_out/stamps_$v.err | tee gpurun_out/stamps_$v.json || { tail -5 gpurun_out/stamps_$v.err; exit 1; }
done
