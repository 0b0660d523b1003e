set -o pipefail
for cfg in "" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=8"; do
  env $cfg timeout -k 10 150 python3 tools/graph_launch_probe.py > gpurun_out/glp.log 2>&1 || { tail -5 gpurun_out/glp.log; exit 1; }
  tail -1 gpurun_out/glp.log | tee -a gpurun_out/glp_all.txt
done
