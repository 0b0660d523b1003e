cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ut
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ut -o ut --output-format csv -- python3 tools/update_trace.py > gpurun_out/ut.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -20 gpurun_out/ut.log; exit $rc; }
f=$(find gpurun_out/ut -name '*kernel_trace.csv' | head -1)
python3 tools/update_trace.py --analyse "$f" > gpurun_out/ut_analysis.txt
head -3 gpurun_out/ut_analysis.txt
