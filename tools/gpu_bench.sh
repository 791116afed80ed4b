#!/bin/bash
# bench.py (default run, CPU baselines included) + the rocprofv3 kernel-trace summary of the same
# command (without the CPU legs); logs under gpurun_out/.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
rm -rf gpurun_out/prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/rocprof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -c 300 gpurun_out/rocprof_bench.log
exit $rc
