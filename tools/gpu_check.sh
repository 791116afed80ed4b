#!/bin/bash
# One GPU session: parity tests, phase diagnostics, bench, rocprof kernel-trace summary.
# Stops at the first crash / timeout (exit codes other than 0/1 from pytest).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ba_quick.py > gpurun_out/ba_quick.log 2>&1
rc=$?; echo "ba_quick rc=$rc"; tail -12 gpurun_out/ba_quick.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/rocprof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/rocprof_bench.log
exit $rc
