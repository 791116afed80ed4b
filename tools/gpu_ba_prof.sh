#!/bin/bash
# BA parity tests, then per-kernel times of a 256-window batch (phase kernels) under rocprofv3.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ba.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ba -o ba --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-global --no-klt > gpurun_out/bench_ba.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/bench_ba.log | cut -c1-400
exit $rc
