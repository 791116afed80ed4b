#!/bin/bash
# window GPU test + BA iteration timings after the occupancy bounds
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_window_gpu.py tests/test_init_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_win.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_win.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_ba_iter.sh
