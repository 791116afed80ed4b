#!/bin/bash
# tracker: GPU parity tests, config-1 stage times, GFTT selection breakdown (debug build)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tracker_gpu.py tests/test_frontend_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_trk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_trk.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python3 tools/trk_time.py 20 > gpurun_out/trk_time.log 2>&1 || exit 1
cat gpurun_out/trk_time.log
VIO360_LIB=tools/probe/libvio360_dbg.so timeout -k 10 120 python3 tools/trk_time.py 2 > gpurun_out/trk_dbg.log 2>&1 || exit 1
grep gftt_select gpurun_out/trk_dbg.log | tail -9
