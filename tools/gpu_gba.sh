#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q -k "global" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gba.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gba.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python3 tools/gba_time.py 5 > gpurun_out/gba_time.log 2>&1 || exit 1
VIO_GBA_NO_CU_SPLIT=1 timeout -k 10 200 python3 tools/gba_time.py 5 >> gpurun_out/gba_time.log 2>&1 || exit 1
grep gba gpurun_out/gba_time.log
