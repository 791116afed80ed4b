#!/bin/bash
# BA parity tests + phase diagnostics (ba_quick).  Stops at the first crash / timeout.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_ba.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ba_quick.py > gpurun_out/ba_quick.log 2>&1
rc=$?; echo "ba_quick rc=$rc"; cat gpurun_out/ba_quick.log
exit $rc
