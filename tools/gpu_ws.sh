#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ba_quick.py > gpurun_out/ba_quick.log 2>&1 || exit 1
grep -E "windows=|cfg3" gpurun_out/ba_quick.log
VIO_BA_SCHUR_GS=10 timeout -k 10 200 python3 tools/ba_quick.py > gpurun_out/ba_quick_gs10.log 2>&1 || exit 1
echo "gs=10 (ws)"; grep -E "windows=256" gpurun_out/ba_quick_gs10.log
timeout -k 10 400 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ba.log
exit $rc
