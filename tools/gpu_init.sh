#!/bin/bash
# Monocular-initialisation parity tests, then the phase-route kernel trace at 256 windows.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_init_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_init.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_init.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_phtrace.sh
