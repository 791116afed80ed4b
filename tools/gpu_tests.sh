#!/bin/bash
# GPU parity suite only (per-test thread timeouts); log under gpurun_out/
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|PASSED|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -25
exit $rc
