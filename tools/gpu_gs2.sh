#!/bin/bash
# Schur-side assembly: BA GPU tests, then the Schur group-size sweep by batch size and ph_* stamps
set -u
mkdir -p gpurun_out
tag=${1:-gs2}
timeout -k 10 420 python -u -m pytest tests/test_ba_gpu.py tests/test_gather.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" gpurun_out/pytest_$tag.log | head -8; exit $rc; fi
export VIO_BA_PHASES=1
for cfg in "1 1" "1 2" "1 3" "1 5" "32 1" "32 2" "32 3" "32 5" "256 5" "256 10"; do
  set -- $cfg
  echo "gs=$2 $(VIO_BA_SCHUR_GS=$2 timeout -k 10 120 python3 tools/ba_batch_run.py $1 20 | tail -1)"
done
timeout -k 10 120 python -u tools/ph_solve_stamps.py 1 > gpurun_out/stamps_$tag.log 2>&1 && cat gpurun_out/stamps_$tag.log
