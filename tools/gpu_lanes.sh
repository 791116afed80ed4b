#!/bin/bash
# phase-route sub-batch lanes (VIO_BA_LANES) and small-batch IMU placement (VIO_BA_IMU_BACK_MAX):
# BA GPU tests, then timings at 1 / 32 / 256 windows
set -u
mkdir -p gpurun_out
tag=${1:-lanes}
timeout -k 10 420 python -u -m pytest tests/test_ba_gpu.py tests/test_gather.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" gpurun_out/pytest_$tag.log | head -8; exit $rc; fi
export VIO_BA_PHASES=1
for L in 1 2 3 4; do echo "lanes=$L $(VIO_BA_LANES=$L timeout -k 10 120 python3 tools/ba_batch_run.py 256 20 | tail -1)"; done
for L in 1 2; do echo "lanes=$L $(VIO_BA_LANES=$L timeout -k 10 120 python3 tools/ba_batch_run.py 32 20 | tail -1)"; done
for M in 0 8; do echo "imu_back_max=$M $(VIO_BA_IMU_BACK_MAX=$M timeout -k 10 120 python3 tools/ba_batch_run.py 1 20 | tail -1)"; done
