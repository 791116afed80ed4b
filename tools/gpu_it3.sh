#!/bin/bash
# BA phase route after a kernel change: BA GPU tests, per-kernel stats at 1 / 32 / 256 windows, timings
set -u
mkdir -p gpurun_out
tag=${1:-it3}
timeout -k 10 420 python -u -m pytest tests/test_ba_gpu.py tests/test_gather.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" gpurun_out/pytest_$tag.log | head -8; exit $rc; fi
bash tools/gpu_prof_ba.sh $tag || exit $?
export VIO_BA_PHASES=1
for W in 1 32 256; do timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 || exit $?; done
