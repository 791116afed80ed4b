#!/bin/bash
# iteration loop: GPU parity suite (or a -k subset), isolated per-workload phase-kernel stats,
# ph_* shader-clock stamps at 1 / 32 windows
set -u
mkdir -p gpurun_out
tag=${1:-it}; sel=${2:-}
if [ -n "$sel" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$sel" > gpurun_out/pytest_$tag.log 2>&1
else
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$tag.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" gpurun_out/pytest_$tag.log | head -8; exit $rc; fi
bash tools/gpu_prof_ba.sh $tag || exit $?
for W in 1 32; do timeout -k 10 120 python -u tools/ph_solve_stamps.py $W > gpurun_out/stamps_${tag}_$W.log 2>&1 || exit $?; done
cat gpurun_out/stamps_${tag}_1.log
