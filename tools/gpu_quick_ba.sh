#!/bin/bash
# quick window-BA check of a build: timings at 1 / 32 / 256 windows (default route), the cluster route's
# shader-clock stamps at one window, then the BA GPU tests
set -u
tag=${1:-x}
out=gpurun_out/quick_$tag
mkdir -p $out
for W in 1 32 256; do
  timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 > $out/w$W.log 2>&1 || { echo "w$W failed"; tail -5 $out/w$W.log; exit 1; }
  tail -1 $out/w$W.log
done
timeout -k 10 120 python3 tools/ph_solve_stamps.py 1 > $out/stamps1.log 2>&1 || { echo stamps failed; tail -5 $out/stamps1.log; exit 1; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $out/pytest_ba.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_ba.log
  exit $rc
fi
