#!/bin/bash
# round-6 tracker session 3: tracker / front-end GPU suites, then same-box A/B runs of the working tree
# (AB_VAR / AB_VALS, default the presort window) with the last value's timeline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_tracker_gpu.py \
  tests/test_frontend_gpu.py > gpurun_out/r6e_trk_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6e_trk_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6e_trk_tests.log | tail -2
ROUNDS=3 AB_VAR=${AB_VAR:-VIO_TRK_PRESORT_WIN} AB_VALS=${AB_VALS:-"0 1"} bash tools/ab_trk.sh e > gpurun_out/r6e_ab.log 2>&1 || { echo "ab failed"; cat gpurun_out/r6e_ab.log; exit 1; }
cat gpurun_out/r6e_ab.log
