#!/bin/bash
# One gpurun session of same-box A/B runs: a GPU test subset of the working tree (TESTS, space-separated files;
# empty: none), then tools/ab_<kind>.sh with the remaining arguments.  Logs: gpurun_out/<tag>_tests.log,
# gpurun_out/<tag>_ab.log.
# Usage: TESTS="tests/test_ba_gpu.py" tools/gpu_ab.sh <tag> ba <lib>...         (window-BA builds, WINDOWS / ROUNDS)
#        TESTS="tests/test_tracker_gpu.py" AB_VAR=X AB_VALS="0 1" tools/gpu_ab.sh <tag> trk   (tracker env toggle)
set -o pipefail
tag=$1 kind=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread $TESTS > gpurun_out/${tag}_tests.log 2>&1 \
    || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests.log
fi
ROUNDS=${ROUNDS:-3} bash tools/ab_$kind.sh $tag "$@" > gpurun_out/${tag}_ab.log 2>&1 || { echo "ab failed"; cat gpurun_out/${tag}_ab.log; exit 1; }
cat gpurun_out/${tag}_ab.log
