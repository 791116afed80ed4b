#!/bin/bash
# round-6 tracker session 3: tracker / front-end GPU suites, same-box A/B of the HEAD build (tools/probe/libvio360_base.so)
# against the working tree's library, LK stamps of the working tree (tools/probe/libvio360_dbg.so)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_tracker_gpu.py \
  tests/test_frontend_gpu.py > gpurun_out/r6e_trk_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6e_trk_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6e_trk_tests.log | tail -2
ROUNDS=3 AB_VAR=VIO360_LIB AB_VALS="tools/probe/libvio360_base.so 360_visual_inertial_odometry_amd/libvio360.so" \
  bash tools/ab_trk.sh lib > gpurun_out/r6e_ab_lib.log 2>&1 || { echo "ab failed"; cat gpurun_out/r6e_ab_lib.log; exit 1; }
cat gpurun_out/r6e_ab_lib.log
VIO360_LIB=tools/probe/libvio360_dbg.so timeout -k 10 120 python3 tools/trk_time.py 1 > gpurun_out/r6e_lk_stamps.log 2>&1 || { tail -20 gpurun_out/r6e_lk_stamps.log; exit 1; }
grep -E "^lk pt" gpurun_out/r6e_lk_stamps.log | tail -6
