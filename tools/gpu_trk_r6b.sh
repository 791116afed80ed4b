#!/bin/bash
# round-6 tracker session 2: GPU tracker / front-end suites; A/B of the presort hand-off (device counter vs stream
# join), of the side stream's host enqueue position, and of the HEAD build against the working tree; stamps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_tracker_gpu.py \
  tests/test_frontend_gpu.py > gpurun_out/r6c_trk_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6c_trk_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6c_trk_tests.log | tail -2
TIMELINE=0 ROUNDS=3 AB_VAR=VIO_TRK_PRESEL_FLAG AB_VALS="0 1" bash tools/ab_trk.sh flag > gpurun_out/r6c_ab_flag.log 2>&1 || { echo "ab failed"; cat gpurun_out/r6c_ab_flag.log; exit 1; }
cat gpurun_out/r6c_ab_flag.log
TIMELINE=0 ROUNDS=2 AB_VAR=VIO_TRK_SIDE AB_VALS="0 1" bash tools/ab_trk.sh side > gpurun_out/r6c_ab_side.log 2>&1 || { echo "ab failed"; cat gpurun_out/r6c_ab_side.log; exit 1; }
cat gpurun_out/r6c_ab_side.log
ROUNDS=3 AB_VAR=VIO360_LIB AB_VALS="tools/probe/libvio360_base.so 360_visual_inertial_odometry_amd/libvio360.so" \
  bash tools/ab_trk.sh lib > gpurun_out/r6c_ab_lib.log 2>&1 || { echo "ab failed"; cat gpurun_out/r6c_ab_lib.log; exit 1; }
cat gpurun_out/r6c_ab_lib.log
VIO360_LIB=tools/probe/libvio360_dbg.so timeout -k 10 120 python3 tools/trk_time.py 3 > gpurun_out/r6c_trk_stamps.log 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/r6c_trk_stamps.log; exit 1; }
grep -E "ransac_|gftt_select" gpurun_out/r6c_trk_stamps.log | tail -6
