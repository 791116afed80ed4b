#!/bin/bash
# round 4 (m): compressed linearisation (r + Jacobian scale per observation): BA GPU tests, route A/B at
# 1 / 32 / 256 windows, phase-route kernel stats at 256 windows
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_m.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ba_m.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/pytest_ba_m.log | head -10; exit $rc; }
timeout -k 10 200 python3 tools/ba_route_ab.py 1 32 256 > gpurun_out/route_ab_m.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_m.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_stats.sh 256 360_visual_inertial_odometry_amd/libvio360.so
