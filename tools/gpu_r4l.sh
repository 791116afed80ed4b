#!/bin/bash
# round 4 (l): stamps at one window, route A/B at 1 / 16 windows, BA GPU tests
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_cluster_1l.log 2>&1 || { cat gpurun_out/stamps_cluster_1l.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_cluster_1l.log
timeout -k 10 200 python3 tools/ba_route_ab.py 1 16 > gpurun_out/route_ab_l.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_l.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ba_l.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/pytest_ba_l.log | head -10; exit $rc; }
