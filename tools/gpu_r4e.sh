#!/bin/bash
# round 4 (e): Cholesky probe, stamps (cluster / phases, one window), route A/B, BA GPU tests
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/cholmw_probe > gpurun_out/cholmw_e.log 2>&1; head -2 gpurun_out/cholmw_e.log
timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_cluster_1e.log 2>&1 || { cat gpurun_out/stamps_cluster_1e.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_cluster_1e.log
VIO_BA_PHASES=1 timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_phases_1e.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamps_phases_1e.log | grep -E "solve|prep"
timeout -k 10 240 python3 tools/ba_route_ab.py 1 32 256 > gpurun_out/route_ab_e.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_e.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ba_e.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/pytest_ba_e.log | head -10; exit $rc; }
