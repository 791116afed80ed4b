#!/bin/bash
# round 4 (c): Cholesky probe (ds_ LDS accesses), per-phase stamps (cluster / phases at one window),
# route A/B at 1 / 32 / 256 windows, then the BA GPU tests.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/cholmw_probe > gpurun_out/cholmw_c.log 2>&1; cat gpurun_out/cholmw_c.log
timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_cluster_1c.log 2>&1 || { cat gpurun_out/stamps_cluster_1c.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_cluster_1c.log
VIO_BA_PHASES=1 timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_phases_1c.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamps_phases_1c.log
timeout -k 10 240 python3 tools/ba_route_ab.py 1 32 256 > gpurun_out/route_ab_c.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_c.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ba_c.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/pytest_ba_c.log | head -10; exit $rc; }
