#!/bin/bash
# round 4 (h): reduced-solve probes (chol6 / chol_mw / chol_tile), then route A/B with the default reduced
# solve and with VIO_BA_CHOL=2 (chol_tile_solve2), BA GPU tests with VIO_BA_CHOL=2
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/cholmw_probe > gpurun_out/cholmw_h.log 2>&1; cat gpurun_out/cholmw_h.log
timeout -k 10 200 python3 tools/ba_route_ab.py 1 8 32 256 > gpurun_out/route_ab_h0.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_h0.log; [ $rc -eq 0 ] || exit $rc
VIO_BA_CHOL=2 timeout -k 10 200 python3 tools/ba_route_ab.py 1 8 32 256 > gpurun_out/route_ab_h2.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_h2.log; [ $rc -eq 0 ] || exit $rc
VIO_BA_CHOL=2 timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_cluster_1h.log 2>&1 || { cat gpurun_out/stamps_cluster_1h.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_cluster_1h.log
VIO_BA_CHOL=2 timeout -k 10 600 python -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ba_h.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error|assert" gpurun_out/pytest_ba_h.log | head -10; exit $rc; }
