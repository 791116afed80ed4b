#!/bin/bash
# round 4: Cholesky probe, route A/B (phases vs cluster; default vs lane-per-row reduced solve), then the
# full GPU suite + smoke + bench (tools/gpu_round.sh).  Logs under gpurun_out/.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/cholmw_probe > gpurun_out/cholmw.log 2>&1; cat gpurun_out/cholmw.log
timeout -k 10 240 python3 tools/ba_route_ab.py 1 32 256 > gpurun_out/route_ab.log 2>&1
rc=$?; cat gpurun_out/route_ab.log; [ $rc -eq 0 ] || exit $rc
VIO_BA_CHOL=1 timeout -k 10 240 python3 tools/ba_route_ab.py 1 32 256 > gpurun_out/route_ab_mw.log 2>&1
rc=$?; cat gpurun_out/route_ab_mw.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh ${1:-r4a}
rc=$?; [ $rc -eq 0 ] || exit $rc
# global BA: the 76.8 KB Cholesky LDS layout (two fused-step workgroups per CU) against HEAD
for rep in 1 2; do
  for lib in 360_visual_inertial_odometry_amd/libvio360.so ab/lib_lds768.so; do
    echo "$(basename $lib) $(VIO360_LIB=$lib timeout -k 10 200 python3 tools/gba_time.py 5 3 2>&1 | grep -v amdgpu.ids | tail -1)" || exit 1
  done
done
