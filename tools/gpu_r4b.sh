#!/bin/bash
# round 4 (b): per-phase stamps of the cluster route and the phase route at one window, per-kernel stats
# of the phase route at 1 / 256 windows for HEAD, the plain-access A/B build and the round-4 base build.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_cluster_1.log 2>&1 || { cat gpurun_out/stamps_cluster_1.log; exit 1; }
cat gpurun_out/stamps_cluster_1.log | grep -v amdgpu.ids
VIO_BA_PHASES=1 timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_phases_1.log 2>&1 || exit 1
cat gpurun_out/stamps_phases_1.log | grep -v amdgpu.ids
for W in 1 256; do
  bash tools/gpu_ab_stats.sh $W 360_visual_inertial_odometry_amd/libvio360.so ab/lib_plainx.so ab/lib_r4base.so || exit 1
done
