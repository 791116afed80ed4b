#!/bin/bash
# round 4 (g): per-phase stamps at one window (cluster / phases), route A/B at 1..32 windows
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_cluster_1g.log 2>&1 || { cat gpurun_out/stamps_cluster_1g.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_cluster_1g.log
VIO_BA_PHASES=1 timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_phases_1g.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamps_phases_1g.log
timeout -k 10 300 python3 tools/ba_route_ab.py 1 2 4 8 16 32 > gpurun_out/route_ab_g.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_g.log; exit $rc
