#!/bin/bash
# round 4 (d): latency constants of the pivot chain, stamps at one window (cluster / phases), route A/B
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/lat_probe > gpurun_out/lat.log 2>&1; cat gpurun_out/lat.log
timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_cluster_1d.log 2>&1 || { cat gpurun_out/stamps_cluster_1d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_cluster_1d.log
timeout -k 10 240 python3 tools/ba_route_ab.py 1 32 > gpurun_out/route_ab_d.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_d.log; exit $rc
