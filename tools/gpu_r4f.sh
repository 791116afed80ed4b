#!/bin/bash
# round 4 (f, fresh container): route A/B at 1 / 32 / 256 windows, then suite + smoke + bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python3 tools/ba_route_ab.py 1 32 256 > gpurun_out/route_ab_f.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/route_ab_f.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_round.sh r4f
rc=$?; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc_cfg2.sh
