#!/bin/bash
# round 4 (k): stamps at one window, full GPU suite + smoke + bench (tile reduced solve by default)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps_cluster_1k.log 2>&1 || { cat gpurun_out/stamps_cluster_1k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps_cluster_1k.log
bash tools/gpu_round.sh r4k
