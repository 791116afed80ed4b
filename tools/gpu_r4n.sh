#!/bin/bash
# round 4 (n): PMC HBM traffic of the 256-window step, config-2 solve traffic, then suite + smoke + bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_pmc_ba.sh || exit 1
bash tools/gpu_pmc_cfg2.sh || exit 1
bash tools/gpu_round.sh r4n
