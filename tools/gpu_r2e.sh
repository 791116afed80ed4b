#!/bin/bash
# Route A/B at the config-4 shard size, then the PMC traffic and instruction-mix passes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in VIO_BA_PHASES VIO_BA_MONOLITHIC; do
  env $r=1 timeout -k 10 120 python3 tools/ba_batch_run.py 256 10 >> gpurun_out/route_ab.log 2>&1 || exit 1
done
cat gpurun_out/route_ab.log
bash tools/gpu_pmc.sh && bash tools/gpu_pmc_mix.sh
