#!/bin/bash
# round-3 measurement pass: PMC HBM traffic of the bench workload (tracker + BA + the small legs), of the
# 256-window phase-route step and of a config-5 LM iteration; the SQ instruction-mix passes; kernel stats
# of a config-5-only run
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_pmc.sh || exit $?
bash tools/gpu_pmc_ba.sh || exit $?
bash tools/gpu_pmc_gba.sh || exit $?
bash tools/gpu_pmc_mix.sh || exit $?
d=gpurun_out/prof_gba
rm -rf $d
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/gba_run.py 3 > $d.log 2>&1
echo "gba stats rc=$?"
