#!/bin/bash
set -u
bash tools/gpu_trk7.sh trk10 || exit $?
bash tools/gpu_pmc_gba.sh || exit $?
bash tools/gpu_pmc_mix.sh || exit $?
d=gpurun_out/prof_gba
rm -rf $d
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 tools/gba_run.py 3 > $d.log 2>&1
echo "gba stats rc=$?"
