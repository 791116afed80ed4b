#!/bin/bash
# ph_prep timing (kernel statistics at 256 windows) and the phase-route stamps on the same box
set -u
tag=${1:-x}
mkdir -p gpurun_out/prep_$tag
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prep_$tag/ks -o run --output-format csv -- python3 tools/ba_batch_run.py 256 5 > gpurun_out/prep_$tag/ks.log 2>&1 || exit 1
grep -h "ph_prep\|ph_back_kernel" gpurun_out/prep_$tag/ks/run_kernel_stats.csv | cut -d, -f1-6
VIO_BA_PHASES=1 timeout -k 10 120 python3 tools/ph_solve_stamps.py 256 > gpurun_out/prep_$tag/stamps.log 2>&1 || exit 1
grep -E "prep|ctrl" gpurun_out/prep_$tag/stamps.log
