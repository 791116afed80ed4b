#!/bin/bash
# route comparison at 256 windows: HIP-event times and rocprofv3 kernel statistics of both routes
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in PHASES MONOLITHIC; do
  for w in 256 32 1; do
    env VIO_BA_$r=1 timeout -k 10 120 python tools/ba_batch_run.py $w 10 >> gpurun_out/route.log 2>&1 || exit 1
  done
done
cat gpurun_out/route.log | grep W=
export VIO_BA_PHASES=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ph -o ph --output-format csv -- python3 tools/ba_batch_run.py 256 10 > gpurun_out/prof_ph.log 2>&1 || exit 1
unset VIO_BA_PHASES
export VIO_BA_MONOLITHIC=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mono -o mono --output-format csv -- python3 tools/ba_batch_run.py 256 10 > gpurun_out/prof_mono.log 2>&1 || exit 1
unset VIO_BA_MONOLITHIC
timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1
echo done
