#!/bin/bash
# Kernel trace of the phase route at the config-4 shard size (256 windows x 10 LM iterations).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_ph256
VIO_BA_PHASES=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ph256 -o ph --output-format csv -- python3 tools/ba_batch_run.py 256 10 > gpurun_out/ph256.log 2>&1
rc=$?; echo "rc=$rc"; tail -2 gpurun_out/ph256.log; exit $rc
