#!/bin/bash
# A/B of libvio360 builds on one box: phase-route batch timing at 1 / 32 / 256 windows per library
set -u
mkdir -p gpurun_out
export VIO_BA_PHASES=1
for rep in 1 2; do
for lib in "$@"; do
  for W in 1 32 256; do
    echo "$(basename $lib) $(VIO360_LIB=$lib timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 | tail -1)" || exit 1
  done
done
done
