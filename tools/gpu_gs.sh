#!/bin/bash
# Schur group size sweep (VIO_BA_SCHUR_GS) by batch size: W windows x 10 fixed LM iterations
set -u
mkdir -p gpurun_out
export VIO_BA_PHASES=1
for cfg in "1 1" "1 2" "1 3" "1 5" "32 1" "32 2" "32 3" "32 5" "256 5" "256 10"; do
  set -- $cfg
  VIO_BA_SCHUR_GS=$2 timeout -k 10 120 python3 tools/ba_batch_run.py $1 20 > gpurun_out/gs_$1_$2.log 2>&1 || exit 1
  echo "gs=$2 $(tail -1 gpurun_out/gs_$1_$2.log)"
done
