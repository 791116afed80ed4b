#!/bin/bash
# IMU candidate terms: ph_solve (default above 64 windows) against ph_back_x's extra workgroup
# (VIO_BA_IMU_BACK_MAX=1000) at 256 / 32 windows, alternating, same box
set -u
for rep in 1 2; do
  for W in 256 32; do
    echo "solve $(timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 2>&1 | tail -1)" || exit 1
    echo "backx $(VIO_BA_IMU_BACK_MAX=1000 timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 2>&1 | tail -1)" || exit 1
  done
done
