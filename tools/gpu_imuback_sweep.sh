#!/bin/bash
# phase route: the IMU candidate terms at the end of ph_solve (default above VIO_BA_IMU_BACK_MAX windows) or in
# ph_back_x's extra workgroup beside the walk, at 32 / 64 / 256 windows
set -u
export VIO_BA_PHASES=1
for W in 32 64 256; do
  for M in 0 1000; do
    VIO_BA_IMU_BACK_MAX=$M timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 > gpurun_out/imuback_${M}_$W.log 2>&1 || { echo fail; tail -3 gpurun_out/imuback_${M}_$W.log; exit 1; }
    echo "imu_back_max=$M $(tail -1 gpurun_out/imuback_${M}_$W.log)"
  done
done
