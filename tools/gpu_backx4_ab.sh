#!/bin/bash
# phase route A/B: IMU candidate terms in ph_solve (default above 64 windows) / in ph_back_x's extra workgroup /
# in ph_back_x4's (the same at 4 waves per SIMD), at 32 / 64 / 256 windows
set -u
export VIO_BA_PHASES=1
for W in 32 64 256; do
  for V in solve x x4; do
    case $V in
      solve) E="VIO_BA_IMU_BACK_MAX=0";;
      x) E="VIO_BA_IMU_BACK_MAX=1000";;
      x4) E="VIO_BA_IMU_BACK_MAX=1000 VIO_BA_BACKX4=1";;
    esac
    env $E timeout -k 10 120 python3 tools/ba_batch_run.py $W 20 > gpurun_out/bx4_${V}_$W.log 2>&1 || { echo fail; tail -3 gpurun_out/bx4_${V}_$W.log; exit 1; }
    echo "$V $(tail -1 gpurun_out/bx4_${V}_$W.log)"
  done
done
