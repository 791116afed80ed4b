#!/bin/bash
# Schur group size sweep (VIO_BA_SCHUR_GS) at the 256-window shard
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 10 20 7; do
  VIO_BA_SCHUR_GS=$g timeout -k 10 200 python3 tools/ba_quick.py > gpurun_out/ba_quick_gs$g.log 2>&1 || exit 1
  echo "gs=$g"; grep -E "windows=256" gpurun_out/ba_quick_gs$g.log
done
