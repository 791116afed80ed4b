#!/bin/bash
# Schur split-k group size A/B (VIO_BA_SCHUR_GS), phase route, over window counts
set -u
export TMPDIR=/tmp VIO_BA_PHASES=1
for W in "$@"; do
  for gs in 2 3 4 5 10; do
    echo "GS=$gs $(VIO_BA_SCHUR_GS=$gs timeout -k 10 120 python3 tools/ba_batch_run.py $W 30 2>&1 | grep -v amdgpu.ids | tail -1)" || exit 1
  done
done
