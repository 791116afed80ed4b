#!/bin/bash
# same-box A/B of library builds: W-window config-3 shard, S solves each, alternating builds twice
# usage: bash tools/gpu_ab_libs.sh W S lib...
set -u
export TMPDIR=/tmp
W=$1; S=$2; shift 2
for rep in 1 2; do
  for lib in "$@"; do
    echo "$(basename $lib) $(VIO360_LIB=$lib timeout -k 10 120 python3 tools/ba_batch_run.py $W $S 2>&1 | grep -v amdgpu.ids | tail -1)" || exit 1
  done
done
