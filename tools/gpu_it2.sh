#!/bin/bash
set -u
mkdir -p gpurun_out
bash tools/gpu_iter.sh it2 || exit $?
bash tools/gpu_gs.sh
