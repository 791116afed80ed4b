#!/bin/bash
# tracker timing repeated (box noise): three runs of 30 steps
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do timeout -k 10 120 python3 tools/trk_time.py 30 > gpurun_out/trk_time$i.log 2>&1 || exit 1; grep total gpurun_out/trk_time$i.log; done
