#!/bin/bash
# ph_solve shader-clock breakdown at 1 / 256 windows and the multi-stream split of a 256-window shard
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/ph_solve_stamps.py 1 > gpurun_out/stamps.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/ph_solve_stamps.py 256 >> gpurun_out/stamps.log 2>&1 || exit 1
cat gpurun_out/stamps.log
VIO_BA_PHASES=1 timeout -k 10 200 python3 tools/ba_streams_run.py 256 10 1,2,4 > gpurun_out/streams.log 2>&1 || exit 1
grep W= gpurun_out/streams.log
