#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
VIO_BA_PHASES=1 timeout -k 10 200 python3 tools/ba_streams_run.py 256 10 1,2,4,8 > gpurun_out/streams.log 2>&1 || exit 1
VIO_BA_MONOLITHIC=1 timeout -k 10 200 python3 tools/ba_streams_run.py 256 10 1,2 >> gpurun_out/streams.log 2>&1 || exit 1
grep W= gpurun_out/streams.log
