#!/bin/bash
# kernel trace of the config-5 global BA (fused steps at the default threshold)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/gbaprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/gbaprof -o gba --output-format csv -- python3 tools/gba_time.py 3 1 > gpurun_out/gba_prof.log 2>&1 || exit 1
echo prof ok
