#!/bin/bash
# kernel trace of the config-1 tracker pipeline (tools/trk_time.py) and the timeline of its last run
set -u
tag=${1:-tl}
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$tag -o run --output-format csv -- python3 tools/trk_time.py 20 > gpurun_out/trk_$tag.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
python3 tools/trk_timeline.py $f > gpurun_out/timeline_trk_$tag.log
cat gpurun_out/timeline_trk_$tag.log
rm -rf gpurun_out/prof_$tag
