#!/bin/bash
# kernel trace of config-5 global BA (tools/gba_time.py 3 1), timeline of the Cholesky launches
set -u
tag=${1:-gt}
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 tools/gba_time.py 3 1 > gpurun_out/prof_$tag.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
python3 tools/gba_timeline.py $f 0 40 > gpurun_out/timeline_$tag.log
python3 tools/gba_timeline.py $f 80 40 >> gpurun_out/timeline_$tag.log
python3 tools/gba_chol_span.py $f >> gpurun_out/timeline_$tag.log
cat gpurun_out/timeline_$tag.log
