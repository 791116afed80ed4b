#!/bin/bash
# round 4 (o): suite + smoke + bench, then the rocprofv3 kernel statistics of a short bench run
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_round.sh r4o || exit 1
rm -rf gpurun_out/prof_bench_r4o
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_r4o -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_bench_r4o.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
